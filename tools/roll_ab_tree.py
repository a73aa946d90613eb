"""Rollout timing of another tree's library (e.g. ab/r04, a `git worktree` of an earlier round
with its library built) on THIS tree's bench workload (bench.rollout_launcher with the per-launch
state reset, so both libraries see the same finite states).  Run once per tree, alternately, on
one box.  usage: python tools/roll_ab_tree.py [--tree DIR] [--dtype f64] [--rounds 3]
                                               [--steps 100] [--tuning key=value ...]"""
import argparse
import importlib.util
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default=REPO)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--tuning", nargs="*", default=[])
    a = ap.parse_args()
    tree = os.path.abspath(a.tree)
    os.environ.setdefault("RB_EXPERIMENTAL", "1")
    sys.path.insert(0, os.path.join(tree, "rigidbody-rs_amd"))
    from rigidbody_amd import ffi  # noqa: F401  (the tree's library, cached for bench's import)

    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert os.path.dirname(os.path.abspath(bench.ffi.__file__)).startswith(tree), bench.ffi.__file__
    for kv in a.tuning:
        k, v = kv.split("=")
        assert bench.ffi.lib().rb_set_tuning(k.encode(), int(v)) == 0, bench.ffi.last_error()
    mb = bench.ffi.Multibody.new()
    mb.upload()
    rl = bench.rollout_launcher(mb, a.batch, bench.DT[a.dtype], 16)
    ms = []
    for r in range(a.rounds):
        _, m = bench.time_launches(rl, a.steps, 5, 1, 300.0 if r == 0 else 0.0)
        ms.append(m * 1e3)
    print(json.dumps({"tree": os.path.relpath(tree, REPO), "dtype": a.dtype, "batch": a.batch,
                      "tuning": a.tuning, "launch_us_rounds": [round(x, 1) for x in ms],
                      "launch_us_min": round(min(ms), 1)}), flush=True)


if __name__ == "__main__":
    main()
