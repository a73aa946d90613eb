"""bench.py's multi-rank launch on CPU: `--gpus N` started by hand spawns N ranks itself
(the parent never touches a GPU), every rank joins one process group of size N, and exactly
one JSON line comes back -- the driver's `python bench.py --gpus N` contract.  --stub runs
the same spawning, rank setup, model broadcast, shard split, max-over-ranks reduction and
reporting over gloo with no kernels."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, run_bench


def _strict(_c):
    raise ValueError(f"non-strict JSON constant {_c}")


def _run(*args, env=None):
    """bench.py --stub: (compact stdout line, full detail file) -- conftest.run_bench."""
    return run_bench(["--stub", "--steps", "5", "--warmup", "0", *args], env)


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline")


@pytest.mark.parametrize("split", ["weak", "strong"])
def test_gpus2_spawns_two_ranks(split):
    compact, line = _run("--gpus", "2", "--split", split)
    for k in REQUIRED:
        assert k in compact, k
    assert compact["n_gpus"] == 2 and compact["value"] == line["value"]
    assert len(compact["per_rank"]) == 2 and compact["roofline"]["check"] == "ok"
    if split == "weak":
        assert set(compact["secondary"]) >= {"strong_split", "strong_split_rnea_fd"}
    assert line["n_gpus"] == 2
    assert line["scaling"] == split
    cfg = line["config"]
    if split == "weak":
        assert cfg["global_batch"] == 2 * (1 << 20) and cfg["batch_per_gpu"] == 1 << 20
    else:
        assert cfg["global_batch"] == 1 << 20 and cfg["batch_per_gpu"] == 1 << 19
    assert line["value"] > 0 and line["metric"].startswith("RNEA evals/sec")
    assert line["dtype"] == "f64"  # the reference's Real (lib.rs:15)
    # per-GPU times beside the max over ranks; no CPU baseline at world > 1, said so
    assert [r["rank"] for r in line["per_rank"]] == [0, 1]
    assert all(r["steps"] == 5 and r["wall_s"] > 0 for r in line["per_rank"])
    assert "cpu_baseline" not in line and "world > 1" in line["cpu_baseline_note"]
    if split == "weak":
        # the strong split beside the weak line times its own launch budget, not --steps
        import bench

        st = line["secondary"]["strong_split"]
        assert st["launches"] >= bench.SIDE_MIN_LAUNCHES
        assert len(st["per_rank"]) == 2 and all(r["steps"] == st["launches"] for r in st["per_rank"])
        assert st["global_batch"] == 1 << 20 and st["batch_per_gpu_max"] == 1 << 19
        # SURVEY §8(d) config 4 (fp64 RNEA + FD on shards of one global 2^20 batch) beside it
        c4 = line["secondary"]["strong_split_rnea_fd"]
        assert c4["global_batch"] == bench.CONFIG4_BATCH and c4["batch_per_gpu_max"] == bench.CONFIG4_BATCH // 2
        assert c4["launches"] >= bench.SIDE_MIN_LAUNCHES and len(c4["per_rank"]) == 2
        assert c4["dtype"] == "f64" and c4["scaling"] == "strong" and "config 4" in c4["config"]
    assert line["roofline_check"] == "ok"


def test_single_rank_default():
    compact, line = _run()
    for k in REQUIRED:
        assert k in compact, k
    assert line["n_gpus"] == 1 and line["scaling"] == "weak"
    assert compact["config"]["workload"] == line["config"]["workload"] == "rnea_fr3_f64_tiled_b1048576"
    assert compact["roofline"]["bound"] == "hbm" and compact["roofline"]["unit"] == "GB/s"


def test_compact_line_of_a_full_driver_line():
    """The round-5 driver-style full line (22 KB, the size BENCH_r05 could not parse) through
    bench.compact_line: strict JSON, < 16 KB, every contract key, the headline numbers unchanged,
    a {us, frac} summary per secondary workload; and the same line grown to 8 ranks stays < 16 KB."""
    sys.argv = ["bench.py"]
    bench = pytest.importorskip("bench")
    with open(os.path.join(REPO, "profiles", "r05", "session2", "bench_driver_e.json")) as f:
        full = json.load(f)
    assert len(json.dumps(full)) > 16384
    full["per_rank"] = [{"rank": r, "wall_s": 1e-3, "kernel_ms_avg": 0.04, "steps": 20} for r in range(8)]
    full["secondary"]["bad"] = {"kernel_ms_avg": float("nan"), "hbm_frac": float("inf")}
    out = bench.dumps_strict(bench.compact_line(full))
    assert len(out) < bench.LINE_MAX_BYTES, len(out)
    c = json.loads(out, parse_constant=_strict)
    for k in REQUIRED + ("cpu_baseline",):
        assert k in c, k
    assert c["value"] == full["value"] and c["roofline"]["frac"] == full["roofline"]["frac"]
    assert c["cpu_baseline"]["cores"] == full["cpu_baseline"]["cores"] and c["cpu_baseline"]["kind"] == "port"
    sec = c["secondary"]
    assert sec["rnea_fr3_f32_b65536_graph"]["us"] > 0 and 0 < sec["fd_fr3_f64"]["frac"] <= 1
    assert sec["layout_ab_rnea_f64"]["tiled_us"] > 0 and sec["native_batch"]
    assert sec["bad"] == {} or all(v is None for v in sec["bad"].values())
    for tok in ("NaN", "Infinity"):
        assert tok not in out


def test_failed_rank_fails_the_job():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    # an impossible model size makes every rank raise before the process group forms
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--stub", "--gpus", "2", "--dof", "9999",
                        "--steps", "1"], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_cpu_share_reads_the_cgroup_quota(tmp_path):
    """cpu_baseline's core count comes from the cgroup CPU quota when one is set (v2
    cpu.max, v1 cfs quota/period), capped by the affinity set, else the affinity set."""
    import bench

    vis = bench.host_cores()
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    cores, how = bench.cpu_share(str(tmp_path))
    assert cores == min(16, vis) and "cpu.max" in how
    (tmp_path / "cpu.max").write_text("max 100000\n")
    cores, how = bench.cpu_share(str(tmp_path))
    assert cores == vis and "affinity" in how
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("250000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.cpu_share(str(v1))[0] == min(2, vis)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cpu_share(str(v1))[0] == vis


def test_batch_launcher_owns_its_sets():
    """The launch closures hold raw device pointers; they must keep the tensors those point
    to alive, or a caller that drops its input sets times kernels on freed memory (which a
    HIP-graph capture's empty_cache then unmaps).  CPU tensors stand in for the sets; no
    launch is issued."""
    import gc
    import types
    import weakref

    import torch

    import bench

    sets = [([torch.zeros(7, 8, dtype=torch.float64) for _ in range(3)], [torch.zeros(7, 8, dtype=torch.float64)])]
    ref = weakref.ref(sets[0][0][0])
    launch = bench.batch_launcher(types.SimpleNamespace(handle=None), sets, "rnea", torch.float64, "soa")
    del sets
    gc.collect()
    assert ref() is not None
    del launch
    gc.collect()
    assert ref() is None


@pytest.mark.parametrize("workload,op,clock,dt,packed,ms", [
    ("fd_fr3_f64_tiled_b1048576", "fd_fr3", "fd_fr3_f64", "f64", False, 0.051),
    ("fd_fr3_f32_tiled_b1048576", "fd_fr3", "fd_fr3_f32", "f32", True, 0.0256),
    ("rnea_chain30_f32_tiled_b1048576", "rnea_chain30", "rnea_chain30_f32", "f32", False, 0.1019),
])
def test_valu_roofline_from_committed_counters(workload, op, clock, dt, packed, ms):
    """roofline.valu from the committed PMC summary (profiles/traffic_*.json), the op-counting
    oracle's FLOPs (profiles/r04/op_counts.json) and the clock probe (profiles/r04/
    clock_probe.jsonl) at a kernel time of the measured order: every fraction present and in
    (0, 1], the FLOP counters scaled to lanes (kernel FLOPs per evaluation within 2x of the
    VALU instruction count per evaluation x 2 per FMA)."""
    sys.path.insert(0, REPO)
    sys.argv = ["bench.py"]
    bench = pytest.importorskip("bench")
    v = bench.valu_roofline(workload, op, clock, dt, 1 << 20, ms, packed)
    for k in ("issue_frac_2p4ghz", "issue_frac_held", "flop_frac"):
        assert 0 < v[k] <= 1.0, (k, v[k])
    assert v["held_clock_ghz"] < 2.4 and v["kernel_tflops"] <= v["flop_peak_tflops"]
    per_inst = v["kernel_flops_per_eval"] / v["insts_per_eval"]
    assert 0.5 < per_inst < (4.5 if packed else 2.5), per_inst
    # the reference formulation's operation count lives beside the roofline, not in it
    assert not any(k.startswith("ref") or "flops_per_eval_ref" in k for k in v)
    ref = bench.reference_formulation(op, 1 << 20, ms)
    assert ref["flops_per_eval"] > 1000 and ref["flops_per_eval"] > v["kernel_flops_per_eval"]


def _driver_lines():
    """The committed driver-style bench lines (profiles/r0*/session*/bench_driver*.log)."""
    import glob

    out = []
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r0*", "session*", "bench_driver*.log"))):
        for ln in open(path):
            if ln.startswith("{") and '"metric"' in ln:
                out.append((os.path.relpath(path, REPO), json.loads(ln)))
    return out


def test_roofline_block_consistent():
    """Every *_frac in a bench line is in (0, 1] and no rate under roofline exceeds its peak
    (bench.roofline_violations, which bench.py also writes into each line as roofline_check):
    on synthetic lines that break each rule, and on the committed driver-style lines after the
    reference formulation's rate is moved out of the roofline block as bench.py now does."""
    sys.argv = ["bench.py"]
    bench = pytest.importorskip("bench")
    good = {"roofline": {"achieved": 5000.0, "peak": 8000.0, "frac": 0.625,
                         "valu": {"issue_frac_held": 0.8, "kernel_tflops": 30.0, "flop_peak_tflops": 78.6}},
            "secondary": {"x": {"hbm_frac": 0.5, "valu": {"flop_frac": 0.4}}}}
    assert bench.roofline_violations(good) == []
    for path, val in ((("roofline", "frac"), 1.2), (("roofline", "achieved"), 9000.0),
                      (("roofline", "valu", "kernel_tflops"), 90.0), (("secondary", "x", "hbm_frac"), 0.0)):
        bad = json.loads(json.dumps(good))
        d = bad
        for k in path[:-1]:
            d = d[k]
        d[path[-1]] = val
        assert bench.roofline_violations(bad), path
    lines = _driver_lines()
    assert lines
    for path, line in lines:
        for v in [line.get("roofline", {}).get("valu", {})] + [s.get("valu", {}) for s in
                                                               (line.get("secondary") or {}).values()
                                                               if isinstance(s, dict)]:
            for k in ("ref_equiv_tflops", "flops_per_eval_ref", "ref_source"):
                (v or {}).pop(k, None)
        assert bench.roofline_violations(line) == [], path
