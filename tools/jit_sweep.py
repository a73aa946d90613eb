"""Resource sweep of every model-specialised kernel the library would build (CPU only): for each
model x kind x dtype x launch shape, the hipRTC code object the launch takes (RB_JIT_DUMP) --
VGPRs, AGPRs, scratch bytes, LDS, waves/SIMD -- with scratch flagged.  A kernel that spills runs
several times slower than its neighbours (the round-5 fp64 ABA rollout under a 4-wave target:
436 B of scratch, 4131 vs 984 us), so every shape is listed, not just the bench's.

usage: python tools/jit_sweep.py [--json out.json] [--models fr3 chain12 ...]"""
import argparse
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd"))

KINDS = ("rnea", "fd", "crba", "rollout", "fwd_kin", "jac")
SHAPES = ((65536, False), (1 << 20, False), (1 << 20, True))  # (batch, tiled)


def notes(co):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                         text=True).stdout
    r = {}
    for key, name in ((".vgpr_count", "vgpr"), (".agpr_count", "agpr"), (".sgpr_count", "sgpr"),
                      (".group_segment_fixed_size", "lds"), (".private_segment_fixed_size", "scratch")):
        m = re.search(re.escape(key) + r":\s+(\d+)", out)
        r[name] = int(m.group(1)) if m else None
    return r


def waves(v, a):
    # gfx950: 512 unified registers (VGPRs + AGPRs) per lane per SIMD, in granules of 8, at most 8
    # waves; the code object's .vgpr_count is already the unified total (arch VGPRs + AGPRs)
    del a
    return min(8, 512 // max(((v or 0) + 7) // 8 * 8, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--models", nargs="+", default=["fr3", "chain12", "chain30", "tree9", "floating14"])
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="rb_sweep_")
    os.environ["RB_JIT_DUMP"] = d
    from rigidbody_amd import chains, ffi

    def model(name):
        if name == "fr3":
            return ffi.Multibody.new()
        if name.startswith("chain"):
            return ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(int(name[5:])))
        floating = name.startswith("floating")
        return ffi.Multibody.from_urdf_string(chains.tree_urdf(floating=floating),
                                              ffi.FLOATING_BASE if floating else ffi.URDF_TREE | ffi.GENERAL_AXES)

    rows = []
    for mname in a.models:
        mb = model(mname)
        for kind in KINDS:
            for f64 in (True, False):
                for B, tiled in SHAPES:
                    if tiled and kind == "rollout":
                        continue
                    before = set(glob.glob(os.path.join(d, "*.co")))
                    try:
                        mb.jit_compile(f64, kind=kind, batch=B, tiled=tiled)
                    except Exception as e:  # a shape the library serves with a precompiled kernel
                        rows.append({"model": mname, "kind": kind, "dtype": "f64" if f64 else "f32", "batch": B,
                                     "tiled": tiled, "error": str(e)[:120]})
                        continue
                    new = sorted(set(glob.glob(os.path.join(d, "*.co"))) - before, key=os.path.getmtime)
                    if not new:  # cached: the same kernel as an earlier shape
                        continue
                    r = notes(new[-1])
                    r.update({"model": mname, "kind": kind, "dtype": "f64" if f64 else "f32", "batch": B,
                              "tiled": tiled, "waves_per_simd": waves(r["vgpr"], r["agpr"])})
                    rows.append(r)
                    flag = "  <-- SCRATCH" if r["scratch"] else ""
                    print(f"{mname:11s} {kind:8s} {r['dtype']} B={B:<8d} {'tiled' if tiled else 'soa  '} "
                          f"vgpr {r['vgpr']:3d} agpr {r['agpr'] or 0:3d} lds {r['lds']:6d} scratch {r['scratch']:4d} "
                          f"waves {r['waves_per_simd']}{flag}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    bad = [r for r in rows if r.get("scratch")]
    print(f"{len(rows)} kernels, {len(bad)} with scratch")


if __name__ == "__main__":
    main()
