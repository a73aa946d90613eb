"""Offline audit of a model-specialised (hipRTC) kernel: dump its source, compile it with
hipcc for gfx950 with the same options, and report registers / occupancy and an
instruction mix from the ISA.  CPU only (hipcc cross-compiles).

usage: python tools/jit_audit.py KIND {f32,f64} [DOF] [--batch B] [--tiled]
       KIND in rnea fd crba rollout fwd_kin jac; the kernel a launch of B configurations takes
       (default 2^20, SoA), as multibody_jit_source_ex resolves it
"""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd"))
from rigidbody_amd import chains, ffi  # noqa: E402

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd", "csrc")


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("kind")
    ap.add_argument("dt", choices=["f32", "f64"])
    ap.add_argument("dof", type=int, nargs="?", default=7)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--tiled", action="store_true")
    a = ap.parse_args()
    kind, dt, dof = a.kind, a.dt, a.dof
    mb = ffi.Multibody.new() if dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof))
    src = mb.jit_source(dt == "f64", kind, batch=a.batch, tiled=a.tiled)
    d = f"/tmp/jit_audit_{kind}_{dt}_{dof}_{a.batch}{'_t' if a.tiled else ''}"
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "k.hip")
    open(path, "w").write(src)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffinite-math-only",
           "-fno-signed-zeros", "-I", CSRC, "--cuda-device-only", "-S", "-o", os.path.join(d, "k.s"),
           "-Rpass-analysis=kernel-resource-usage", path]
    if kind == "rollout" and "RB_ROLLOUT_NO_HOIST 1" in src:  # as jit.cpp compiles it
        cmd[1:1] = ["-mllvm", "-disable-machine-licm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-4000:])
        sys.exit(1)
    for line in r.stderr.splitlines():
        m = re.search(r"remark: .*?(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize|Occupancy|LDS Size).*?: (\S+)", line)
        if m:
            print(f"  {m.group(1)}: {m.group(2)}")
    mix = collections.Counter()
    for line in open(os.path.join(d, "k.s")):
        t = line.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        cls = op.split("_")[0]
        if cls == "v":
            cls = "v_" + ("trans" if re.match(r"v_(rcp|rsq|sqrt|sin|cos|exp|log)", op) else "alu")
        mix[cls] += 1
        mix[op] += 0
        if op.startswith(("v_fma", "v_mul", "v_add", "v_sub", "v_pk")):
            mix["  " + op] += 1
    print("  mix:", {k: v for k, v in sorted(mix.items()) if v and not k.startswith("  ")})
    print("  top:", sorted(((v, k.strip()) for k, v in mix.items() if k.startswith("  ")), reverse=True)[:10])
    print("  isa:", os.path.join(d, "k.s"))


if __name__ == "__main__":
    main()
