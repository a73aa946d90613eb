"""Per-stage instruction count of the model-specialised mass-matrix forward dynamics (CPU only).

Compiles the hipRTC source the library would build (Multibody.jit_source) with hipcc for gfx950,
once as is and once with RB_STAGE_MARKS=1 (fdh_body.hip.hpp: an assembler comment fenced by
scheduling barriers at each stage boundary), and counts the VALU instructions between the
markers: loads | bias forward sweep (incl. the joint sincos) | bias backward sweep (+ tau loads) |
composite-rigid-body mass matrix | L D L^T | solves + stores.  The joint sincos is counted from a
separate kernel of the same header that evaluates only the N angles.  The marked build must stay
within a few instructions of the product build (printed), else the markers moved code.

usage: python tools/fd_stages.py {f64,f32} [DOF] [--pack P] [--json out.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd"))
from rigidbody_amd import chains, ffi  # noqa: E402

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd", "csrc")
TRANS = re.compile(r"v_(rcp|rsq|sqrt|sin|cos|exp|log)")


def compile_s(src, d, name):
    path = os.path.join(d, name + ".hip")
    open(path, "w").write(src)
    out = os.path.join(d, name + ".s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffinite-math-only",
           "-fno-signed-zeros", "-I", CSRC, "--cuda-device-only", "-S", "-o", out, path]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-4000:])
    return out


def sections(asm_path):
    """VALU / SALU / memory counts per marked section of the kernel body."""
    cur = "loads"
    order = [cur]
    cnt = collections.defaultdict(collections.Counter)
    in_fn = False
    for line in open(asm_path):
        t = line.strip()
        if t.startswith("rb_jit_kernel:") or t.startswith("rb_stage_probe:"):
            in_fn = True
            continue
        if not in_fn:
            continue
        if t.startswith(".Lfunc_end"):
            break
        m = re.match(r";\s*rb_stage (\w+)", t)
        if m:
            cur = m.group(1)
            if cur not in order:
                order.append(cur)
            continue
        tok = t.split()
        if not tok or tok[0].startswith((".", ";")) or tok[0].endswith(":"):
            continue
        op = tok[0]
        if op.startswith("v_"):
            cls = "trans" if TRANS.match(op) else "valu"
            if op.startswith(("v_mov", "v_cndmask", "v_readfirstlane", "v_accvgpr")):
                cnt[cur]["moves"] += 1
        elif op.startswith("s_"):
            cls = "salu"
        elif op.startswith(("global_", "buffer_")):
            cls = "vmem"
        elif op.startswith("ds_"):
            cls = "lds"
        else:
            cls = "other"
        cnt[cur][cls] += 1
    return order, cnt


SINCOS_PROBE = r"""
#include "spatial.hip.hpp"
using T = %(T)s;
extern "C" __global__ __launch_bounds__(256) void rb_stage_probe(const T *__restrict__ q, T *__restrict__ o) {
%(init)s  const uint32_t b = blockIdx.x * 256u + threadIdx.x;
  T acc = T(0);
#pragma unroll
  for (int j = 0; j < %(N)d; ++j) {
    T s, c;
    rbamd::dev::sin_cos<%(fast)s>(rbamd::dev::ld_row(q, j * 65536, b * (uint32_t)sizeof(T)), s, c);
    acc = rbamd::dev::fmadd(s, c, acc);
  }
  rbamd::dev::st_row(o, 0, b * (uint32_t)sizeof(T), acc);
}
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dt", choices=["f64", "f32"])
    ap.add_argument("dof", nargs="?", type=int, default=7)
    ap.add_argument("--pack", type=int, default=None, help="jit pack (fp32: 1 one per lane, 2 pair)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    f64 = a.dt == "f64"
    if a.pack is not None:
        os.environ["RB_PACK"] = str(a.pack)
    mb = ffi.Multibody.new() if a.dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(a.dof))
    if a.pack is not None:
        ffi.set_tuning("pack", a.pack)
    src = mb.jit_source(f64, "fd")
    assert "fdh_body.hip.hpp" in src, "not the mass-matrix form"
    d = f"/tmp/fd_stages_{a.dt}_{a.dof}_p{a.pack}"
    os.makedirs(d, exist_ok=True)
    plain = sections(compile_s(src, d, "plain"))
    marked = sections(compile_s("#define RB_STAGE_MARKS 1\n" + src, d, "marked"))
    total_plain = sum(c["valu"] + c["trans"] for c in plain[1].values())
    order, cnt = marked
    total_marked = sum(c["valu"] + c["trans"] for c in cnt.values())
    paired = "TV{" in src
    fast = "true" if (not f64 and ", true>" in src) else "false"
    probe = SINCOS_PROBE % {"T": "double" if f64 else "float", "N": a.dof, "fast": fast,
                            "init": "  rbamd::dev::sctab_init();\n" if "sctab_init" in src else ""}
    if "RB_SINCOS_TAB 1" in src:
        at = src.index("static __device__ constexpr double rb_sctab_src")
        probe = "#define RB_SINCOS_TAB 1\n" + src[at:src.index("};", at) + 3] + probe
    sc = sections(compile_s(probe, d, "sincos"))[1]
    sincos = sum(c["valu"] + c["trans"] for c in sc.values()) - a.dof  # minus the probe's fma per angle
    rows = []
    for s in order:
        c = cnt[s]
        rows.append({"stage": s, "valu": c["valu"] + c["trans"], "moves": c["moves"], "salu": c["salu"],
                     "vmem": c["vmem"], "lds": c["lds"]})
    res = {"dtype": a.dt, "dof": a.dof, "paired": paired, "valu_plain": total_plain, "valu_marked": total_marked,
           "sincos_all_joints_est": sincos, "stages": rows}
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
