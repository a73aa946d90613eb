"""In-kernel shader clock of the model-specialised kernels under sustained load (diagnostic
build, measurement only -- never part of the product library).

MI355X_MICROARCH.md 'DVFS give-back': the chip lowers its clock under load, so a VALU floor
priced at 2.4 GHz understates what a VALU-dense kernel can reach.  This tool compiles the
exact hipRTC source the product compiles (multibody_jit_source) plus a stamped twin of its
entry point: each wave records s_memtime (shader cycles) and s_memrealtime (100 MHz) when it
starts and when it has issued its stores (lane 0 writes them with vector stores).  After
>= 2 s of back-to-back launches of the product kernel the twin runs back to back for ~1 s; from
its last launch:

  clock      = median over waves of d(memtime) / d(memrealtime) * 100 MHz
  wave_us    = median wave lifetime
  residency  = sum of wave lifetimes / (1024 SIMDs x waves-per-SIMD limit x in-kernel span)

usage:
  python tools/clock_probe.py build                      # CPU: hipcc --genco the twins
  python tools/clock_probe.py run [--seconds 2] [--batch B] [--only NAME ...]   # GPU: a JSON line per kernel
"""
import argparse
import ctypes
import json
import os
import re
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(REPO, "rigidbody-rs_amd"))
CSRC = os.path.join(REPO, "rigidbody-rs_amd", "csrc")
OUT = os.path.join(HERE, "microbench")

# (name, kind, f64, dof, waves-per-SIMD limit of the product kernel, configurations per lane,
#  the `pack` tuning the source is generated under: -1 = the large-batch form; 1 = one per
#  lane; 4 = the fp32 FD packed wave split, the form launches of <= 2^17 configurations take, capi.cpp jit_fd)
CASES = [
    ("rnea_fr3_f64", "rnea", True, 7, 4, 2, -1),
    ("fd_fr3_f64", "fd", True, 7, 4, 1, -1),
    ("fd_fr3_f32", "fd", False, 7, 4, 2, -1),
    ("fd_fr3_f32_p4", "fd", False, 7, 8, 1, 4),  # small-batch split: waves 0/1 bias, 2/3 mass matrix
    ("rnea_fr3_f32", "rnea", False, 7, 8, 1, -1),
    ("rnea_chain30_f32", "rnea", False, 30, 3, 1, -1),  # parked forces (rnea_lane_park): 3 waves/SIMD
]


def _model(dof):
    from rigidbody_amd import chains, ffi

    return ffi.Multibody.new() if dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof))


def twin_source(src):
    """The product source plus rb_clock_kernel: the same parameters + a stamp buffer, the same
    body between two stamps."""
    m = re.search(r'extern "C" (__global__[^\n]*?) void rb_jit_kernel\(([^)]*)\) \{\n(.*?)\n\}\n', src, re.S)
    if not m:
        raise RuntimeError("rb_jit_kernel entry point not found in the JIT source")
    attrs, params, body = m.group(1), m.group(2), m.group(3)
    body = body.replace("return;", "goto rb_stamp_end;")
    twin = (f'\nextern "C" {attrs} void rb_clock_kernel({params}, unsigned long long *__restrict__ rb_stamps) {{\n'
            "  const unsigned long long rb_t0 = __builtin_amdgcn_s_memtime();\n"
            "  const unsigned long long rb_r0 = __builtin_amdgcn_s_memrealtime();\n"
            "  asm volatile(\"\" ::: \"memory\");\n"
            "  {\n" + body + "\n  }\n"
            "rb_stamp_end:\n"
            "  asm volatile(\"\" ::: \"memory\");\n"
            "  const unsigned long long rb_t1 = __builtin_amdgcn_s_memtime();\n"
            "  const unsigned long long rb_r1 = __builtin_amdgcn_s_memrealtime();\n"
            "  if ((threadIdx.x & 63u) == 0u) {\n"
            "    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;\n"
            "    rb_stamps[4u * w + 0u] = rb_t0; rb_stamps[4u * w + 1u] = rb_t1;\n"
            "    rb_stamps[4u * w + 2u] = rb_r0; rb_stamps[4u * w + 3u] = rb_r1;\n"
            "  }\n}\n")
    return src + twin


def build():
    os.environ.setdefault("RB_EXPERIMENTAL", "1")  # `pack` is an experimental tuning key
    from rigidbody_amd import ffi

    for name, kind, f64, dof, _, _, pack in CASES:
        mb = _model(dof)
        assert ffi.lib().rb_set_tuning(b"pack", pack) == 0, ffi.last_error()
        src = twin_source(mb.jit_source(f64, kind))
        assert ffi.lib().rb_set_tuning(b"pack", -1) == 0
        path = os.path.join(OUT, f"clock_{name}.hip")
        with open(path, "w") as f:
            f.write(src)
        co = os.path.join(OUT, f"clock_{name}.hsaco")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffinite-math-only",
               "-fno-signed-zeros", "-I", CSRC, "--genco", "-o", co, path]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"{name}: {r.stderr[-3000:]}")
        print(f"built {co}")


def _hip():
    import torch  # noqa: F401  (loads the HIP runtime torch uses)

    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1])
    return ctypes.CDLL("libamdhip64.so")


def run(seconds, B, only):
    import numpy as np
    import torch

    from rigidbody_amd import ffi

    hip = _hip()
    dev = torch.device("cuda:0")
    torch.cuda.init()
    for name, kind, f64, dof, wps, per_lane, pack in CASES:
        if only and name not in only:
            continue
        # fp32 FD: the packed pair from 2^17 + 1 configurations, the packed wave split (pack 4)
        # up to 2^17 (capi.cpp jit_fd); a case whose form the product launch would not take is
        # skipped at this batch size
        if kind == "fd" and not f64 and (pack == 4) != (B <= (1 << 17)):
            continue
        co = os.path.join(OUT, f"clock_{name}.hsaco")
        if not os.path.exists(co):
            sys.exit(f"{co} missing: python tools/clock_probe.py build")
        mb = _model(dof)
        mb.upload()
        if pack == 4:  # the split form runs only when selected (tuning pack 4)
            assert ffi.lib().rb_set_tuning(b"pack", 4) == 0, ffi.last_error()
        n = mb.n
        dt = torch.float64 if f64 else torch.float32
        g = torch.Generator(device=dev).manual_seed(7)
        x = [(torch.rand((n, B), generator=g, device=dev, dtype=dt) * 2 - 1) for _ in range(3)]
        out = torch.empty((n, B), device=dev, dtype=dt)

        def product():
            if kind == "rnea":
                mb.rnea_batch(x[0], x[1], x[2], out=out)
            else:
                mb.fd_batch(x[0], x[1], x[2], out=out)

        product()
        torch.cuda.synchronize()
        t = time.time()
        while time.time() - t < seconds:  # sustained load first (DVFS settles)
            for _ in range(200):
                product()
            torch.cuda.synchronize()
        # product kernel time, events around 2000 launches
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2000):
            product()
        e1.record()
        torch.cuda.synchronize()
        product_us = e0.elapsed_time(e1) / 2000 * 1e3

        module, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = open(co, "rb").read()
        assert hip.hipModuleLoadData(ctypes.byref(module), data) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), module, b"rb_clock_kernel") == 0
        grid = (B + 256 * per_lane - 1) // (256 * per_lane)
        waves = grid * 4
        stamps = torch.zeros(4 * waves, device=dev, dtype=torch.int64)
        a = [ctypes.c_void_p(t.data_ptr()) for t in (x[0], x[1], x[2], out)]
        Bc, ld, bs, sp = ctypes.c_uint32(B), ctypes.c_int64(B), ctypes.c_int64(256), ctypes.c_void_p(stamps.data_ptr())
        args = (ctypes.c_void_p * 8)(*[ctypes.cast(ctypes.pointer(v), ctypes.c_void_p) for v in (*a, Bc, ld, bs, sp)])
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

        def twin():
            rc = hip.hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, stream, args, None)
            assert rc == 0, rc

        twin()
        torch.cuda.synchronize()
        e0.record()
        nl = 0
        t = time.time()
        while time.time() - t < max(1.0, seconds / 2):
            for _ in range(200):
                twin()
            nl += 200
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        twin_us = e0.elapsed_time(e1) / nl * 1e3
        s = stamps.view(waves, 4).cpu().numpy().astype(np.float64)
        hip.hipModuleUnload(module)
        cyc, real = s[:, 1] - s[:, 0], s[:, 3] - s[:, 2]
        ok = real > 0
        clk = cyc[ok] / real[ok] * 100e6
        span = (s[:, 3].max() - s[:, 2].min()) / 100e6
        life = real / 100e6
        line = {"kernel": name, "batch": B, "product_kernel_us": round(product_us, 2),
                "stamped_kernel_us": round(twin_us, 2),
                "clock_GHz_median": round(float(np.median(clk)) / 1e9, 3),
                "clock_GHz_p10_p90": [round(float(np.percentile(clk, p)) / 1e9, 3) for p in (10, 90)],
                "wave_us_median": round(float(np.median(life)) * 1e6, 2),
                "wave_cycles_median": int(np.median(cyc)),
                "in_kernel_span_us": round(span * 1e6, 2),
                "residency": round(float(life.sum() / (1024 * wps * span)), 3),
                "waves": waves, "waves_per_simd_limit": wps}
        # where the unoccupied slots are: resident fraction of the 1024 x wps wave slots over
        # 20 equal bins of the in-kernel span, and when the last wave started / the first ended
        t0, t1 = s[:, 2].min(), s[:, 3].max()
        edges = np.linspace(t0, t1, 21)
        lo_, hi_ = np.maximum(s[ok, 2][:, None], edges[None, :-1]), np.minimum(s[ok, 3][:, None], edges[None, 1:])
        occ = np.clip(hi_ - lo_, 0, None).sum(0) / (1024 * wps * (edges[1] - edges[0]))
        line.update({"occupancy_by_twentieth": [round(float(v), 3) for v in occ],
                     "last_start_us": round(float(s[:, 2].max() - t0) / 100, 2),
                     "first_end_us": round(float(s[:, 3].min() - t0) / 100, 2)})
        if pack == 4:  # per role: wave w % 4 in {0, 1} bias torques, {2, 3} mass matrix + solve
            role = np.arange(waves) % 4 >= 2
            t0 = s[:, 2].min()
            for nm, sel in (("bias", ~role), ("mass", role)):
                line[nm] = {"wave_us_median": round(float(np.median(life[sel])) * 1e6, 2),
                            "start_us_median": round(float(np.median(s[sel, 2] - t0)) / 100, 2),
                            "end_us_median": round(float(np.median(s[sel, 3] - t0)) / 100, 2),
                            "end_us_max": round(float(np.max(s[sel, 3] - t0)) / 100, 2)}
            assert ffi.lib().rb_set_tuning(b"pack", -1) == 0
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--only", nargs="*", default=[])
    a = ap.parse_args()
    build() if a.mode == "build" else run(a.seconds, a.batch, a.only)


if __name__ == "__main__":
    main()
