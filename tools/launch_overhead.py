"""Host cost of one batched C-ABI call (ctypes -> multibody_rnea_batch_f32 -> hipModuleLaunchKernel)
against the device time of back-to-back launches, at a small batch where the two compete.

usage: python tools/launch_overhead.py [B]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import torch  # noqa: E402

from rigidbody_amd import ffi  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
mb = ffi.Multibody.new()
x = [torch.rand((7, B), device="cuda") for _ in range(3)]
out = torch.empty_like(x[0])
lib = ffi.lib()
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
args = (mb.handle, x[0].data_ptr(), x[1].data_ptr(), x[2].data_ptr(), out.data_ptr(), B, B, sp)
for rep in range(3):
    lib.multibody_rnea_batch_f32(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(2000):
        lib.multibody_rnea_batch_f32(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B} host us/launch {(t1 - t0) / 2000 * 1e6:.2f}  wall us/launch {(t2 - t0) / 2000 * 1e6:.2f}", flush=True)
