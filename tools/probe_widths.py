"""Pattern ceiling of the batched dynamics' HBM stream by per-lane access width: the no-math
probe (probe.hip: 21 rows read, 7 written, tiled, non-temporal) at the byte totals of the FR3
kernels -- fp32 2^20 (117 MB) and fp64 2^20 (235 MB: 2^21 floats per row) -- with 4, 8 and
16 B per lane.  Event pair around back-to-back launches over rotated buffers (> Infinity Cache).

usage: python tools/probe_widths.py [launches]
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
from rigidbody_amd import ffi  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_lib  # noqa: E402

plib = probe_lib.lib()


def run(B, width, launches):
    per = 28 * B * 4
    nsets = max(2, -(-(5 << 28) // per))
    bufs = [(torch.rand((21 * B,), device="cuda"), torch.empty((7 * B,), device="cuda")) for _ in range(nsets)]
    lib = ffi.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    code = width + 16 * 7  # NT loads + NT stores + tiled

    def go(k):
        i, o = bufs[k % nsets]
        if plib.rb_probe_rows_f32(i.data_ptr(), o.data_ptr(), 21, 7, B, B, code, sp):
            raise RuntimeError(ffi.last_error())

    for k in range(20):
        go(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(launches):
        go(k)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / launches * 1e3
    del bufs
    torch.cuda.empty_cache()
    return {"us": round(us, 2), "TBps": round(per / us / 1e6, 3)}


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    res = {}
    for name, B in (("fp32_2^20", 1 << 20), ("fp64_2^20", 1 << 21)):
        for w in (1, 2, 4):
            r = run(B, w, launches)
            res[f"{name}_w{4 * w}B"] = r
            print(name, f"{4 * w} B/lane", r, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
