"""HBM ceiling for the batched kernels' SoA access pattern (rb_probe_rows_f32):
rows_in rows read + rows_out rows written per configuration, at 4 B and 16 B per lane,
over rotated buffers (> Infinity Cache), hipEvent timing, median of rounds."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
from rigidbody_amd import ffi  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_lib  # noqa: E402

plib = probe_lib.lib()


def run(rows_in, rows_out, width, nt=0, B=1 << 20, steps=100, rounds=5):
    per = (rows_in + rows_out) * B * 4
    nsets = max(2, int(np.ceil(1.25 * (1 << 30) / per)))
    sets = [(torch.rand((rows_in, B), device="cuda"), torch.empty((max(rows_out, 1), B), device="cuda"))
            for _ in range(nsets)]
    lib = ffi.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = [(i.data_ptr(), o.data_ptr(), rows_in, rows_out, B, B, width + 16 * nt, sp) for i, o in sets]
    for k in range(200):
        assert plib.rb_probe_rows_f32(*args[k % nsets]) == 0, ffi.last_error()
    ms = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(steps):
            plib.rb_probe_rows_f32(*args[k % nsets])
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1) / steps)
    med = float(np.median(ms))
    return {"rows_in": rows_in, "rows_out": rows_out, "width_bytes": 4 * width, "nt": nt, "us": med * 1e3,
            "TBps": (rows_in + rows_out) * B * 4 / (med * 1e-3) / 1e12}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "qkernels":
        # FR3 CRBA / Jacobian / forward-kinematics shapes in fp64 (2^20 configurations = 2^21
        # floats per row, 8 B per lane) and fp32 (2^20 floats, 4 B per lane), SoA, with and
        # without non-temporal stores
        out = [run(7, ro, w, nt, B=B) for ro in (49, 42, 3) for (w, B) in ((2, 1 << 21), (1, 1 << 20))
               for nt in (0, 2, 3)]
    elif len(sys.argv) > 1 and sys.argv[1] == "qtiled":
        # CRBA / Jacobian fp64 shapes: SoA rows vs the tiled layout (nt bit 2), with / without
        # non-temporal stores
        out = [run(7, ro, 2, nt, B=1 << 21) for ro in (49, 42) for nt in (2, 4, 6, 7)]
    elif len(sys.argv) > 1 and sys.argv[1] == "chain30":
        # the 30-DOF RNEA shape (90 rows in / 30 out), SoA and tiled, with / without nt
        out = [run(90, 30, 1, nt, B=1 << 20) for nt in (0, 3, 4, 7)]
    elif len(sys.argv) > 1 and sys.argv[1] == "tiled":
        # SoA rows vs the tiled layout (nt bit 2), 4 B lanes, RNEA 7-DOF shape, three batch sizes
        out = [run(21, 7, 1, nt, B=B) for B in (1 << 20, 1 << 21, 1 << 22) for nt in (0, 3, 4, 7)]
    else:
        out = [run(ri, ro, w, nt) for ri, ro in ((21, 7), (90, 30), (4, 4)) for w in (1, 4) for nt in (0, 1, 2, 3)]
    print(json.dumps(out, indent=1))
