"""Per-node cost of a HIP graph of tiny kernels, to read the model-specialised kernels' launch
floor against: 100 launches of a one-block torch elementwise kernel captured once and replayed,
hipEvent pair; beside it the same for one of our kernels at one block (FR3 fp32 RNEA, B = 256)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rigidbody_amd import chains, ffi  # noqa: E402


def graph_us(launch, per=100, reps=200):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for i in range(per):
            launch(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(per):
            launch(i)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * per)


x = torch.zeros(256, device="cuda")
out = {"torch_fill_256": graph_us(lambda i: x.fill_(float(i))),
       "torch_add_256": graph_us(lambda i: x.add_(1.0))}
mb = ffi.Multibody.new()
mb.upload()
sets = bench.make_sets(mb, 256, torch.float32, "rnea", 4, chains.SEED, "tiled")
ln = bench.batch_launcher(mb, sets, "rnea", torch.float32, "tiled", 256)
out["rnea_f32_b256"] = graph_us(lambda i: ln(i, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
print(json.dumps(out))
