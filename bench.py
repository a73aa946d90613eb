#!/usr/bin/env python3
"""Benchmark: batched RNEA (fr3 7-DOF) evals/s on MI355X, BASELINE.json's metric.

One step = one launch of the RNEA kernel over one batch of B configurations
(default B = 2^20 per GPU, fp32, SoA, inputs already resident in HBM).  The input
sets rotate through >1 GiB of device memory so the 256 MiB Infinity Cache cannot
serve them.  N > 1: one process per GPU (torch.distributed.run), the model is loaded
on rank 0 and broadcast as a blob over RCCL, every rank evaluates its own batch
(weak scaling, no data-path collective), timing is max over ranks.

Prints ONE JSON line (rank 0).  See DESIGN.md §5 for how roofline/cpu_baseline are
derived; profiles/ holds the rocprofv3 summaries these numbers are checked against.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "rigidbody-rs_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from rigidbody_amd import chains, ffi  # noqa: E402
from rigidbody_amd import dist as rdist  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (/opt/skills/guides/MI355X_MICROARCH.md)
DT = {"f32": torch.float32, "f64": torch.float64}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000,
                    help="timed steps (~90 ms at the headline): long enough to average over the clock / "
                         "power phases a sustained load goes through (a 1000-step window lands either in a "
                         "~20.3 or a ~25 us phase on some boxes; tools/drift.py, DESIGN.md §8)")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1 << 20, help="configurations per GPU per step")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--kernel", choices=["rnea", "fd", "rnea_fd"], default="rnea",
                    help="rnea_fd = SURVEY §8(d) config 4: each step runs RNEA then forward dynamics on "
                         "its torques (q, qd, qdd -> tau -> qdd'), 8·N·s bytes per configuration")
    ap.add_argument("--dof", type=int, default=7, help="7 = FR3; other values = synthetic z-chain")
    ap.add_argument("--layout", choices=["tiled", "soa"], default="tiled",
                    help="device array layout: tiled [B/256][n][256] (rigidbody_batch.h *_tiled entry points, "
                         "the headline) or plain SoA rows [n][B] (reported as a secondary line)")
    ap.add_argument("--rotate-gib", type=float, default=1.25, help="device memory the input sets span")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU work budget of the baseline sample")
    ap.add_argument("--no-secondary", action="store_true", help="skip the fp64 / forward-dynamics side lines")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the timed batches rotate over (1 = strictly serial launches, the "
                         "headline; the overlapped 2-stream rate is reported under 'secondary')")
    ap.add_argument("--sync-every", type=int, default=0,
                    help="host-synchronize every N timed steps (0 = never; the sync time stays inside the "
                         "timed region)")
    ap.add_argument("--spinup-ms", type=float, default=300.0,
                    help="untimed launches before the warmup so the GPU clock reaches steady state")
    return ap.parse_args()


def init_dist():
    """One process per GPU (torch.distributed.run).  Backend "nccl" = RCCL over xGMI;
    RB_DIST_BACKEND=gloo rehearses the multi-process path with several ranks sharing
    one GPU (ranks map to devices round-robin)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local % ndev)
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("RB_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def load_model(world, rank, dof):
    """Rank 0 parses the URDF; the packed fp64 model blob is broadcast over RCCL
    (rigidbody_amd.dist.broadcast_model)."""
    def make():
        return ffi.Multibody.new() if dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof))

    mb = rdist.broadcast_model(make, rank, world, torch.device("cuda"))
    mb.upload()
    return mb


def make_sets(mb, B, dtype, kernel, nsets, seed, pad=0, layout="soa"):
    """nsets independent (inputs, outputs) sets on the device.  rnea / rnea_fd read
    (q, qd, qdd); fd reads (q, qd, tau).  rnea_fd has two outputs (tau, qdd').
    pad > 0: rows are ld = B + pad elements apart ([n, ld] buffers used as [n, B] views).
    layout "tiled": [ceil(B/256), n, 256] tensors (rigidbody_batch.h), filled with the
    same values as the SoA sets (device fill, then rb_to_tiled)."""
    if layout == "tiled":
        # pad > 0 (tiled): array k of a set starts k * pad elements into its own buffer --
        # staggers the arrays' base addresses (channel-aliasing experiments, tools/ab_bench.py)
        def placed(t, k):
            tt = ffi.to_tiled(t)
            if not pad:
                return tt
            buf = torch.empty(k * pad + tt.numel(), dtype=tt.dtype, device=tt.device)
            v = buf[k * pad:].view(tt.shape)
            v.copy_(tt)
            return v

        sets = []
        for ins, outs in make_sets(mb, B, dtype, kernel, nsets, seed):
            sets.append(([placed(t, k) for k, t in enumerate(ins)],
                         [placed(t, len(ins) + k) for k, t in enumerate(outs)]))
            del ins, outs
        torch.cuda.synchronize()
        return sets
    ld = B + pad
    lim = mb.limits()
    kinds = ("q", "qd", "tau") if kernel == "fd" else ("q", "qd", "qdd")
    nout = 2 if kernel == "rnea_fd" else 1
    sets = []
    for s in range(nsets):
        ins = []
        for k, kind in enumerate(kinds):
            lo, hi = chains.input_ranges(lim, kind)
            t = torch.empty((mb.n, ld), dtype=dtype, device="cuda")[:, :B]
            ffi.fill_uniform(t, lo, hi, seed + 1000 * s + k)
            ins.append(t)
        outs = [torch.empty((mb.n, ld), dtype=dtype, device="cuda")[:, :B] for _ in range(nout)]
        sets.append((ins, outs))
    torch.cuda.synchronize()
    return sets


def set_bytes(n, B, esize, kernel):
    return (8 if kernel == "rnea_fd" else 4) * n * B * esize


def time_launches(launch, steps, warmup, world, spinup_ms=0.0, streams=1, sync_every=0):
    """launch(i, stream_ptr) issues step i.  Warmup, then exactly `steps` launches
    bracketed by barrier + synchronize and one hipEvent pair on the launch stream (no
    per-launch events inside the timed region: an event record between launches on one
    stream inflates a ~22 us step to ~32 us).  With streams > 1 consecutive steps rotate
    over that many streams (independent batches overlap the previous launch's ramp and
    tail); the event pair then spans all of them.  Returns (wall s, device ms per step)."""
    main = torch.cuda.current_stream()
    strs = [main] + [torch.cuda.Stream() for _ in range(streams - 1)]
    sps = [ctypes.c_void_p(st.cuda_stream) for st in strs]
    # spin-up: the clock ramps over the first tens of ms of load
    t_spin = time.perf_counter()
    i = 0
    while (time.perf_counter() - t_spin) * 1e3 < spinup_ms:
        launch(i, sps[i % streams])
        i += 1
        if i % 64 == 0:
            torch.cuda.synchronize()
    for i in range(warmup):
        launch(i, sps[i % streams])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event() for _ in strs]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(main)
    for st in strs[1:]:
        st.wait_event(e0)
    for i in range(steps):
        launch(i, sps[i % streams])
        if sync_every and (i + 1) % sync_every == 0 and i + 1 < steps:
            torch.cuda.synchronize()  # host waits for the queue to drain (inside the timed region)
    for st, end in zip(strs[1:], ends[1:]):
        end.record(st)
        main.wait_event(end)
    e1.record(main)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        torch.distributed.barrier()
    return t1 - t0, e0.elapsed_time(e1) / steps


def time_graph(launch, steps, per_graph=100, spinup_ms=100.0):
    """The same launches replayed from a HIP graph: `per_graph` consecutive launches (rotating
    input sets) are stream-captured once (torch.cuda.graph), then the graph is replayed
    steps / per_graph times between one hipEvent pair -- the host issues one graph launch per
    `per_graph` steps instead of one C-ABI call per step, which is what a short kernel (a
    65536-configuration batch runs ~4 us) needs.  Returns (wall s, device ms per step)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # JIT compile + warm outside the capture
        sp = ctypes.c_void_p(side.cuda_stream)
        for i in range(per_graph):
            launch(i, sp)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for i in range(per_graph):
            launch(i, sp)
    torch.cuda.synchronize()
    t_spin = time.perf_counter()
    while (time.perf_counter() - t_spin) * 1e3 < spinup_ms:
        g.replay()
        torch.cuda.synchronize()
    reps = max(1, steps // per_graph)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    del g
    return t1 - t0, e0.elapsed_time(e1) / (reps * per_graph)


def batch_launcher(mb, sets, kernel, dtype, layout="soa", B=None):
    """Closure issuing the batched entry point(s) of `kernel` on input set i % len(sets)."""
    lib = ffi.lib()
    suffix = "f32" if dtype == torch.float32 else "f64"
    ns = len(sets)
    if layout == "tiled":
        rnea_t = getattr(lib, f"multibody_rnea_batch_tiled_{suffix}")
        fd_t = getattr(lib, f"multibody_fd_batch_tiled_{suffix}")
        calls = []
        for i, o in sets:
            p = [t.data_ptr() for t in i] + [t.data_ptr() for t in o]
            if kernel == "rnea_fd":
                calls.append(((rnea_t, (mb.handle, p[0], p[1], p[2], p[3], B)),
                              (fd_t, (mb.handle, p[0], p[1], p[3], p[4], B))))
            else:
                calls.append(((rnea_t if kernel == "rnea" else fd_t, (mb.handle, p[0], p[1], p[2], p[3], B)),))

        def launch_t(i, sp):
            for fn, a in calls[i % ns]:
                if fn(*a, sp):
                    raise RuntimeError(ffi.last_error())

        return launch_t
    rnea = getattr(lib, f"multibody_rnea_batch_{suffix}")
    fd = getattr(lib, f"multibody_fd_batch_{suffix}")
    B = sets[0][1][0].shape[1]
    ld = sets[0][1][0].stride(0) if sets[0][1][0].shape[0] > 1 else B
    if kernel == "rnea_fd":
        args = [((mb.handle, i[0].data_ptr(), i[1].data_ptr(), i[2].data_ptr(), o[0].data_ptr(), B, ld),
                 (mb.handle, i[0].data_ptr(), i[1].data_ptr(), o[0].data_ptr(), o[1].data_ptr(), B, ld))
                for i, o in sets]

        def launch(i, sp):
            a1, a2 = args[i % ns]
            if rnea(*a1, sp) or fd(*a2, sp):
                raise RuntimeError(ffi.last_error())
    else:
        fn = rnea if kernel == "rnea" else fd
        args = [(mb.handle, i[0].data_ptr(), i[1].data_ptr(), i[2].data_ptr(), o[0].data_ptr(), B, ld)
                for i, o in sets]

        def launch(i, sp):
            if fn(*args[i % ns], sp):
                raise RuntimeError(ffi.last_error())

    return launch


def rollout_launcher(mb, B, dtype, K, dt=1e-3, seed=chains.SEED):
    """Closure issuing multibody_rollout_batch_* on one resident state (q, qd updated in
    place by every launch) and a [K*n, B] torque sequence."""
    n = mb.n
    q = torch.empty((n, B), dtype=dtype, device="cuda")
    qd = torch.empty_like(q)
    lim = mb.limits()
    ffi.fill_uniform(q, *chains.input_ranges(lim, "q"), seed)
    ffi.fill_uniform(qd, *chains.input_ranges(lim, "qd"), seed + 1)
    tau = torch.empty((K * n, B), dtype=dtype, device="cuda")
    lo, hi = chains.input_ranges(lim, "tau")
    ffi.fill_uniform(tau, lo * K, hi * K, seed + 2)
    fn = getattr(ffi.lib(), f"multibody_rollout_batch_{'f32' if dtype == torch.float32 else 'f64'}")
    args = (mb.handle, q.data_ptr(), qd.data_ptr(), tau.data_ptr(), dt, K, None, B, B)

    def launch(i, sp):
        rc = fn(*args, sp)
        if rc:
            raise RuntimeError(ffi.last_error())

    launch.keep = (q, qd, tau)
    return launch


def run_timed(mb, sets, kernel, dtype, steps, warmup, world, spinup_ms=0.0, streams=1, layout="soa", B=None,
              sync_every=0):
    return time_launches(batch_launcher(mb, sets, kernel, dtype, layout, B), steps, warmup, world, spinup_ms, streams,
                         sync_every)


def side_workloads(mb7, a, rotate_gib):
    """Secondary measurements (one GPU, serial launches): the other SURVEY §8(d) configs."""
    sec = {}
    steps = max(20, a.steps // 4)

    def one(name, mb, kernel, dt_name, B=a.batch, graph=False):
        ds = DT[dt_name]
        es = 4 if dt_name == "f32" else 8
        per = set_bytes(mb.n, B, es, kernel)
        sets = make_sets(mb, B, ds, kernel, max(2, int(np.ceil(rotate_gib * (1 << 30) / per))), chains.SEED + 31,
                         layout=a.layout)
        w, km = run_timed(mb, sets, kernel, ds, steps, 5, 1, 300.0, 1, a.layout, B)
        sec[name] = {"evals_per_s": B * steps / w, "kernel_ms_avg": km, "batch": B, "layout": a.layout,
                     "hbm_frac": per / (km * 1e-3) / HBM_PEAK,
                     "kernel_path": "+".join(mb.kernel_path(k, dt_name == "f64") for k in kernel.split("_"))}
        if graph:  # the same launches replayed from a HIP graph
            gw, gkm = time_graph(batch_launcher(mb, sets, kernel, ds, a.layout, B), steps)
            sec[name + "_graph"] = {"evals_per_s": B * steps / gw, "kernel_ms_avg": gkm, "batch": B,
                                    "layout": a.layout, "hbm_frac": per / (gkm * 1e-3) / HBM_PEAK,
                                    "launch": "HIP graph of 100 captured C-ABI launches, replayed"}
        del sets
        torch.cuda.empty_cache()

    one("rnea_fr3_f32_b65536", mb7, "rnea", "f32", 65536, graph=True)    # config 2
    one("fd_fr3_f32_b65536", mb7, "fd", "f32", 65536, graph=True)        # config 3
    one("rnea_fr3_f64", mb7, "rnea", "f64")
    one("fd_fr3_f32", mb7, "fd", "f32")
    one("fd_fr3_f64", mb7, "fd", "f64")
    one("rnea_fd_fr3_f64_b131072", mb7, "rnea_fd", "f64", 1 << 17, graph=True)  # config 4, one GPU's 2^17 shard
    mb30 = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30))
    mb30.upload()
    one("rnea_chain30_f32", mb30, "rnea", "f32")             # config 5
    # a floating-base branching tree (6 virtual + 8 joints, 2 prismatic)
    mbt = ffi.Multibody.from_urdf_string(chains.tree_urdf(floating=True), ffi.FLOATING_BASE)
    mbt.upload()
    one("rnea_float14_tree_f32", mbt, "rnea", "f32")
    one("fd_float14_tree_f32", mbt, "fd", "f32")
    # fused rollout: K forward-dynamics + Euler steps per launch
    # (its clock settles only after ~150 ms of this VALU-dense load: 495 -> 357 us per launch)
    K, nl = 16, 40
    w, km = time_launches(rollout_launcher(mb7, a.batch, torch.float32, K), nl, 3, 1, 300.0)
    sec["rollout_fr3_f32_K16"] = {"steps_per_launch": K, "evals_per_s": a.batch * K * nl / w,
                                  "kernel_ms_avg": km, "kernel_path": mb7.kernel_path("rollout", False),
                                  "note": "evals = configurations x Euler steps; q, qd stay on chip (LDS)"}
    return sec


def cpu_baseline(n, B_sample_hint, kernel, cpu_seconds):
    """fp64 CPU restatement (oracle/, kind "port") timed on this host's cores."""
    from oracle import oracle, urdf_model

    oracle.build()
    xml = chains.fr3_urdf_text() if n == 7 else chains.synthetic_chain_urdf(n)
    raw = urdf_model.model_raw_from_urdf(xml)
    om = oracle.Model(raw)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(16, cores))  # the GPU box's CPU share is 16
    mbl = ([l["lower"] for l in raw["limits"]], [l["upper"] for l in raw["limits"]],
           [l["velocity"] for l in raw["limits"]], [l["effort"] for l in raw["limits"]])
    kinds = ("q", "qd", "tau") if kernel == "fd" else ("q", "qd", "qdd")

    def inputs(B):
        return [chains.host_uniform(n, B, *chains.input_ranges(mbl, kind), chains.SEED + k)
                for k, kind in enumerate(kinds)]

    if kernel == "rnea_fd":
        def call(q, qd, qdd, nthreads):
            return om.fd_batch(q, qd, om.rnea_batch(q, qd, qdd, nthreads=nthreads), nthreads=nthreads)
    else:
        call = om.rnea_batch if kernel == "rnea" else om.fd_batch
    cal = inputs(20000)
    t = time.perf_counter()
    call(*cal, nthreads=1)
    rate1 = 20000 / (time.perf_counter() - t)
    sample = int(min(max(rate1 * cpu_seconds, 1e5), 5e7))
    x = inputs(sample)
    t = time.perf_counter()
    call(*x, nthreads=cores)
    dt = time.perf_counter() - t
    return {"value": sample / dt, "unit": "evals/s", "cores": cores, "kind": "port",
            "sample": f"{sample} fr3 configs (same distributions/seed as the GPU run), fp64 oracle "
                      f"{kernel} over {cores} OpenMP threads, {dt:.2f} s wall; single-thread {rate1:.3g} evals/s"}


def load_traffic(workload):
    path = os.path.join(REPO, "profiles", f"traffic_{workload}.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def main():
    a = parse()
    world, rank, local = init_dist()
    n = a.dof
    dtype = DT[a.dtype]
    esize = 4 if a.dtype == "f32" else 8
    mb = load_model(world, rank, n)
    per_set = set_bytes(n, a.batch, esize, a.kernel)
    nsets = max(2, int(np.ceil(a.rotate_gib * (1 << 30) / per_set)))
    sets = make_sets(mb, a.batch, dtype, a.kernel, nsets, rdist.rank_seed(chains.SEED, rank), layout=a.layout)
    wall, kern_avg_ms = run_timed(mb, sets, a.kernel, dtype, a.steps, a.warmup, world, a.spinup_ms, a.streams,
                                  a.layout, a.batch, a.sync_every)
    wall, kern_avg_ms = rdist.max_over_ranks([wall, kern_avg_ms], world, torch.device("cuda"))
    evals = world * a.batch * a.steps
    value = evals / wall
    # q, qd, qdd|tau read + tau|qdd written per kernel; rnea_fd counts both
    bytes_per_eval = set_bytes(n, 1, esize, a.kernel)
    achieved = bytes_per_eval * a.batch / (kern_avg_ms * 1e-3)
    workload = f"{a.kernel}_{'fr3' if n == 7 else f'chain{n}'}_{a.dtype}_{a.layout}_b{a.batch}"
    traffic = load_traffic(workload)
    line = {
        "metric": "RNEA evals/sec (fr3 7-DOF, batch 2^20) at 1/2/4/8 MI355X; % HBM roofline",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (device splitmix64, SURVEY.md §8(d) distributions, seed 20250224)",
        "config": {"workload": workload, "kernel": a.kernel, "model": "fr3 7-DOF" if n == 7 else f"chain{n}",
                   "layout": ("tiled [B/256][n][256] (each 256-configuration tile of all joints contiguous)"
                              if a.layout == "tiled" else "SoA rows [n][B]"),
                   "streams": a.streams,
                   "batch_per_gpu": a.batch, "global_batch": a.batch * world, "dof": n,
                   "parallelism": f"dp{world} (independent shards, RCCL model broadcast)",
                   "input_sets": nsets, "rotated_bytes": nsets * per_set,
                   "kernel_path": "+".join(mb.kernel_path(k, a.dtype == "f64") for k in a.kernel.split("_"))},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK,
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "bytes_per_eval": bytes_per_eval, "evals_per_launch": a.batch, "kernel_ms_avg": kern_avg_ms,
                     "timing": (f"kernel_ms_avg = hipEvent pair on the launch stream around the {a.steps} timed "
                                f"launches / {a.steps} ({a.streams} stream(s); includes the inter-launch gap)")},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(n, a.batch, a.kernel, a.cpu_seconds)
    if rank == 0 and not a.no_secondary and world == 1 and n == 7:
        # the same workload with consecutive batches overlapped on 2 streams
        w2, k2 = run_timed(mb, sets, a.kernel, dtype, a.steps, 5, 1, 50.0, 2, a.layout, a.batch)
        sec = {f"{a.kernel}_{a.dtype}_{a.layout}_2streams": {
            "evals_per_s": a.batch * a.steps / w2, "step_ms_device": k2,
            "hbm_frac_effective": bytes_per_eval * a.batch / (k2 * 1e-3) / HBM_PEAK}}
        del sets
        torch.cuda.empty_cache()
        if a.layout != "soa":  # the same workload on plain SoA rows
            sets = make_sets(mb, a.batch, dtype, a.kernel, nsets, chains.SEED + 7)
            w3, k3 = run_timed(mb, sets, a.kernel, dtype, a.steps, 5, 1, 100.0)
            sec[f"{a.kernel}_{a.dtype}_soa"] = {"evals_per_s": a.batch * a.steps / w3, "kernel_ms_avg": k3,
                                                "hbm_frac": bytes_per_eval * a.batch / (k3 * 1e-3) / HBM_PEAK}
            del sets
            torch.cuda.empty_cache()
        sec.update(side_workloads(mb, a, a.rotate_gib))
        line["secondary"] = sec
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
