#!/usr/bin/env python3
"""Benchmark: batched RNEA (fr3 7-DOF) evals/s on MI355X, BASELINE.json's metric.

One step = one launch of the RNEA kernel over one batch of B configurations
(default B = 2^20 per GPU, fp64 -- the reference's `Real = f64`, lib.rs:15 -- tiled
[B/256][n][256] layout, inputs already resident in HBM).  The input sets rotate through
>1 GiB of device memory so the 256 MiB Infinity Cache cannot serve them.

Multi-GPU: one process per GPU.  `--gpus N` with N > 1 started by hand spawns N fresh
child ranks itself (this parent never touches the GPU and relays rank 0's JSON line);
under torch.distributed.run the ranks come from the environment.  The model is loaded on
rank 0 and broadcast as a blob over RCCL; each rank evaluates its own 2^20 batch
(`--split weak`, the default) or its contiguous shard of one global 2^20 batch
(`--split strong`, SURVEY §8(e): 2^17 per GPU at N = 8).  No collective touches the data
path; timing is max over ranks.  A weak run also reports the strong split beside it.

Prints ONE JSON line (rank 0).  See DESIGN.md §5 for how roofline/cpu_baseline are
derived; profiles/ holds the rocprofv3 summaries these numbers are checked against.
"""
import argparse
import contextlib
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
METRIC = "RNEA evals/sec (fr3 7-DOF, batch 2^20) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK = 8.0e12  # B/s, MI355X spec (/opt/skills/guides/MI355X_MICROARCH.md)
# VALU roofline: 256 CUs x 4 SIMDs, 2.4 GHz peak engine clock; vector FLOP peaks
# fp32 157.3 TF (MI355X_MICROARCH.md), fp64 78.6 TF (AMD spec: half the fp32 lanes -- the measured
# 4-cycle wave64 v_fma_f64 issue, 16 lanes/clk/SIMD)
SIMDS = 1024
CLOCK_PEAK = 2.4e9
VALU_FLOP_PEAK = {"f32": 157.3e12, "f64": 78.6e12}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 without WORLD_SIZE in the environment spawns N ranks")
    ap.add_argument("--steps", type=int, default=4000,
                    help="timed steps: long enough to average over the clock / power phases a sustained "
                         "load goes through (tools/drift.py, DESIGN.md §5)")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1 << 20,
                    help="configurations per GPU per step (--split weak) or in total (--split strong)")
    ap.add_argument("--split", choices=["weak", "strong"], default="weak",
                    help="weak: every rank evaluates its own --batch; strong: the ranks shard one --batch")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f64",
                    help="f64 = the reference's Real (lib.rs:15), the headline; f32 is a reduced-precision "
                         "variant reported under 'secondary'")
    ap.add_argument("--kernel", choices=["rnea", "fd", "rnea_fd"], default="rnea",
                    help="rnea_fd = SURVEY §8(d) config 4: each step evaluates tau = rnea(q, qd, qdd) and "
                         "qdd' = fd(q, qd, tau_in) (multibody_rnea_fd_batch_*, one fused launch), 6·n·s bytes "
                         "per configuration")
    ap.add_argument("--dof", type=int, default=7, help="7 = FR3; other values = synthetic z-chain")
    ap.add_argument("--layout", choices=["tiled", "soa"], default="tiled",
                    help="device array layout: tiled [B/256][n][256] (rigidbody_batch.h *_tiled entry points, "
                         "the headline) or plain SoA rows [n][B] (reported as a secondary line)")
    ap.add_argument("--rotate-gib", type=float, default=1.25, help="device memory the input sets span")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU work budget of the baseline sample")
    ap.add_argument("--no-secondary", action="store_true", help="skip the side lines")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the timed batches rotate over (1 = strictly serial launches, the "
                         "headline; the overlapped 2-stream rate is reported under 'secondary')")
    ap.add_argument("--sync-every", type=int, default=0,
                    help="host-synchronize every N timed steps (0 = never; inside the timed region)")
    ap.add_argument("--spinup-ms", type=float, default=300.0,
                    help="untimed launches before the warmup so the GPU clock reaches steady state")
    ap.add_argument("--stub", action="store_true",
                    help="CPU rehearsal of the launch / rank / reporting plumbing (gloo, no kernels, "
                         "no GPU); the JSON line says data='stub'")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ rank spawning
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(a, argv):
    """Parent of an N-rank run started as `python bench.py --gpus N`: starts N fresh child
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, the same
    arguments), waits for all, relays rank 0's stdout and returns non-zero if any rank
    failed.  Never imports torch, never touches a GPU."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    base = dict(os.environ, MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port,
                WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus))
    import tempfile

    procs = []
    with tempfile.TemporaryFile() as out0:
        for r in range(a.gpus):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                          stdout=out0 if r == 0 else subprocess.DEVNULL))
        # a rank that fails leaves the others blocked in a collective: stop them (exact PIDs)
        failed = None
        while any(p.poll() is None for p in procs):
            for r, p in enumerate(procs):
                if p.returncode not in (None, 0) and failed is None:
                    failed = r
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
            time.sleep(0.1)
        for p in procs:
            p.wait()
        out0.seek(0)
        # rank 0's JSON line to stdout; anything else it printed (library chatter) to stderr
        for ln in out0.read().decode(errors="replace").splitlines():
            (sys.stdout if ln.startswith("{") else sys.stderr).write(ln + "\n")
        sys.stdout.flush()
    bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0]
    if bad:
        print(f"bench.py: rank(s) failed (rank, exit status): {bad}", file=sys.stderr)
        first = dict(bad).get(failed, bad[0][1]) if failed is not None else bad[0][1]
        return first if 0 < first < 256 else 1
    return 0


if __name__ == "__main__":
    _ARGS = parse()
    if _ARGS.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(_ARGS, sys.argv[1:]))

# ----------------------------------------------------------------- rank process
import numpy as np  # noqa: E402
import torch  # noqa: E402

for _p in (REPO, os.path.join(REPO, "rigidbody-rs_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from rigidbody_amd import chains, ffi  # noqa: E402
from rigidbody_amd import dist as rdist  # noqa: E402

DT = {"f32": torch.float32, "f64": torch.float64}


def init_dist(a):
    """One process per GPU.  Backend "nccl" = RCCL over xGMI; RB_DIST_BACKEND=gloo rehearses
    the multi-process path (ranks then share GPUs round-robin); --stub uses gloo on CPU.
    Returns (world, rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.stub:
        dev = torch.device("cpu")
    else:
        ndev = max(1, torch.cuda.device_count())
        dev = torch.device("cuda", local % ndev)
        torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        backend = "gloo" if a.stub else os.environ.get("RB_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
        world = dist.get_world_size()
    if a.gpus > 1 or world > 1:
        assert world == a.gpus, f"--gpus {a.gpus} but the job has {world} rank(s)"
    return world, rank, dev


def load_model(world, rank, dof, dev):
    """Rank 0 parses the URDF; the packed fp64 model blob is broadcast over RCCL
    (rigidbody_amd.dist.broadcast_model)."""
    def make():
        return ffi.Multibody.new() if dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof))

    mb = rdist.broadcast_model(make, rank, world, dev)
    if dev.type == "cuda":
        mb.upload()
    return mb


def make_sets(mb, B, dtype, kernel, nsets, seed, layout="soa"):
    """nsets independent (inputs, outputs) sets on the device.  rnea reads (q, qd, qdd); fd
    reads (q, qd, tau); rnea_fd reads (q, qd, qdd, tau_in) and has two outputs (tau, qdd').
    layout "tiled": [ceil(B/256), n, 256] tensors (rigidbody_batch.h), filled with the
    same values as the SoA sets (device fill, then rb_to_tiled)."""
    if layout == "tiled":
        sets = []
        for ins, outs in make_sets(mb, B, dtype, kernel, nsets, seed):
            sets.append(([ffi.to_tiled(t) for t in ins], [ffi.to_tiled(t) for t in outs]))
            del ins, outs
        torch.cuda.synchronize()
        return sets
    lim = mb.limits()
    kinds = {"fd": ("q", "qd", "tau"), "rnea_fd": ("q", "qd", "qdd", "tau")}.get(kernel, ("q", "qd", "qdd"))
    nout = 2 if kernel == "rnea_fd" else 1
    sets = []
    for s in range(nsets):
        ins = []
        for k, kind in enumerate(kinds):
            lo, hi = chains.input_ranges(lim, kind)
            t = torch.empty((mb.n, B), dtype=dtype, device="cuda")
            ffi.fill_uniform(t, lo, hi, seed + 1000 * s + k)
            ins.append(t)
        outs = [torch.empty((mb.n, B), dtype=dtype, device="cuda") for _ in range(nout)]
        sets.append((ins, outs))
    torch.cuda.synchronize()
    return sets


def set_bytes(n, B, esize, kernel):
    """Algorithmic HBM bytes: q, qd, qdd|tau read + tau|qdd written, 4·n·s per
    configuration; rnea_fd reads q, qd, qdd, tau_in and writes tau, qdd', 6·n·s."""
    return (6 if kernel == "rnea_fd" else 4) * n * B * esize


def nsets_for(n, B, esize, kernel, rotate_gib):
    return max(2, int(np.ceil(rotate_gib * (1 << 30) / max(1, set_bytes(n, B, esize, kernel)))))


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def time_launches(launch, steps, warmup, world, spinup_ms=0.0, streams=1, sync_every=0):
    """launch(i, stream_ptr) issues step i.  Warmup, then exactly `steps` launches
    bracketed by barrier + synchronize on both sides (the clock stops at the closing
    synchronize, before the closing barrier) and one hipEvent pair on the launch stream (no
    per-launch events inside the timed region: an event record between launches on one
    stream inflates a ~22 us step to ~32 us).  With streams > 1 consecutive steps rotate
    over that many streams; the event pair then spans all of them.
    Returns (wall s, device ms per step)."""
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
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    e0.record(main)
    for st in strs[1:]:
        st.wait_event(e0)
    for i in range(steps):
        launch(i, sps[i % streams])
        if sync_every and (i + 1) % sync_every == 0 and i + 1 < steps:
            torch.cuda.synchronize()
    for st, end in zip(strs[1:], ends[1:]):
        end.record(st)
        main.wait_event(end)
    e1.record(main)
    torch.cuda.synchronize()
    # the region ends at this rank's synchronize; the barrier after it only re-aligns the
    # ranks (its collective latency is not step time), and max over ranks takes the slowest
    t1 = time.perf_counter()
    barrier(world)
    return t1 - t0, e0.elapsed_time(e1) / steps


def time_graph(launch, steps, per_graph=100, spinup_ms=100.0):
    """The same launches replayed from a HIP graph: `per_graph` consecutive launches (rotating
    input sets) are stream-captured once (torch.cuda.graph), then the graph is replayed
    ceil(steps / per_graph) times between one hipEvent pair.
    Returns (wall s, device ms per launch, launches replayed)."""
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
    reps = max(1, -(-steps // per_graph))
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
    launches = reps * per_graph
    return t1 - t0, e0.elapsed_time(e1) / launches, launches


def batch_launcher(mb, sets, kernel, dtype, layout="soa", B=None):
    """Closure issuing the batched C-ABI entry point(s) of `kernel` on input set i % len(sets)."""
    lib = ffi.lib()
    suffix = "f32" if dtype == torch.float32 else "f64"
    ns = len(sets)
    lay = "tiled_" if layout == "tiled" else ""
    rnea = getattr(lib, f"multibody_rnea_batch_{lay}{suffix}")
    fd = getattr(lib, f"multibody_fd_batch_{lay}{suffix}")
    idfd = getattr(lib, f"multibody_rnea_fd_batch_{lay}{suffix}")
    if layout == "tiled":
        tail = (B,)
    else:
        B = sets[0][1][0].shape[1]
        tail = (B, B)
    calls = []
    for i, o in sets:
        p = [t.data_ptr() for t in i] + [t.data_ptr() for t in o]
        if kernel == "rnea_fd":
            calls.append(((idfd, (mb.handle,) + tuple(p) + tail),))
        else:
            calls.append(((rnea if kernel == "rnea" else fd, (mb.handle, p[0], p[1], p[2], p[3]) + tail),))

    def launch(i, sp):
        for fn, args in calls[i % ns]:
            if fn(*args, sp):
                raise RuntimeError(ffi.last_error())

    # `calls` holds raw device pointers: the closure owns the tensors, or a caller that drops
    # its `sets` leaves the launches on freed (and, after torch.cuda.graph's empty_cache,
    # unmapped) memory
    launch.keep = sets
    return launch


# the batched mass matrix and kinematics read q (n rows) and write
# rows_out rows per configuration (SoA, one write each): CRBA n*n (the ABI's column-major matrix,
# lower triangle exact zeros), Jacobian 6n, forward kinematics 3
Q_KERNELS = {"crba": lambda n: n * n, "jac": lambda n: 6 * n, "fwd_kin": lambda n: 3}


def q_launcher(mb, kernel, B, dtype, rotate_gib, seed=chains.SEED, layout="soa"):
    """Closure issuing multibody_{crba,jac,fwd_kin}_batch_* (or *_batch_tiled_*) on input set
    i % nsets (q only); returns (launch, bytes per launch)."""
    n, rows = mb.n, Q_KERNELS[kernel](mb.n)
    es = 4 if dtype == torch.float32 else 8
    per = (n + rows) * B * es
    ns = max(2, int(np.ceil(rotate_gib * (1 << 30) / per)))
    lo, hi = chains.input_ranges(mb.limits(), "q")
    qs, outs = [], []
    for s in range(ns):
        q = torch.empty((n, B), dtype=dtype, device="cuda")
        ffi.fill_uniform(q, lo, hi, seed + 1000 * s)
        if layout == "tiled":
            q = ffi.to_tiled(q)
            outs.append(torch.empty((q.shape[0], rows, ffi.TILE), dtype=dtype, device="cuda"))
        else:
            outs.append(torch.empty((rows, B), dtype=dtype, device="cuda"))
        qs.append(q)
    torch.cuda.synchronize()
    sfx = ("tiled_" if layout == "tiled" else "") + ("f32" if dtype == torch.float32 else "f64")
    fn = getattr(ffi.lib(), f"multibody_{kernel}_batch_{sfx}")
    tail = (B,) if layout == "tiled" else (B, B)
    calls = [(mb.handle, q.data_ptr(), o.data_ptr()) + tail for q, o in zip(qs, outs)]

    def launch(i, sp):
        if fn(*calls[i % ns], sp):
            raise RuntimeError(ffi.last_error())

    launch.keep = (qs, outs)
    return launch, per


def _on_stream(sp):
    """torch stream context for a raw stream pointer (the timing helpers pass torch's own)."""
    cur = torch.cuda.current_stream()
    if sp is None or (sp.value or 0) == cur.cuda_stream:
        return contextlib.nullcontext()
    return torch.cuda.stream(torch.cuda.ExternalStream(sp.value))


def rollout_launcher(mb, B, dtype, K, dt=1e-3, seed=chains.SEED, reset=True, reset_only=False):
    """Closure issuing multibody_rollout_batch_* (q, qd updated in place) on a [K*n, B] torque
    sequence drawn within the effort limits.  reset=True (the bench's workload): every launch
    first restores q, qd from the initial draw (one [2][n][B] device copy on the launch stream),
    as an MPC iteration restarts its candidates from the measured state.  Without it the state
    integrates launch after launch: random torques at the effort limits drive the light wrist
    links past 1e3 rad/s within 50 launches (800 steps) and 95% of the configurations to Inf/NaN
    within 200 (tools/roll_state.py, profiles/r05/roll_state.log) -- the timed region would run
    on a diverged state.  reset_only=True issues the copy alone (its cost, reported beside)."""
    n = mb.n
    state = torch.empty((2, n, B), dtype=dtype, device="cuda")
    q, qd = state[0], state[1]
    lim = mb.limits()
    ffi.fill_uniform(q, *chains.input_ranges(lim, "q"), seed)
    ffi.fill_uniform(qd, *chains.input_ranges(lim, "qd"), seed + 1)
    init = state.clone()
    tau = torch.empty((K * n, B), dtype=dtype, device="cuda")
    lo, hi = chains.input_ranges(lim, "tau")
    ffi.fill_uniform(tau, lo * K, hi * K, seed + 2)  # list * K: the joints' ranges for every step row
    fn = getattr(ffi.lib(), f"multibody_rollout_batch_{'f32' if dtype == torch.float32 else 'f64'}")
    args = (mb.handle, q.data_ptr(), qd.data_ptr(), tau.data_ptr(), dt, K, None, B, B)
    marks = []  # (start, end) hipEvent pairs around the kernel alone, when launch.mark is set

    def launch(i, sp):
        if reset:
            with _on_stream(sp):
                state.copy_(init)
        if reset_only:
            return
        if launch.mark:
            with _on_stream(sp):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if fn(*args, sp):
                    raise RuntimeError(ffi.last_error())
                e1.record()
            marks.append((e0, e1))
        elif fn(*args, sp):
            raise RuntimeError(ffi.last_error())

    def kernel_ms(n, warm=3):
        """Mean device time of the rollout kernel alone over n reset + launch steps: an event pair
        around each kernel (after its reset copy) on the launch stream."""
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for i in range(warm):
            launch(i, sp)
        torch.cuda.synchronize()
        marks.clear()
        launch.mark = True
        try:
            for i in range(n):
                launch(i, sp)
            torch.cuda.synchronize()
        finally:
            launch.mark = False
        return float(np.mean([a.elapsed_time(b) for a, b in marks]))

    launch.mark = False
    launch.kernel_ms = kernel_ms
    launch.keep = (q, qd, tau, init)
    return launch


# Timed work of every secondary line, independent of --steps (the driver runs --steps 20): at
# least SIDE_MIN_LAUNCHES launches and at least SIDE_TARGET_MS of them.
SIDE_TARGET_MS = 60.0
SIDE_MIN_LAUNCHES = 200
SIDE_MAX_LAUNCHES = 40000


def budget_steps(launch, target_ms=SIDE_TARGET_MS, lo=SIDE_MIN_LAUNCHES, hi=SIDE_MAX_LAUNCHES):
    """Launch count for ~target_ms of timed work, from a 20-launch calibration."""
    _, ms = time_launches(launch, 20, 3, 1, 0.0)
    return int(min(hi, max(lo, np.ceil(target_ms / max(ms, 1e-4)))))


def per_rank(r, world, dev):
    """[{rank, wall_s, kernel_ms_avg, steps}] of every rank, in rank order (per-GPU
    device time beside the max-over-ranks line)."""
    rows = rdist.gather_over_ranks([r["wall"], r["kernel_ms_avg"], r["steps"]], world, dev)
    return [{"rank": k, "wall_s": w, "kernel_ms_avg": km, "steps": int(st)} for k, (w, km, st) in enumerate(rows)]


def measure(mb, kernel, dt_name, B, layout, steps, warmup, world, rotate_gib, seed, spinup_ms=300.0, streams=1,
            sync_every=0, graph=False, extra_streams=(), dev=None):
    """Time `steps` launches of `kernel` over batches of B resident configurations (steps=None:
    a budget of ~SIDE_TARGET_MS of launches, budget_steps).  Returns a dict (wall,
    kernel_ms_avg, bytes, sets, steps) plus the graph-replay figures if asked."""
    ds = DT[dt_name]
    es = 4 if dt_name == "f32" else 8
    ns = nsets_for(mb.n, B, es, kernel, rotate_gib)
    sets = make_sets(mb, B, ds, kernel, ns, seed, layout=layout)
    launch = batch_launcher(mb, sets, kernel, ds, layout, B)
    if steps is None:
        # every rank times the same launch count (the largest budget), so max-over-ranks compares
        # equal work
        steps = int(rdist.max_over_ranks([budget_steps(launch)], world, dev)[0]) if world > 1 else budget_steps(launch)
    wall, km = time_launches(launch, steps, warmup, world, spinup_ms, streams, sync_every)
    r = {"wall": wall, "kernel_ms_avg": km, "bytes": set_bytes(mb.n, B, es, kernel), "sets": ns, "steps": steps}
    if graph:
        gw, gkm, gl = time_graph(launch, steps)
        r.update({"graph_wall": gw, "graph_kernel_ms_avg": gkm, "graph_launches": gl})
    if extra_streams:
        r["streams_ms"] = {ns: time_launches(launch, steps, warmup, world, 50.0, ns)[1] for ns in extra_streams}
    del sets, launch
    torch.cuda.empty_cache()
    return r


def layout_ab(mb, kernel, dt_name, B, rounds=5, seed=chains.SEED + 5):
    """The same kernel on SoA rows and on the tiled layout, interleaved round by round in one
    process (each round ~SIDE_TARGET_MS / 2 of launches per layout): per-launch medians."""
    ds = DT[dt_name]
    es = 4 if dt_name == "f32" else 8
    ns = nsets_for(mb.n, B, es, kernel, 1.25)
    launches = {lay: batch_launcher(mb, make_sets(mb, B, ds, kernel, ns, seed, layout=lay), kernel, ds, lay, B)
                for lay in ("soa", "tiled")}
    steps = budget_steps(launches["soa"], SIDE_TARGET_MS / 2)
    res = {lay: [] for lay in launches}
    for r in range(rounds):
        for lay, launch in launches.items():
            res[lay].append(time_launches(launch, steps, 5, 1, 100.0 if r == 0 else 0.0)[1] * 1e3)
    del launches
    torch.cuda.empty_cache()
    out = {f"{lay}_us_median": float(np.median(v)) for lay, v in res.items()}
    out.update({f"{lay}_us_rounds": [round(x, 3) for x in v] for lay, v in res.items()})
    out.update({"launches_per_round": steps, "rounds": rounds, "batch": B, "dtype": dt_name,
                "note": "interleaved in one process: soa then tiled, every round"})
    return out


def side_workloads(mb7, a):
    """Secondary measurements (one GPU, serial launches): the other SURVEY §8(d) configs."""
    sec = {}

    def one(name, mb, kernel, dt_name, B=a.batch, layout=a.layout, graph=False, streams=(1,)):
        r = measure(mb, kernel, dt_name, B, layout, None, 5, 1, a.rotate_gib, chains.SEED + 31, graph=graph,
                    extra_streams=streams[1:])
        sec[name] = {"evals_per_s": B * r["steps"] / r["wall"], "kernel_ms_avg": r["kernel_ms_avg"], "batch": B,
                     "launches": r["steps"],
                     "layout": layout, "dtype": dt_name, "hbm_frac": r["bytes"] / (r["kernel_ms_avg"] * 1e-3) / HBM_PEAK,
                     "kernel_path": mb.kernel_path(kernel, dt_name == "f64", B, layout == "tiled"),
                     "kernel_form": str(mb.kernel_form(kernel, dt_name == "f64", B, layout == "tiled"))}
        if kernel in ("rnea", "fd"):
            model = "fr3" if mb.n == 7 else f"chain{mb.n}" if "tree" not in name else None
            if model:
                form = mb.kernel_form(kernel, dt_name == "f64", B, layout == "tiled")
                sec[name]["valu"] = valu_roofline(workload_name(kernel, mb.n, dt_name, layout, B), f"{kernel}_{model}",
                                                  f"{kernel}_{model}_{dt_name}" + ("" if B == a.batch else f"_b{B}"),
                                                  dt_name, B, r["kernel_ms_avg"], form in (2, 4))
                ref = reference_formulation(f"{kernel}_{model}", B, r["kernel_ms_avg"])
                if ref:
                    sec[name]["reference_formulation"] = ref
        if graph:  # the same launches replayed from a HIP graph; rates over the launches replayed
            gl = r["graph_launches"]
            # eager back-to-back launches from Python are host-bound when the graph replay of the
            # same launches is faster: the graph line is then the device-bound rate
            sec[name]["host_bound"] = bool(r["kernel_ms_avg"] > 1.05 * r["graph_kernel_ms_avg"])
            sec[name + "_graph"] = {"evals_per_s": B * gl / r["graph_wall"],
                                    "kernel_ms_avg": r["graph_kernel_ms_avg"], "batch": B, "layout": layout,
                                    "dtype": dt_name, "launches": gl,
                                    "hbm_frac": r["bytes"] / (r["graph_kernel_ms_avg"] * 1e-3) / HBM_PEAK,
                                    "launch": "HIP graph of 100 captured C-ABI launches, replayed"}
        for ns, km in r.get("streams_ms", {}).items():  # independent batches kept in flight on ns streams
            sec[f"{name}_{ns}streams"] = {"evals_per_s": B / (km * 1e-3), "step_ms_device": km, "batch": B,
                                          "dtype": dt_name, "streams": ns,
                                          "hbm_frac_effective": r["bytes"] / (km * 1e-3) / HBM_PEAK,
                                          "launch": f"consecutive batches rotate over {ns} HIP streams"}

    one("rnea_fr3_f32_b65536", mb7, "rnea", "f32", 65536, graph=True, streams=(1, 2, 4))    # config 2
    one("fd_fr3_f32_b65536", mb7, "fd", "f32", 65536, graph=True, streams=(1, 2, 4))        # config 3
    one("fd_fr3_f64", mb7, "fd", "f64")
    one("fd_fr3_f32", mb7, "fd", "f32", streams=(1, 2))
    one("rnea_fd_fr3_f64_b131072", mb7, "rnea_fd", "f64", 1 << 17, graph=True)  # config 4, one GPU's 2^17 shard
    # SURVEY §8(e) scaling caveat: an extra large-batch point (2^24 configurations per launch,
    # 3.8 GB per input set) where the launch's ramp and tail are amortised
    one("rnea_fr3_f64_b16777216", mb7, "rnea", "f64", 1 << 24)
    mb30 = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30))
    mb30.upload()
    one("rnea_chain30_f32", mb30, "rnea", "f32")             # config 5
    one("rnea_chain30_f64", mb30, "rnea", "f64")             # the same chain in the reference's Real
    # a floating-base branching tree (6 virtual + 8 joints, 2 prismatic)
    mbt = ffi.Multibody.from_urdf_string(chains.tree_urdf(floating=True), ffi.FLOATING_BASE)
    mbt.upload()
    one("rnea_float14_tree_f32", mbt, "rnea", "f32")
    one("fd_float14_tree_f32", mbt, "fd", "f32")
    # batched mass matrix / Jacobian / forward kinematics: q in, n*n /
    # 6n / 3 rows out per configuration, SoA (fp64 also tiled), 2^20 configurations
    for kern in ("crba", "jac", "fwd_kin"):
        for dn, dt, lay in (("f64", torch.float64, "soa"), ("f64", torch.float64, "tiled"),
                            ("f32", torch.float32, "soa")):
            ql, per = q_launcher(mb7, kern, a.batch, dt, a.rotate_gib, layout=lay)
            nl = budget_steps(ql)
            w, km = time_launches(ql, nl, 3, 1, 100.0)
            name = f"{kern}_fr3_{dn}" + ("_tiled" if lay == "tiled" else "")
            sec[name] = {"evals_per_s": a.batch * nl / w, "kernel_ms_avg": km, "batch": a.batch,
                         "launches": nl, "layout": lay, "dtype": dn,
                         "bytes_per_eval": per // a.batch,
                         "hbm_frac": per / (km * 1e-3) / HBM_PEAK,
                         "kernel_path": mb7.kernel_path(kern, dn == "f64", a.batch)}
            del ql
    torch.cuda.empty_cache()
    # fused rollout: K forward-dynamics + Euler steps per launch
    K = 16
    for dn, dt in (("f32", torch.float32), ("f64", torch.float64)):
        rl = rollout_launcher(mb7, a.batch, dt, K)
        nl = budget_steps(rl, lo=100)
        w, lm = time_launches(rl, nl, 3, 1, 300.0)
        _, cm = time_launches(rollout_launcher(mb7, a.batch, dt, K, reset_only=True), nl, 3, 1, 0.0)
        km = rl.kernel_ms(min(nl, 100))
        sec[f"rollout_fr3_{dn}_K16"] = {"steps_per_launch": K, "evals_per_s": a.batch * K * nl / w,
                                        "launches": nl, "launch_ms_avg": lm, "reset_ms_avg": cm,
                                        "kernel_ms_avg": km, "kernel_path": mb7.kernel_path("rollout", dn == "f64"),
                                        "note": ("evals = configurations x Euler steps; q, qd stay on chip (LDS); "
                                                 "every launch restarts from the initial state (a [2][n][B] device "
                                                 "copy, reset_ms_avg, timed alone); evals_per_s includes it; "
                                                 "kernel_ms_avg = an event pair around each rollout kernel inside the "
                                                 "reset + launch loop (the copy excluded), mean over launches"),
                                        "valu": valu_roofline(f"rollout_fr3_{dn}_K16_b{a.batch}", "rollout_step_fr3",
                                                              f"rollout_fr3_{dn}", dn, a.batch * K, km, dn == "f32"),
                                        "reference_formulation": reference_formulation("rollout_step_fr3", a.batch * K, km)}
    # the MPC-sized rollout (65536 configurations, K = 16): the split of packed waves per step
    # (rollout_split_block2), device-bound rate from a HIP graph
    Bs = 65536
    rl = rollout_launcher(mb7, Bs, torch.float32, K)
    nl = budget_steps(rl, lo=200)
    w, lm, gl = time_graph(rl, nl)
    _, cm, _ = time_graph(rollout_launcher(mb7, Bs, torch.float32, K, reset_only=True), nl)
    sec["rollout_fr3_f32_K16_b65536_graph"] = {"steps_per_launch": K, "batch": Bs, "evals_per_s": Bs * K * gl / w,
                                               "launches": gl, "launch_ms_avg": lm, "reset_ms_avg": cm,
                                               "kernel_ms_avg": lm - cm,
                                               "launch": "HIP graph of 100 captured (reset copy + C-ABI launch) pairs, replayed",
                                               "note": "evals = configurations x Euler steps; kernel_ms_avg = "
                                                       "launch_ms_avg - reset_ms_avg (the copy's graph timed alone)"}
    return sec


def single_call(iters=2000):
    """latency of the reference's single-configuration ABI calls
    (multibody_rnea / _crba / _jac / _fwd_kin, rigidbody_bindings/src/lib.rs:15-70) as the C++
    consumer main.cpp:69-96 times them -- examples/single_call_bench.cpp, a child process
    linked against librigidbody_bindings.so.  Two runs: the default dispatch (the calling
    thread evaluates the GPU lane bodies compiled for the host, host_eval.cpp) and
    RB_SINGLE_GPU=1 (every call a GPU round trip: H2D, kernel, D2H, stream sync)."""
    exe = os.path.join(REPO, "rigidbody-rs_amd", "bin", "single_call_bench")
    if not os.path.exists(exe):
        return {"error": f"{exe} not built (make -C rigidbody-rs_amd)"}
    out = {}
    for name, env in (("host", {}), ("gpu", {"RB_SINGLE_GPU": "1"})):
        r = subprocess.run([exe, str(iters)], capture_output=True, text=True, timeout=300,
                           env={**os.environ, **env})
        if r.returncode != 0:
            out[name] = {"error": r.stderr[-500:]}
            continue
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
    out["how"] = ("C++ consumer (examples/single_call_bench.cpp), std::chrono around each call on the "
                  "main.cpp:103-105 input after 50 warm calls, result buffer freed per call; 'host' = the "
                  "default dispatch (lane bodies on the calling thread), 'gpu' = RB_SINGLE_GPU=1")
    return out


def native_batch(cases=(("rnea", "f32", 65536), ("fd", "f32", 65536), ("rnea", "f64", 131072), ("fd", "f64", 131072),
                        ("rnea_fd", "f64", 131072), ("rnea+fd", "f64", 131072))):
    """SURVEY §8(d) configs 2 / 3 (and config 4's 2^17 fp64 shard) as a native caller drives the
    batched C ABI: examples/batch_bench.cpp, a child process linked against
    librigidbody_bindings.so -- eager back-to-back calls on one stream (and their host cost per
    call) and the same calls replayed from a HIP graph, tiled layout, no Python in the loop."""
    exe = os.path.join(REPO, "rigidbody-rs_amd", "bin", "batch_bench")
    if not os.path.exists(exe):
        return {"error": f"{exe} not built (make -C rigidbody-rs_amd)"}
    out = {}
    for kind, dt, B in cases:
        r = subprocess.run([exe, kind, dt, str(B), "20000", "tiled"], capture_output=True, text=True, timeout=300)
        key = f"{kind}_fr3_{dt}_b{B}"
        out[key] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-500:]}
    out["how"] = ("C++ consumer (examples/batch_bench.cpp): 20000 calls of multibody_{rnea,fd,rnea_fd}_batch_tiled_* "
                  "over input sets rotated through >= 1.25 GiB, hipEvent pair on the stream; eager = back-to-back "
                  "calls, graph = the same calls captured 100 per HIP graph and replayed; rnea+fd = config 4's pair "
                  "as two calls (rnea then fd), rnea_fd = the same pair in one fused call")
    return out


def host_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share(cgroup_root="/sys/fs/cgroup"):
    """(cores, how): the host cores this process may use, read at run time -- the cgroup CPU
    quota when one is set (v2 cpu.max, or v1 cpu.cfs_quota_us / cpu.cfs_period_us), capped by
    the affinity set; otherwise the affinity set itself."""
    visible = host_cores()
    quota = None
    try:
        with open(os.path.join(cgroup_root, "cpu.max")) as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = (int(q) / int(period), f"cgroup v2 cpu.max = {q} {period}")
    except (OSError, ValueError):
        try:
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_quota_us")) as f:
                q = int(f.read())
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_period_us")) as f:
                period = int(f.read())
            if q > 0:
                quota = (q / period, f"cgroup v1 cfs quota {q} / period {period}")
        except (OSError, ValueError):
            pass
    if quota is not None:
        cores = max(1, min(visible, int(quota[0])))
        return cores, f"{quota[1]} -> {quota[0]:.2f} CPUs, affinity set {visible}"
    return visible, f"no cgroup CPU quota; affinity set of {visible} CPUs"


def cpu_baseline(n, kernel, cpu_seconds):
    """fp64 CPU restatement (oracle/, kind "port") timed on this host's cores."""
    from oracle import oracle, urdf_model

    oracle.build()
    xml = chains.fr3_urdf_text() if n == 7 else chains.synthetic_chain_urdf(n)
    raw = urdf_model.model_raw_from_urdf(xml)
    om = oracle.Model(raw)
    visible = host_cores()
    cores, how = cpu_share()
    mbl = ([l["lower"] for l in raw["limits"]], [l["upper"] for l in raw["limits"]],
           [l["velocity"] for l in raw["limits"]], [l["effort"] for l in raw["limits"]])
    kinds = {"fd": ("q", "qd", "tau"), "rnea_fd": ("q", "qd", "qdd", "tau")}.get(kernel, ("q", "qd", "qdd"))

    def inputs(B):
        return [chains.host_uniform(n, B, *chains.input_ranges(mbl, kind), chains.SEED + k)
                for k, kind in enumerate(kinds)]

    if kernel == "rnea_fd":
        def call(q, qd, qdd, tau, nthreads):
            return om.rnea_batch(q, qd, qdd, nthreads=nthreads), om.fd_batch(q, qd, tau, nthreads=nthreads)
    else:
        call = om.rnea_batch if kernel == "rnea" else om.fd_batch
    cal = inputs(20000)
    t = time.perf_counter()
    call(*cal, nthreads=1)
    rate1 = 20000 / (time.perf_counter() - t)
    t = time.perf_counter()
    om.crba_batch(cal[0], nthreads=1)
    crba1 = 20000 / (time.perf_counter() - t)
    sample = int(min(max(rate1 * cpu_seconds, 1e5), 5e7))
    x = inputs(sample)
    t = time.perf_counter()
    call(*x, nthreads=cores)
    dt = time.perf_counter() - t
    return {"value": sample / dt, "unit": "evals/s", "cores": cores, "kind": "port",
            "cores_source": how, "host_cpus_visible": visible, "nproc": os.cpu_count(),
            "single_thread_evals_per_s": rate1, "single_thread_us_per_call": 1e6 / rate1,
            "single_thread_crba_us_per_call": 1e6 / crba1,
            "sample": f"{sample} {'fr3' if n == 7 else f'chain{n}'} configs (same distributions/seed as the GPU run), "
                      f"fp64 oracle {kernel} over {cores} OpenMP threads ({how}), {dt:.2f} s wall; "
                      f"single-thread {rate1:.3g} evals/s (the reference's one-call-per-configuration use, "
                      f"main.cpp:69)"}


def load_traffic(workload):
    path = os.path.join(REPO, "profiles", f"traffic_{workload}.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def _load_json(rel):
    path = os.path.join(REPO, rel)
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def held_clock(name):
    """Median in-kernel shader clock (GHz) of kernel `name` under sustained load, from the
    committed clock probe (tools/clock_probe.py, profiles/r06/clock_probe.jsonl), or None."""
    path = os.path.join(REPO, "profiles", "r06", "clock_probe.jsonl")
    if not os.path.exists(path):
        return None
    for ln in open(path):
        if ln.strip().startswith("{"):
            d = json.loads(ln)
            if d.get("kernel") == name:
                return d.get("clock_GHz_median")
    return None


def valu_roofline(workload, op_key, clock_key, dt_name, evals, kern_ms, packed):
    """roofline.valu for a VALU-heavy kernel (SURVEY §8(d) "reported alongside"): the committed
    PMC counters of this workload's kernel (profiles/traffic_<workload>.json) over this run's
    kernel time.
      issue_frac = SQ_INSTS_VALU x cycles per wave64 VALU instruction / (1024 SIMDs x clock x
        kernel time): the fraction of the SIMDs' vector issue the kernel's instructions fill, at
        2.4 GHz and at the clock the chip holds under this kernel (clock probe).  4 cycles for
        fp64 and packed fp32 (v_pk_*) kernels (the measured wave64 issue of v_fma_f64 /
        v_pk_fma_f32: 16 lanes/clk/SIMD fp64, 2 x 16 packed), 2 for scalar fp32 (32 lanes/clk,
        MI355X_MICROARCH.md 'Per-instruction cycle constants').
      flop_frac = VALU FLOPs executed (gfx950 SQ_INSTS_VALU_FLOPS_*, x 64 lanes) / the dtype's
        vector peak (fp32 157.3 TF, fp64 78.6 TF at 2.4 GHz).
    Every figure here is what the kernel itself executes, so each *_frac is <= 1 and no rate
    exceeds its peak (roofline_violations); the reference formulation's operation count is
    reported beside the roofline, not in it (reference_formulation)."""
    tr = load_traffic(workload)
    t = kern_ms * 1e-3
    cyc = 4 if (dt_name == "f64" or packed) else 2
    out = {"bound": "valu", "unit": "fraction", "evals_per_launch": evals, "cycles_per_valu_inst": cyc}
    sq = (tr or {}).get("sq_counters_per_launch", {})
    if "SQ_INSTS_VALU" in sq:
        busy = sq["SQ_INSTS_VALU"] * cyc / SIMDS  # vector issue cycles per SIMD per launch
        # SQ_INSTS_VALU counts wave-instructions: x 64 lanes / evaluations = the VALU instructions
        # one lane issues per configuration it evaluates (half a packed pair's stream)
        out.update({"insts_per_eval": sq["SQ_INSTS_VALU"] * 64 / evals,
                    "issue_frac_2p4ghz": busy / (CLOCK_PEAK * t)})
        if "SQ_ACTIVE_INST_VALU" in sq:  # wave-cycles a VALU instruction holds its wave (quad-cycles x 4)
            out["wave_cycles_per_valu_inst"] = sq["SQ_ACTIVE_INST_VALU"] * 4 / sq["SQ_INSTS_VALU"]
        clk = held_clock(clock_key)
        if clk:
            out.update({"held_clock_ghz": clk, "issue_frac_held": busy / (clk * 1e9 * t),
                        "clock_source": f"profiles/r06/clock_probe.jsonl [{clock_key}]"})
        fl = tr.get("valu_flops_per_launch", {})
        # the SQ_INSTS_VALU_FLOPS_* counters count per wave-instruction (an FMA 2, a packed FMA 4):
        # x 64 lanes for the FLOPs executed, as rocprof-compute's VALU FLOP metric
        kf = 64 * sum(v for k, v in fl.items() if dt_name.upper()[1:] in k)  # FP32 / FP64 (+ _TRANS)
        if kf:
            out.update({"kernel_flops_per_eval": kf / evals, "kernel_tflops": kf / t / 1e12,
                        "flop_frac": kf / t / VALU_FLOP_PEAK[dt_name], "flop_peak_tflops": VALU_FLOP_PEAK[dt_name] / 1e12})
        out["counters_source"] = f"profiles/traffic_{workload}.json (rocprofv3 PMC passes of this kernel)"
    return out


CONFIG4_BATCH = 1 << 20  # the global fp64 RNEA + FD batch


def reference_formulation(op_key, evals, kern_ms):
    """The reference formulation's operations per evaluation (op-counting build of the oracle,
    oracle/flops.cpp -> profiles/r04/op_counts.json: quaternion transforms, isometry inverses,
    6-vector cross products as multibody.rs / spatial.rs / inertia.rs write them) and the FLOP
    rate that formulation would need to match this kernel's evaluation rate.  Not a roofline
    figure: the kernel executes 2.7-4.4x fewer operations (roofline.valu.kernel_flops_per_eval),
    so this rate may exceed the VALU peak."""
    ops = _load_json("profiles/r04/op_counts.json")
    if not ops or op_key not in ops or not kern_ms:
        return None
    ref = ops[op_key]["flops"]
    return {"flops_per_eval": ref, "equiv_tflops_at_this_rate": ref * evals / (kern_ms * 1e-3) / 1e12,
            "source": f"profiles/r04/op_counts.json [{op_key}] (oracle/flops.cpp)",
            "note": "what the reference's formulation would have to execute per second for this "
                    "evaluation rate; not a roofline figure (the kernel runs fewer operations)"}


def roofline_violations(line):
    """Consistency of a bench line's roofline block (tests/test_bench_launch.py): every *_frac
    anywhere in the line within (0, 1], roofline.achieved <= roofline.peak, and the VALU block's
    kernel_tflops <= flop_peak_tflops.  Returns the list of violations (empty = consistent)."""
    bad = []

    def walk(x, path):
        if isinstance(x, dict):
            for k, v in x.items():
                p = f"{path}.{k}" if path else k
                if k.endswith("frac") and isinstance(v, (int, float)) and not (0 < v <= 1.0):
                    bad.append(f"{p} = {v}")
                walk(v, p)
        elif isinstance(x, list):
            for i, v in enumerate(x):
                walk(v, f"{path}[{i}]")

    walk(line, "")
    rf = line.get("roofline") or {}
    if rf.get("achieved") is not None and rf.get("peak") and rf["achieved"] > rf["peak"]:
        bad.append(f"roofline.achieved {rf['achieved']} > peak {rf['peak']}")

    def valu_rates(x, path):
        if isinstance(x, dict):
            if "kernel_tflops" in x and "flop_peak_tflops" in x and x["kernel_tflops"] > x["flop_peak_tflops"]:
                bad.append(f"{path}.kernel_tflops {x['kernel_tflops']} > {x['flop_peak_tflops']}")
            for k, v in x.items():
                valu_rates(v, f"{path}.{k}")

    valu_rates(rf, "roofline")
    for k, v in (line.get("secondary") or {}).items():
        if isinstance(v, dict) and isinstance(v.get("valu"), dict):
            valu_rates(v["valu"], f"secondary.{k}.valu")
    return bad


def workload_name(kernel, n, dt_name, layout, B):
    return f"{kernel}_{'fr3' if n == 7 else f'chain{n}'}_{dt_name}_{layout}_b{B}"


# ------------------------------------------------------------------ the printed line
LINE_MAX_BYTES = 16384  # the one stdout line stays well under this (tests/test_bench_launch.py)


def finite(x):
    """x with every non-finite float replaced by None (strict JSON has no NaN / Infinity)."""
    if isinstance(x, float):
        return x if np.isfinite(x) else None
    if isinstance(x, dict):
        return {k: finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite(v) for v in x]
    return x


def _sig(x, digits=4):
    if isinstance(x, (int, float)) and not isinstance(x, bool) and np.isfinite(x) and x != 0:
        return float(f"{x:.{digits}g}")
    return x


def _summary(v):
    """One secondary entry of the full line -> {us, frac} (+ a rate where there is no kernel time)."""
    if not isinstance(v, dict):
        return None
    if "soa_us_median" in v:  # layout A/B
        return {"soa_us": _sig(v["soa_us_median"]), "tiled_us": _sig(v["tiled_us_median"])}
    out = {}
    ms = v.get("kernel_ms_avg", v.get("step_ms_device", v.get("kernel_ms_avg_max_rank", v.get("ms_per_step"))))
    if isinstance(ms, (int, float)):
        out["us"] = _sig(ms * 1e3)
    if isinstance(v.get("graph_ms_per_step_max_rank"), (int, float)):
        out["graph_us"] = _sig(v["graph_ms_per_step_max_rank"] * 1e3)
    fr = v.get("hbm_frac", v.get("hbm_frac_effective", v.get("hbm_frac_max_rank")))
    if isinstance(fr, (int, float)):
        out["frac"] = _sig(fr, 3)
    iv = (v.get("valu") or {}).get("issue_frac_held")
    if isinstance(iv, (int, float)):
        out["valu_frac"] = _sig(iv, 3)
    for k in ("evals_per_s", "pairs_per_s", "graph_pairs_per_s"):
        if isinstance(v.get(k), (int, float)) and ("us" not in out or "per_rank" in v):
            out[k] = _sig(v[k])  # the N > 1 split lines: their whole-job rate too
    return out or None


def compact_line(full):
    """The ONE line bench.py prints: the contract keys, roofline, cpu_baseline and a per-workload
    {us, frac} summary of every secondary measurement; everything else stays in the detail file
    (write_detail).  Strict JSON, < LINE_MAX_BYTES even at --gpus 8."""
    cfg = full["config"]
    rf = full["roofline"]
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    line["config"] = {k: cfg[k] for k in ("workload", "kernel", "model", "split", "batch_per_gpu", "global_batch",
                                          "parallelism", "kernel_path", "input_sets") if k in cfg}
    line["config"]["layout"] = "tiled [B/256][n][256]" if cfg["layout"].startswith("tiled") else "SoA [n][B]"
    line["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                               "bytes_per_eval", "evals_per_launch", "kernel_ms_avg")}
    vl = rf.get("valu") or {}
    if "issue_frac_held" in vl:
        line["roofline"]["valu_issue_frac_held"] = vl["issue_frac_held"]
    line["roofline"]["check"] = full.get("roofline_check", "ok")
    if "cpu_baseline" in full:
        cb = full["cpu_baseline"]
        line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind") if k in cb}
        line["cpu_baseline"]["sample"] = str(cb.get("sample", ""))[:240]
        if "single_thread_evals_per_s" in cb:
            line["cpu_baseline"]["single_thread_evals_per_s"] = cb["single_thread_evals_per_s"]
    elif "cpu_baseline_note" in full:
        line["cpu_baseline_note"] = full["cpu_baseline_note"][:200]
    if "per_rank" in full:  # [wall s, device ms per launch] by rank
        line["per_rank"] = [[_sig(r["wall_s"]), _sig(r["kernel_ms_avg"])] for r in full["per_rank"]]
    sec = {}
    for name, v in (full.get("secondary") or {}).items():
        if name == "single_call":
            s = {f"{k}_{w}_us": v[w][k]["median_us"] for w in ("host", "gpu") if isinstance(v.get(w), dict)
                 for k in ("rnea", "crba") if isinstance(v[w].get(k), dict)}
        elif name == "native_batch":
            s = {k: _sig(x["graph_us_per_call"]) for k, x in v.items()
                 if isinstance(x, dict) and "graph_us_per_call" in x}
        else:
            s = _summary(v)
        if s:
            sec[name] = s
    if sec:
        line["secondary"] = sec
    if full.get("detail_file"):
        line["detail_file"] = full["detail_file"]
    return finite(line)


def dumps_strict(obj):
    return json.dumps(finite(obj), allow_nan=False, separators=(",", ":"))


def write_detail(full, world):
    """The full line (every secondary block, notes, VALU counters) to a file beside the run:
    $RB_BENCH_DETAIL, else gpurun_out/bench_detail_n<world>.json.  Returns the path or None."""
    path = os.environ.get("RB_BENCH_DETAIL") or os.path.join(REPO, "gpurun_out", f"bench_detail_n{world}.json")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(json.dumps(finite(full), allow_nan=False, indent=1) + "\n")
        return os.path.relpath(path, REPO) if path.startswith(REPO) else path
    except OSError as e:
        print(f"bench.py: detail file not written ({e})", file=sys.stderr)
        return None


def main(a):
    world, rank, dev = init_dist(a)
    n = a.dof
    esize = 4 if a.dtype == "f32" else 8
    mb = load_model(world, rank, n, dev)
    strong = a.split == "strong"
    lo, hi = rdist.shard(a.batch, rank, world) if strong else (0, a.batch)
    B = hi - lo  # this rank's configurations per step
    global_batch = a.batch if strong else a.batch * world
    seed = chains.SEED if strong else rdist.rank_seed(chains.SEED, rank)
    def stub_measure(B_, steps):
        # plumbing rehearsal: same ranks, collectives and reporting, no device work
        t0 = time.perf_counter()
        barrier(world)
        wall_ = time.perf_counter() - t0 + 1e-9
        return {"wall": wall_, "kernel_ms_avg": wall_ / steps * 1e3, "bytes": set_bytes(n, B_, esize, a.kernel),
                "sets": 0, "steps": steps}

    if a.stub:
        r = stub_measure(B, a.steps)
        kpath = "stub"
    else:
        r = measure(mb, a.kernel, a.dtype, B, a.layout, a.steps, a.warmup, world, a.rotate_gib, seed, a.spinup_ms,
                    a.streams, a.sync_every)
        kpath = mb.kernel_path(a.kernel, a.dtype == "f64", B, a.layout == "tiled")
    ranks = per_rank(r, world, dev)
    wall, kern_ms = rdist.max_over_ranks([r["wall"], r["kernel_ms_avg"]], world, dev)
    value = global_batch * a.steps / wall
    bytes_per_eval = set_bytes(n, 1, esize, a.kernel)
    achieved = bytes_per_eval * B / (kern_ms * 1e-3)
    workload = workload_name(a.kernel, n, a.dtype, a.layout, a.batch)
    traffic = load_traffic(workload) if not strong else None
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": ("stub (CPU rehearsal of the rank plumbing, no kernels)" if a.stub else
                 "synthetic (device splitmix64, SURVEY.md §8(d) distributions, seed 20250224)"),
        "config": {"workload": workload, "kernel": a.kernel, "model": "fr3 7-DOF" if n == 7 else f"chain{n}",
                   "layout": ("tiled [B/256][n][256] (each 256-configuration tile of all joints contiguous)"
                              if a.layout == "tiled" else "SoA rows [n][B]"),
                   "streams": a.streams, "split": a.split,
                   "batch_per_gpu": B, "global_batch": global_batch, "dof": n,
                   "parallelism": f"dp{world} ({a.split} split; independent shards, RCCL model broadcast)",
                   "input_sets": r["sets"], "rotated_bytes": r["sets"] * r["bytes"], "kernel_path": kpath,
                   "input_domain": ("every input of every configuration is read and checked (NaN / Inf / "
                                    "|q| past 2^41 rad fp64, 2^22 fp32 -> NaN outputs; rigidbody_batch.h "
                                    "'Input domain'), q_0 included, which FR3's torques do not depend on")},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK,
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "bytes_per_eval": bytes_per_eval, "evals_per_launch": B, "kernel_ms_avg": kern_ms,
                     "timing": (f"kernel_ms_avg = hipEvent pair on the launch stream around the {a.steps} timed "
                                f"launches / {a.steps} ({a.streams} stream(s); includes the inter-launch gap); "
                                "max over ranks")},
    }
    if traffic:
        line["roofline"]["traffic_source"] = f"profiles/traffic_{workload}.json (rocprofv3 PMC passes)"
    if not a.stub:
        model = "fr3" if n == 7 else f"chain{n}"
        form = mb.kernel_form(a.kernel.split("_")[0], a.dtype == "f64", B, a.layout == "tiled")
        line["roofline"]["valu"] = valu_roofline(workload, f"{a.kernel.split('_')[0]}_{model}",
                                                 f"{a.kernel}_{model}_{a.dtype}", a.dtype, B, kern_ms, form in (2, 4))
        ref = reference_formulation(f"{a.kernel.split('_')[0]}_{model}", B, kern_ms)
        if ref:
            line["reference_formulation"] = ref
    if world > 1:
        line["per_rank"] = ranks
    sec = {}
    if world > 1 and not strong:
        # the same global 2^20 batch sharded across the ranks, beside the weak line.
        # Its own launch budget (>= SIDE_MIN_LAUNCHES, ~SIDE_TARGET_MS, the same count on every
        # rank): at N = 8 a 2^17 fp64 shard is ~7 us, so the driver's --steps 20 would time
        # ~0.14 ms of work.
        slo, shi = rdist.shard(a.batch, rank, world)
        if a.stub:
            rs = stub_measure(shi - slo, SIDE_MIN_LAUNCHES)
        else:
            rs = measure(mb, a.kernel, a.dtype, shi - slo, a.layout, None, 5, world, a.rotate_gib, chains.SEED, 100.0,
                         dev=dev)
        sw, sk = rdist.max_over_ranks([rs["wall"], rs["kernel_ms_avg"]], world, dev)
        sec["strong_split"] = {"evals_per_s": a.batch * rs["steps"] / sw, "global_batch": a.batch,
                               "batch_per_gpu_max": -(-a.batch // world), "launches": rs["steps"],
                               "ms_per_step": sw / rs["steps"] * 1e3, "kernel_ms_avg_max_rank": sk,
                               "per_rank": per_rank(rs, world, dev), "scaling": "strong",
                               "timing": "own launch budget (bench.budget_steps, max over ranks), not --steps"}
        # SURVEY §8(d) config 4 -- "fr3 RNEA+ABA batch=2^20 fp64, sharded across 8 x MI355X": every
        # rank runs multibody_rnea_batch_f64 then multibody_fd_batch_f64 on its contiguous shard of
        # one global 2^20 batch (2^17 per GPU at N = 8; multibody.rs:111-174), own launch budget
        cfg4 = CONFIG4_BATCH
        c4lo, c4hi = rdist.shard(cfg4, rank, world)
        if a.stub:
            r4 = stub_measure(c4hi - c4lo, SIDE_MIN_LAUNCHES)
            k4 = "stub"
        else:
            # eager C-ABI calls from Python are host-bound at ~7 us per 2^17 fp64 launch: the same
            # launches replayed from a HIP graph give the device-bound rate beside them
            r4 = measure(mb, "rnea_fd", "f64", c4hi - c4lo, a.layout, None, 5, world, a.rotate_gib, chains.SEED,
                         100.0, graph=True, dev=dev)
            k4 = mb.kernel_path("rnea_fd", True, c4hi - c4lo, a.layout == "tiled")
        w4, km4 = rdist.max_over_ranks([r4["wall"], r4["kernel_ms_avg"]], world, dev)
        g4 = rdist.max_over_ranks([r4.get("graph_kernel_ms_avg", 0.0)], world, dev)[0]
        b4 = set_bytes(n, 1, 8, "rnea_fd")
        sec["strong_split_rnea_fd"] = {
            "config": "SURVEY §8(d) config 4: fr3 RNEA + forward dynamics, fp64, one global batch of "
                      f"{cfg4} sharded across {world} GPUs (contiguous shards, no collective on the data path)",
            "pairs_per_s": cfg4 * r4["steps"] / w4, "global_batch": cfg4, "batch_per_gpu_max": -(-cfg4 // world),
            "launches": r4["steps"], "ms_per_step": w4 / r4["steps"] * 1e3, "kernel_ms_avg_max_rank": km4,
            "hbm_frac_max_rank": b4 * -(-cfg4 // world) / (km4 * 1e-3) / HBM_PEAK if not a.stub else None,
            "graph_ms_per_step_max_rank": g4 if not a.stub else None,
            "graph_pairs_per_s": cfg4 / (g4 * 1e-3) if (g4 and not a.stub) else None,
            "bytes_per_pair": b4, "kernel_path": k4, "dtype": "f64", "layout": a.layout,
            "per_rank": per_rank(r4, world, dev), "scaling": "strong",
            "timing": "own launch budget (bench.budget_steps; one step = the RNEA launch + the FD launch on "
                      "the rank's shard), max over ranks; graph_*: the same launches replayed from a HIP graph "
                      "on every rank (device-bound), max over ranks",
            "status": "measured by the driver's N > 1 runs; our 1-GPU leases cannot run it (DESIGN.md §6)"}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.stub:
        line["cpu_baseline"] = cpu_baseline(n, a.kernel, a.cpu_seconds)
    elif world > 1:
        line["cpu_baseline_note"] = ("not measured at world > 1: the CPU baseline runs on rank 0 of the 1-GPU "
                                     "run only (bench.py --gpus 1), so the ranks' host cores stay idle here")
    if rank == 0 and not a.no_secondary and world == 1 and n == 7 and not a.stub:
        r2 = measure(mb, a.kernel, a.dtype, a.batch, a.layout, None, 5, 1, a.rotate_gib, seed, 50.0, 2)
        sec[f"{a.kernel}_{a.dtype}_{a.layout}_2streams"] = {
            "evals_per_s": a.batch * r2["steps"] / r2["wall"], "step_ms_device": r2["kernel_ms_avg"],
            "launches": r2["steps"], "hbm_frac_effective": r2["bytes"] / (r2["kernel_ms_avg"] * 1e-3) / HBM_PEAK}
        # SoA rows (north_star's layout) against the tiled layout, interleaved in this process,
        # for the headline kernel in both precisions and for forward dynamics in fp64
        for kern, dt_name in ((a.kernel, "f64"), (a.kernel, "f32"), ("fd", "f64")):
            sec[f"layout_ab_{kern}_{dt_name}"] = layout_ab(mb, kern, dt_name, a.batch)
        sec.update(side_workloads(mb, a))
        sec["single_call"] = single_call()
        sec["native_batch"] = native_batch()
        if "cpu_baseline" in line:
            cb = line["cpu_baseline"]
            sec["single_call"]["oracle_single_thread_us"] = {"rnea": cb["single_thread_us_per_call"],
                                                             "crba": cb["single_thread_crba_us_per_call"]}
    if sec:
        line["secondary"] = sec
    viol = roofline_violations(line)
    line["roofline_check"] = "ok" if not viol else viol  # fractions <= 1, rates <= peak
    if rank == 0:
        line["detail_file"] = write_detail(line, world)
        # the detail first (stderr: one short pointer), the compact strict-JSON line last on stdout
        print(f"bench.py: full detail in {line['detail_file']}", file=sys.stderr, flush=True)
        out = dumps_strict(compact_line(line))
        if len(out) >= LINE_MAX_BYTES:
            print(f"bench.py: compact line is {len(out)} B (>= {LINE_MAX_BYTES})", file=sys.stderr)
        print(out, flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(_ARGS)
