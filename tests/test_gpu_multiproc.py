"""The sharded batched path on real kernels with more than one rank (BASELINE
config 4 "RNEA+ABA batch=2^20 fp64, sharded across 8xMI355X"): two fresh rank processes,
started before any GPU call of theirs, share cuda:0 (RCCL refuses two ranks on one device,
so the process group is gloo -- the collectives carry only the model blob and the gathered
check data; the data path has none).  Rank 0 parses the URDF and broadcasts the packed model
blob, every rank rebuilds the model from it, takes its contiguous strong-split shard of one
global fp64 batch and runs multibody_rnea_batch_f64 then multibody_fd_batch_f64 on it
(q, qd, qdd -> tau -> qdd').  Rank 0 gathers the shards and checks them: bit-identical to
the unsharded batch evaluated in one process, the round trip qdd' = qdd, and oracle spot
columns (multibody.rs:111-174).  The same path through bench.py's own launcher
(`--gpus 2 --split strong --kernel rnea_fd`, RB_DIST_BACKEND=gloo) must print one line."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

from conftest import PKG, REPO, run_bench

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = textwrap.dedent('''
    import os, sys, json
    sys.path[:0] = [{repo!r}, {pkg!r}]
    import numpy as np, torch, torch.distributed as dist
    from rigidbody_amd import chains, dist as rdist, ffi
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # model: parsed on rank 0, blob broadcast (gloo carries it on the host), rebuilt elsewhere
    mb = rdist.broadcast_model(lambda: ffi.Multibody.new(), rank, world, torch.device("cpu"))
    mb.upload()
    G = {G}
    lim = mb.limits()
    b0, b1 = rdist.shard(G, rank, world)
    # this rank's columns of the one global batch (splitmix counter offset = b0)
    x = [chains.host_uniform(7, b1 - b0, *chains.input_ranges(lim, k), chains.SEED + 60 + i, start=b0)
         for i, k in enumerate(("q", "qd", "qdd"))]
    q, qd, qdd = (torch.as_tensor(a, device=dev) for a in x)
    tau = mb.rnea_batch(q, qd, qdd)          # multibody_rnea_batch_f64 on the shard
    back = mb.fd_batch(q, qd, tau)           # multibody_fd_batch_f64 on its torques
    # the same pair in one fused launch (multibody_rnea_fd_batch_f64, tau_in = the RNEA's torques)
    ftau, fback = mb.rnea_fd_batch(q, qd, qdd, tau)
    torch.cuda.synchronize()
    parts = [None] * world
    dist.all_gather_object(parts, (b0, b1, tau.cpu().numpy(), back.cpu().numpy(), ftau.cpu().numpy(),
                                   fback.cpu().numpy()))
    out = {{"rank": rank, "shard": [b0, b1], "kernel_path": [mb.kernel_path("rnea", True), mb.kernel_path("fd", True)]}}
    if rank == 0:
        from oracle import oracle, urdf_model
        full = [chains.host_uniform(7, G, *chains.input_ranges(lim, k), chains.SEED + 60 + i)
                for i, k in enumerate(("q", "qd", "qdd"))]
        T = np.zeros((7, G)); Q = np.zeros((7, G)); FT = np.zeros((7, G)); FQ = np.zeros((7, G))
        cover = np.zeros(G, int)
        for p0, p1, t, bq, ft, fq_ in parts:
            T[:, p0:p1] = t; Q[:, p0:p1] = bq; FT[:, p0:p1] = ft; FQ[:, p0:p1] = fq_; cover[p0:p1] += 1
        assert (cover == 1).all(), "shards must tile the batch exactly once"
        fq, fqd, fqdd = (torch.as_tensor(a, device=dev) for a in full)
        T1 = mb.rnea_batch(fq, fqd, fqdd).cpu().numpy()
        Q1 = mb.fd_batch(fq, fqd, torch.as_tensor(T1, device=dev)).cpu().numpy()
        out["bit_identical_tau"] = bool(np.array_equal(T, T1))
        out["bit_identical_fd"] = bool(np.array_equal(Q, Q1))
        FT1, FQ1 = (o.cpu().numpy() for o in mb.rnea_fd_batch(fq, fqd, fqdd, torch.as_tensor(T1, device=dev)))
        out["bit_identical_fused"] = bool(np.array_equal(FT, FT1) and np.array_equal(FQ, FQ1))
        out["fused_fd_equals_fd"] = bool(np.array_equal(FQ, Q))
        out["fused_tau_vs_rnea"] = float((np.abs(FT - T) / (1 + np.abs(T))).max())
        out["round_trip"] = float((np.abs(Q - full[2]) / (1 + np.abs(full[2]))).max())
        om = oracle.Model(urdf_model.model_raw_from_urdf(chains.fr3_urdf_text()))
        idx = np.linspace(0, G - 1, 1024).astype(int)
        ref = om.rnea_batch(*[a[:, idx] for a in full])
        out["oracle_tau"] = float((np.abs(T[:, idx] - ref) / (1 + np.abs(ref))).max())
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
''')


def test_two_ranks_shard_rnea_fd_f64(tmp_path):
    G = (1 << 18) + 777  # a ragged global batch: the shards end mid-tile
    script = tmp_path / "rank.py"
    script.write_text(WORKER.format(repo=REPO, pkg=PKG, G=G))
    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    r0 = outs[0]
    assert [o["shard"] for o in outs] == [[0, (G + 1) // 2], [(G + 1) // 2, G]]
    assert all(o["kernel_path"] == ["jit", "jit"] for o in outs)
    assert r0["bit_identical_tau"] and r0["bit_identical_fd"], r0
    assert r0["bit_identical_fused"] and r0["fused_fd_equals_fd"] and r0["fused_tau_vs_rnea"] <= 1e-9, r0
    assert r0["round_trip"] <= 1e-8, r0
    assert r0["oracle_tau"] <= 1e-9, r0


def test_bench_two_ranks_strong_rnea_fd():
    """bench.py's own N-rank launcher on the config-4 kernel pair: one JSON line, n_gpus 2,
    strong split of one global batch."""
    e = dict(os.environ, RB_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    compact, line = run_bench(["--gpus", "2", "--split", "strong", "--kernel", "rnea_fd", "--batch", str(1 << 18),
                               "--steps", "20", "--warmup", "5", "--no-secondary", "--no-cpu-baseline",
                               "--spinup-ms", "50", "--rotate-gib", "0.5"], e)
    assert compact["value"] == line["value"] and len(compact["per_rank"]) == 2
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["global_batch"] == 1 << 18 and line["config"]["batch_per_gpu"] == 1 << 17
    assert line["value"] > 0 and line["config"]["kernel_path"] == "jit"
    assert [x["rank"] for x in line["per_rank"]] == [0, 1] and all(x["kernel_ms_avg"] > 0 for x in line["per_rank"])


def test_bench_two_ranks_weak_with_strong_split():
    """The driver's N > 1 line shape (weak headline, --steps 20): the strong split beside it
    times its own launch budget (>= SIDE_MIN_LAUNCHES on every rank), and both carry per-rank
    device / wall times."""
    import bench

    e = dict(os.environ, RB_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    compact, line = run_bench(["--gpus", "2", "--batch", str(1 << 18), "--steps", "20", "--warmup", "5",
                               "--no-secondary", "--no-cpu-baseline", "--spinup-ms", "50", "--rotate-gib", "0.5"], e)
    assert set(compact["secondary"]) >= {"strong_split", "strong_split_rnea_fd"}
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["steps"] == 20
    assert len(line["per_rank"]) == 2 and all(x["steps"] == 20 for x in line["per_rank"])
    st = line["secondary"]["strong_split"]
    assert st["launches"] >= bench.SIDE_MIN_LAUNCHES
    assert [x["steps"] for x in st["per_rank"]] == [st["launches"]] * 2
    assert st["evals_per_s"] > 0 and "cpu_baseline" not in line
    # SURVEY §8(d) config 4 in the N > 1 line: RNEA + FD fp64 on shards of one global 2^20 batch,
    # both hipRTC kernels, its own budget, per-rank times
    c4 = line["secondary"]["strong_split_rnea_fd"]
    assert c4["kernel_path"] == "jit" and c4["dtype"] == "f64"
    assert c4["global_batch"] == bench.CONFIG4_BATCH and c4["batch_per_gpu_max"] == bench.CONFIG4_BATCH // 2
    assert c4["launches"] >= bench.SIDE_MIN_LAUNCHES and [x["steps"] for x in c4["per_rank"]] == [c4["launches"]] * 2
    assert c4["pairs_per_s"] > 0 and 0 < c4["hbm_frac_max_rank"] <= 1 and c4["graph_pairs_per_s"] > 0
    assert line["roofline_check"] == "ok", line["roofline_check"]


RCCL_WORKER = textwrap.dedent('''
    import os, sys, json
    sys.path[:0] = [{repo!r}, {pkg!r}]
    import numpy as np, torch, torch.distributed as dist
    from rigidbody_amd import chains, ffi
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)   # RCCL, as bench.py at world > 1
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    mb0 = ffi.Multibody.new()
    # the model broadcast of rigidbody_amd.dist.broadcast_model, on device tensors over RCCL
    blob = torch.as_tensor(mb0.blob(), dtype=torch.float64, device=dev)
    size = torch.tensor([blob.numel()], dtype=torch.int64, device=dev)
    dist.broadcast(size, 0)
    got = blob.clone()  # rank 0's buffer (the root of the broadcast)
    dist.broadcast(got, 0)
    mb = ffi.Multibody.from_blob(got.cpu().numpy())
    mb.upload()
    lim = mb.limits()
    x = [ffi.fill_uniform(torch.empty((7, 4099), dtype=torch.float64, device=dev), *chains.input_ranges(lim, k),
                          chains.SEED + i) for i, k in enumerate(("q", "qd", "qdd"))]
    same = bool(torch.equal(mb.rnea_batch(*x), mb0.rnea_batch(*x)))
    # the timing reductions of bench.py (max / gather over ranks) on device tensors
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    outs = [torch.zeros_like(t)]
    dist.all_gather(outs, t)
    dist.barrier()
    torch.cuda.synchronize()
    print(json.dumps({{"backend": dist.get_backend(), "blob_equal": bool(torch.equal(got, blob)),
                      "rebuilt_bit_identical": same, "max": t.tolist(), "gather": outs[0].tolist()}}), flush=True)
    dist.destroy_process_group()
''')


def test_rccl_process_group_world1(tmp_path):
    """The RCCL ("nccl") process group of bench.py's N > 1 path, initialised on the box's one GPU
    (RCCL takes one rank per device, so world 1 -- a 2-rank RCCL run needs two GPUs): the model
    blob broadcast on device tensors, the Multibody rebuilt from it bit-identical on a batch, and
    the max / gather reductions the timing uses."""
    script = tmp_path / "rccl.py"
    script.write_text(RCCL_WORKER.format(repo=REPO, pkg=PKG))
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-u", str(script)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["blob_equal"] and out["rebuilt_bit_identical"], out
    assert out["max"] == [1.5, 2.5] and out["gather"] == [1.5, 2.5], out
