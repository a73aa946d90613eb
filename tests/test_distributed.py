"""Multi-process path on CPU (gloo, world_size 2): the model blob broadcast, per-rank
input streams, strong-scaling shard ranges and max-over-ranks timing, exactly as
bench.py uses them with the nccl (RCCL) backend on GPUs.  No GPU work here."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from conftest import PKG, REPO


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
    dev = torch.device("cpu")
    mb = rdist.broadcast_model(lambda: ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(12)),
                               rank, world, dev)
    blob = mb.blob()
    ref = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(12)).blob()
    assert np.array_equal(blob, ref), "blob differs after broadcast"
    lim = mb.limits()
    lo, hi = chains.input_ranges(lim, "q")
    x = chains.host_uniform(mb.n, 1000, lo, hi, rdist.rank_seed(chains.SEED, rank))
    sums = rdist.gather_checksums(x, world, dev)
    mx = rdist.max_over_ranks([float(rank + 1), 10.0 - rank], world, dev)
    tot = rdist.sum_over_ranks([1.0], world, dev)
    sl = [rdist.shard(1 << 20, r, world) for r in range(world)]
    # dynamics per rank: the strong split of one global batch of 96 configurations, each rank
    # evaluating its shard through the single-configuration ABI (host lane bodies, no GPU here),
    # gathered to rank 0 and checked there against the oracle on the whole batch
    G = 96
    xs = [chains.host_uniform(mb.n, G, *chains.input_ranges(lim, k), chains.SEED + i)
          for i, k in enumerate(("q", "qd", "qdd"))]
    b0, b1 = rdist.shard(G, rank, world)
    mine = np.stack([mb.rnea(xs[0][:, b], xs[1][:, b], xs[2][:, b]) for b in range(b0, b1)], axis=1)
    parts = [None] * world
    dist.all_gather_object(parts, (b0, b1, mine.tolist()))
    err = None
    if rank == 0:
        from oracle import oracle, urdf_model
        om = oracle.Model(urdf_model.model_raw_from_urdf(chains.synthetic_chain_urdf(12)))
        tau = np.zeros((mb.n, G))
        for p0, p1, v in parts:
            tau[:, p0:p1] = np.asarray(v)
        ref = om.rnea_batch(*xs)
        err = float((np.abs(tau - ref) / (1 + np.abs(ref))).max())
    if rank == 0:
        print(json.dumps({{"sums": sums, "max": mx, "tot": tot, "shards": sl, "n": mb.n, "rnea_err": err,
                          "covered": sorted((p[0], p[1]) for p in parts)}}))
    dist.destroy_process_group()
''')


@pytest.mark.parametrize("world", [2])
def test_gloo_model_broadcast_and_sharding(world, tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(repo=REPO, pkg=PKG))
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    import json

    res = json.loads(outs[0][0].strip().splitlines()[-1])
    assert res["n"] == 12
    assert len(res["sums"]) == world and res["sums"][0] != res["sums"][1]  # independent streams
    assert res["max"] == [float(world), 10.0]
    assert res["tot"] == [float(world)]
    sl = res["shards"]
    assert sl[0][0] == 0 and sl[-1][1] == 1 << 20
    assert all(sl[i][1] == sl[i + 1][0] for i in range(world - 1))
    cov = res["covered"]  # the ranks' shards of the 96-configuration batch tile it exactly
    assert cov[0][0] == 0 and cov[-1][1] == 96 and all(cov[i][1] == cov[i + 1][0] for i in range(world - 1))
    assert res["rnea_err"] <= 1e-12, res["rnea_err"]


def test_shard_ranges_cover_exactly():
    import sys as _s

    _s.path[:0] = [PKG]
    from rigidbody_amd import dist as rdist

    for total in (0, 1, 7, 1000, (1 << 20) + 3):
        for world in (1, 2, 3, 8):
            sl = [rdist.shard(total, r, world) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == total
            sizes = [b - a for a, b in sl]
            assert max(sizes) - min(sizes) <= 1
            assert all(sl[i][1] == sl[i + 1][0] for i in range(world - 1))
