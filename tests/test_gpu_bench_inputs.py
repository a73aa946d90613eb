"""The bench's timed workloads run on valid inputs.  bench.rollout_launcher updates q, qd in
place; without its per-launch reset the state integrated launch after launch diverges to Inf /
NaN (tools/roll_state.py: 95% of FR3 configurations within 200 launches of 16 steps), and the
rollout lines would time a diverged state.  With the reset every launch must leave the same,
finite state, equal to one rollout of the initial draw."""
import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("B", [1 << 16, 1 << 20])
def test_rollout_launcher_resets_state(dtype, B):
    import sys

    sys.path[:0] = [REPO, PKG]
    import bench
    from rigidbody_amd import ffi

    dt = bench.DT[dtype]
    mb = ffi.Multibody.new()
    mb.upload()
    rl = bench.rollout_launcher(mb, B, dt, 16)
    q, qd, tau, init = rl.keep
    rl(0, None)
    torch.cuda.synchronize()
    first = torch.stack([q, qd]).clone()
    assert torch.isfinite(first).all(), "one 16-step rollout of the bench draw left a non-finite state"
    # the same rollout through the plain binding, from the initial draw
    q1, qd1 = init[0].clone(), init[1].clone()
    mb.rollout_batch(q1, qd1, tau.view(16, mb.n, B), 1e-3)
    torch.cuda.synchronize()
    assert torch.equal(first, torch.stack([q1, qd1]))
    for i in range(1, 40):
        rl(i, None)
    torch.cuda.synchronize()
    assert torch.equal(first, torch.stack([q, qd])), "the launches do not restart from the initial state"
    # reset_only issues the copy alone
    ro = bench.rollout_launcher(mb, B, dt, 16, reset_only=True)
    ro(0, None)
    torch.cuda.synchronize()
    assert torch.equal(torch.stack(ro.keep[:2]), ro.keep[3])
