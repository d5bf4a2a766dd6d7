"""Long horizons at full size (4096 envs) on the GPU: what a training run does for hours, compressed
to its failure modes. 20 s of simulated time under the tracking action stream of configs[2] (128
clips, device resets included) and 10 s of saturated random actions on the domain-randomised
terrain of configs[5] (mass / friction scales, slope and step fields): the state stays finite, no
joint angle reaches pi (the limit rows), the contact slots stay within capacity with every
overflow counted, rewards stay in the reference's range, bodies stay above the terrain, and
the episodes turn over (device resets happen and leave consistent bookkeeping)."""
import argparse
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch = pytest.importorskip("torch")

from humanoid_amd import _abi  # noqa: E402

pytestmark = pytest.mark.gpu


def _rollout(config, model, seed=0):
    import bench
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    args = argparse.Namespace(config=config, num_envs=4096, clips=128, seed=seed, max_contacts=40)
    return bench.Rollout(args, model, 0, 0)


def _check(ro, rew_max):
    n = ro.args.num_envs
    for t in (ro.eng.root_states, ro.eng.dof_state, ro.eng.rb_state, ro.obs, ro.rew):
        assert torch.isfinite(t).all()
    q = ro.eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3)
    assert q.norm(dim=-1).max().item() < np.pi
    assert (ro.eng.num_contacts <= _abi.MAX_CONTACTS).all() and (ro.eng.num_contacts >= 0).all()
    rows = ro.eng.contact_cache[:, 7].contiguous().view(torch.int32)  # solver rows of the last solve
    assert ((rows >= 0) & (rows <= _abi.MAX_ROWS)).all()
    assert (ro.eng.dropped_contacts >= 0).all()
    assert ro.rew.max().item() <= rew_max
    return q


def test_long_run_tracking_configs2(model):
    ro = _rollout("imitation", model)
    resets = 0
    for s in range(600):
        ro.tracking_actions()
        ro.step()
        resets += int(ro.reset.sum().item()) if s % 10 == 0 else 0
        if s % 50 == 49:
            torch.cuda.synchronize()
            _check(ro, rew_max=1.0 + 1e-6)  # sum of the weights (0.5 + 0.3 + 0.1 + 0.1), power term <= 0
            # the device resets keep the bookkeeping consistent: progress counts steps since the reset
            assert (ro.prog >= 0).all() and ro.prog.max().item() <= s + 1
            # nobody below the plane: the lowest body origin of every env
            z = ro.eng.rb_state.view(4096, 24, 13)[..., 2].min(dim=1).values
            assert z.min().item() > -0.1, z.min().item()
    assert resets > 0, "20 s over 5 s clips: episodes must turn over"


def test_long_run_saturated_actions_dr_terrain(model):
    """Saturated actions are the violent regime of DESIGN §5 (500 N m drives spin light links at the
    100 rad/s cap and bodies fly): asserted is what must hold even there -- finite state, no joint
    past the limit backstop, capacity, reward range, flat-plane envs above the plane."""
    ro = _rollout("dr", model, seed=3)
    rng = np.random.default_rng(5)
    worst = 0.0
    for s in range(300):
        ro.actions.copy_(torch.as_tensor(rng.uniform(-1.0, 1.0, (4096, 69)).astype(np.float32), device=ro.actions.device))
        ro.step()
        if s % 25 == 24:
            torch.cuda.synchronize()
            q = _check(ro, rew_max=1.0 + 1e-6)
            worst = max(worst, q.norm(dim=-1).max().item())
            # flat-plane envs (env % 3 == 0): every body origin above the plane
            z = ro.eng.rb_state.view(4096, 24, 13)[0::3, :, 2].min(dim=1).values
            assert z.min().item() > -0.1, z.min().item()
    assert worst < np.pi
