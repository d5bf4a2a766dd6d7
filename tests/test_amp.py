"""AMP observation path: build_amp_observations_smpl (common.py:191-267), the
history buffer (humanoid_phc.py:1341-1350) and the reference-state history init
(humanoid_phc.py:791-838).

CPU tests pin the oracle to tests/golden/amp.npz (made by running the reference,
tools/gen_golden.py gen_amp). GPU tests run the engine's amp_kernel through the C ABI
(he_set_amp + the imitation launches) against the golden fixtures and the pinned oracle.

Tolerances: float32 reference vs float64 oracle / float32 kernel: 2e-5 absolute + 1e-5 relative
on every entry (tan-norms, heights, local positions and velocities); the history shift is a copy
and is compared exactly. The golden exp maps include the zero vector, a below-threshold (1e-7)
one, ~pi, >pi and >2pi (normalize_angle wrap) rows.
"""
import numpy as np
import pytest

from oracle import oracle as O

ATOL, RTOL = 2e-5, 1e-5


def _tables(g):
    return O.MotionTables(g["gts"], g["grs"], g["lrs"], g["gvs"], g["gavs"], g["dvs"], g["length_starts"],
                          g["num_frames"], g["motion_lengths"], g["motion_dt"])


def test_amp_layout(golden):
    g = golden("amp")
    joints, keys = O.amp_joints()
    # the reference's dof_subset is the 3 dofs of each kept joint
    np.testing.assert_array_equal(g["dof_subset"], (3 * joints[:, None] + np.arange(3)).reshape(-1))
    assert g["amp_obs"].shape[1] == 13 + 9 * len(joints) + 3 * len(keys) == 196
    assert g["amp_buf_in"].shape[1] * g["amp_obs"].shape[1] == 1960  # structs.py:42 amp_obs_size


def test_amp_obs_function(golden):
    g = golden("amp")
    r = O.amp_obs(g["root_pos"], g["root_rot"], g["root_vel"], g["root_ang_vel"], g["dof_pos"], g["dof_vel"],
                  g["key_pos"])
    np.testing.assert_allclose(r, g["amp_obs"], atol=ATOL, rtol=RTOL)


def test_amp_history_step(golden):
    g = golden("amp")
    r = O.amp_step(g["amp_buf_in"], g["env_rb_state"], g["env_dof_state"])
    np.testing.assert_array_equal(r[:, 1:], g["amp_buf_step"][:, 1:])  # the shift is a copy
    np.testing.assert_allclose(r[:, 0], g["amp_buf_step"][:, 0], atol=ATOL, rtol=RTOL)


def test_amp_reset_init(golden):
    g = golden("amp")
    mt = _tables(g)
    ids = g["reset_ids"]
    buf, demo = O.amp_init(g["amp_buf_step"], g["amp_demo_in"], ids, g["env_rb_state_reset"],
                           g["env_dof_state_reset"], mt, g["env_motion_ids"], g["reset_start_times"], 1 / 30)
    np.testing.assert_allclose(buf, g["amp_buf_reset"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(demo, g["amp_demo_reset"], atol=ATOL, rtol=RTOL)
    keep = np.setdiff1d(np.arange(buf.shape[0]), ids)
    np.testing.assert_array_equal(g["amp_demo_reset"][keep], g["amp_demo_in"][keep])


# ----------------------------------------------------------------------------- GPU (C ABI)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return torch


def _cu(torch, x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x), device="cuda:0")
    return t if dtype is None else t.to(dtype)


def _amp_engine(torch, he_model, g):
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.motion_lib import MotionTables
    n = g["env_rb_state"].shape[0]
    eng = Engine(he_model, n, device=0)
    eng.load_motions(MotionTables(gts=g["gts"], grs=g["grs"], lrs=g["lrs"], gvs=g["gvs"], gavs=g["gavs"],
                                  dvs=g["dvs"], num_frames=g["num_frames"], length_starts=g["length_starts"],
                                  lengths=g["motion_lengths"], dt=g["motion_dt"], fps=1.0 / g["motion_dt"]))
    eng.rb_state.copy_(_cu(torch, g["env_rb_state"].reshape(n * 24, 13)))
    eng.dof_state.copy_(_cu(torch, g["env_dof_state"].reshape(n * 69, 2)))
    em = eng.env_motion(_cu(torch, g["env_motion_ids"], torch.int64), _cu(torch, g["env_start_times"]),
                        torch.zeros(n, device="cuda:0"), _cu(torch, g["env_global_offset"]),
                        _cu(torch, g["env_progress"], torch.int16))
    outs = dict(obs=torch.zeros(n, 934, device="cuda:0"), rew=torch.zeros(n, device="cuda:0"),
                reward_raw=torch.zeros(n, 5, device="cuda:0"),
                reset=torch.zeros(n, dtype=torch.uint8, device="cuda:0"),
                terminate=torch.zeros(n, dtype=torch.uint8, device="cuda:0"))
    return eng, em, outs, _abi.imitation_params()


@pytest.mark.gpu
def test_gpu_amp_function_matches_golden(golden):
    torch = _gpu()
    from humanoid_amd.engine import amp_observations
    g = golden("amp")
    ins = [_cu(torch, g[k]) for k in ("root_pos", "root_rot", "root_vel", "root_ang_vel", "dof_pos", "dof_vel",
                                      "key_pos")]
    r = amp_observations(*ins)
    torch.cuda.synchronize()
    np.testing.assert_allclose(r.cpu().numpy(), g["amp_obs"], atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_gpu_amp_step_and_reset_match_golden(he_model, golden):
    """he_imitation_step then he_reset_envs with AMP attached = the reference's step tail and
    _init_amp_obs (tools/gen_golden.py gen_amp)."""
    torch = _gpu()
    g = golden("amp")
    eng, em, o, p = _amp_engine(torch, he_model, g)
    buf = _cu(torch, g["amp_buf_in"])
    demo = _cu(torch, g["amp_demo_in"])
    eng.set_amp(buf, demo)
    eng.imitation_step(p, em, o["obs"], o["rew"], o["reward_raw"], o["reset"], o["terminate"])
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    np.testing.assert_array_equal(got[:, 1:], g["amp_buf_step"][:, 1:])
    np.testing.assert_allclose(got[:, 0], g["amp_buf_step"][:, 0], atol=ATOL, rtol=RTOL)
    np.testing.assert_array_equal(demo.cpu().numpy(), g["amp_demo_in"])  # untouched by a step
    buf.copy_(_cu(torch, g["amp_buf_step"]))  # continue from the reference's buffer
    ids = _cu(torch, g["reset_ids"], torch.int32)
    eng.reset_envs(p, em, ids, _cu(torch, g["reset_phases"]), o["obs"], o["reset"], o["terminate"])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(em.keep_alive[1].cpu().numpy(), g["reset_start_times"])
    np.testing.assert_allclose(buf.cpu().numpy(), g["amp_buf_reset"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(demo.cpu().numpy(), g["amp_demo_reset"], atol=ATOL, rtol=RTOL)
    eng.set_amp(None)  # detached: the next step leaves the buffers alone
    before = buf.clone()
    eng.imitation_step(p, em, o["obs"], o["rew"], o["reward_raw"], o["reset"], o["terminate"])
    torch.cuda.synchronize()
    assert torch.equal(before, buf)


@pytest.mark.gpu
@pytest.mark.parametrize("steps", [10, 2, 1, 16])
def test_gpu_amp_fused_reset_matches_oracle(he_model, golden, steps):
    """he_imitation_reset_step (device resets): step update for envs that continue, history init for
    those reset in the launch; the oracle (pinned above) is composed on the engine's own post-reset
    state. steps=16 takes the chunked (not register) shift path."""
    torch = _gpu()
    g = golden("amp")
    n = g["env_rb_state"].shape[0]
    rng = np.random.default_rng(steps)
    start = g["env_start_times"].copy()
    forced = np.array([0, 4, 9, 13, 20])
    start[forced] = g["motion_lengths"][g["env_motion_ids"][forced]]  # pass_time -> reset
    g = dict(g, env_start_times=start)
    eng, em, o, p = _amp_engine(torch, he_model, g)
    buf_in = rng.normal(size=(n, steps, 196)).astype(np.float32)
    demo_in = rng.normal(size=(n, steps, 196)).astype(np.float32)
    buf, demo = _cu(torch, buf_in), _cu(torch, demo_in)
    eng.set_amp(buf, demo)
    rb0 = g["env_rb_state"]
    ds0 = g["env_dof_state"]
    eng.imitation_reset_step(p, em, o["obs"], o["rew"], o["reward_raw"], o["reset"], o["terminate"], seed=5,
                             step_index=3)
    torch.cuda.synchronize()
    reset = o["reset"].cpu().numpy().astype(bool)
    assert reset[forced].all()
    keep = ~reset
    rb1 = eng.rb_state.view(n, 24, 13).cpu().numpy()
    ds1 = eng.dof_state.view(n, 69, 2).cpu().numpy()
    np.testing.assert_array_equal(rb1[keep], rb0[keep])  # the physics state of continuing envs is untouched
    want = O.amp_step(buf_in, rb0, ds0)
    mt = O.MotionTables(g["gts"], g["grs"], g["lrs"], g["gvs"], g["gavs"], g["dvs"], g["length_starts"],
                        g["num_frames"], g["motion_lengths"], g["motion_dt"])
    ids = np.nonzero(reset)[0]
    want, want_demo = O.amp_init(want, demo_in, ids, rb1, ds1, mt, g["env_motion_ids"],
                                 em.keep_alive[1].cpu().numpy(), p.control_dt)
    got = buf.cpu().numpy()
    if steps > 1:
        np.testing.assert_array_equal(got[keep, 1:], want[keep, 1:])
    np.testing.assert_allclose(got, want, atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(demo.cpu().numpy(), want_demo, atol=ATOL, rtol=RTOL)
