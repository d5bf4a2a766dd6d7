"""Pin the CPU oracle to golden vectors produced by running the reference itself
(tools/gen_golden.py). CPU only.

Tolerances: the reference computes in float32 torch, the oracle in float64 (with the reference's
float32 frame-index arithmetic), so values agree to float32 rounding: 1e-5 absolute on unit-scale
quantities (quaternions, tan-norm, positions), 1e-4 relative on velocity-scale observations.
Quaternions are compared up to sign (q and -q are the same rotation; slerp's sign depends on
the frame pair chosen at exact frame boundaries).
"""
import numpy as np

import pytest

from humanoid_amd import _abi
from humanoid_amd.body_sets import EVAL_BODIES, body_ids
from oracle import oracle as O

import cases


def quat_close(a, b, atol):
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 4)
    d = np.minimum(np.abs(a - b).max(-1), np.abs(a + b).max(-1))
    assert d.max() <= atol, f"max quaternion diff {d.max()}"


def test_quat_prims(golden):
    g = golden("quat_prims")
    r = O.quat_prims(g["q"], g["r"], g["v"], g["e"], g["t"])
    np.testing.assert_allclose(r["mul"], g["quat_mul"], atol=2e-6)
    np.testing.assert_allclose(r["rot"], g["my_quat_rotate"], atol=1e-5)
    np.testing.assert_allclose(r["tan_norm"], g["quat_to_tan_norm"], atol=2e-6)
    # angle of quat_to_angle_axis: near |w|=1 float32 acos is ill-conditioned (~3e-4 rad), and at
    # w~0 the angle sits on the +-pi wrap, so compare modulo 2*pi
    wrap = np.angle(np.exp(1j * (r["angle"].astype(np.float64) - g["angle"])))
    assert np.abs(wrap).max() < 1e-3
    good = (np.abs(g["q"][:, 3]) < 0.999) & (np.abs(g["q"][:, 3]) > 1e-3)
    np.testing.assert_allclose(r["angle"][good], g["angle"][good], atol=2e-5)
    np.testing.assert_allclose(r["axis"][good], g["axis"][good], atol=2e-5)
    np.testing.assert_allclose(r["expmap"][good], g["quat_to_exp_map"][good], atol=2e-5)
    quat_close(r["exp2q"], g["exp_map_to_quat"], 2e-6)
    quat_close(r["slerp"], g["slerp"], 2e-5)
    np.testing.assert_allclose(r["heading"], g["calc_heading"], atol=2e-6)
    quat_close(r["hq"], g["calc_heading_quat"], 2e-6)
    quat_close(r["hqi"], g["calc_heading_quat_inv"], 2e-6)


def test_skeleton_matches_reference_tree(golden, model):
    g = golden("skeleton")
    assert list(g["node_names"]) == model.body_names
    np.testing.assert_array_equal(g["parents"], model.parents)
    np.testing.assert_allclose(g["local_translation"], model.local_pos, atol=1e-6)


def _tables(g):
    return O.MotionTables(g["gts"], g["grs"], g["lrs"], g["gvs"], g["gavs"], g["dvs"], g["length_starts"],
                          g["num_frames"], g["motion_lengths"], g["motion_dt"])


def test_motion_state(golden):
    g = golden("motion_lib")
    mt = _tables(g)
    r = O.motion_state(mt, g["q_ids"], g["q_times"], g["q_offset"])
    np.testing.assert_allclose(r["rg_pos"], g["ms_rg_pos"], atol=2e-6)
    np.testing.assert_allclose(r["body_vel"], g["ms_body_vel"], atol=1e-5)
    np.testing.assert_allclose(r["body_ang_vel"], g["ms_body_ang_vel"], atol=1e-5)
    np.testing.assert_allclose(r["dof_vel"], g["ms_dof_vel"], atol=1e-5)
    quat_close(r["rb_rot"], g["ms_rb_rot"], 5e-6)
    cases.assert_expmap_close(r["dof_pos"], g["ms_dof_pos"])
    np.testing.assert_allclose(r["rg_pos"][:, 0], g["ms_root_pos"], atol=2e-6)
    r0 = O.motion_state(mt, g["q_ids"], g["q_times"], None)
    np.testing.assert_allclose(r0["rg_pos"], g["msno_rg_pos"], atol=2e-6)


def test_sample_time_interval(golden):
    g = golden("motion_lib")
    lens = g["motion_lengths"][g["q_ids"]]
    got = np.array([O.sample_time_interval(p, l) for p, l in zip(g["phases"], lens)], np.float32)
    np.testing.assert_array_equal(got, g["sample_time_interval"])


def test_imitation_functions(golden):
    g = golden("imitation_funcs")
    p = _abi.imitation_params()
    r = O.imitation_from_ref(p, g["body_pos"], g["body_rot"], g["body_vel"], g["body_ang_vel"], g["ref_pos"],
                             g["ref_rot"], g["ref_vel"], g["ref_ang_vel"], g["progress"], g["pass_time"])
    np.testing.assert_allclose(r["rew"], g["rew"], atol=2e-5)
    np.testing.assert_allclose(r["reward_raw"], g["reward_raw"], atol=2e-5)
    np.testing.assert_array_equal(r["reset"], g["reset"])
    np.testing.assert_array_equal(r["terminate"], g["terminate"])
    np.testing.assert_allclose(r["self_obs"], g["self_obs"], atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(r["task_obs"], g["task_obs"], atol=2e-5, rtol=1e-5)
    pe = _abi.imitation_params(eval_mode=True, termination_distance=0.5, reset_body_ids=body_ids(EVAL_BODIES))
    re = O.imitation_from_ref(pe, g["body_pos"], g["body_rot"], g["body_vel"], g["body_ang_vel"], g["ref_pos"],
                              g["ref_rot"], g["ref_vel"], g["ref_ang_vel"], g["progress"], g["pass_time"])
    np.testing.assert_array_equal(re["reset"], g["reset_eval"])
    np.testing.assert_array_equal(re["terminate"], g["terminate_eval"])


def test_env_step_glue(golden):
    """HumanoidPHC.step post-physics half: reward -> reset -> obs (humanoid_phc.py:138-149)."""
    g = golden("env_step")
    mt = _tables(g)
    p = _abi.imitation_params()
    r = O.imitation_step(p, mt, g["rb_state"], g["dof_vel"], g["dof_force"], g["progress_in"], g["motion_ids"],
                         g["start_times"], g["start_offsets"], g["global_offset"])
    np.testing.assert_array_equal(r["progress"], g["progress_out"])
    np.testing.assert_allclose(r["rew"], g["rew"], atol=5e-5, rtol=1e-5)
    np.testing.assert_allclose(r["reward_raw"], g["reward_raw"], atol=5e-5, rtol=1e-5)
    np.testing.assert_array_equal(r["reset"], g["reset"])
    np.testing.assert_array_equal(r["terminate"], g["terminate"])
    np.testing.assert_allclose(r["obs"], g["obs"], atol=5e-5, rtol=1e-5)
    pe = _abi.imitation_params(eval_mode=True, termination_distance=0.5, reset_body_ids=body_ids(EVAL_BODIES))
    re = O.imitation_step(pe, mt, g["rb_state"], g["dof_vel"], g["dof_force"], g["progress_in"], g["motion_ids"],
                          g["start_times"], g["start_offsets"], g["global_offset"])
    np.testing.assert_array_equal(re["reset"], g["reset_eval"])
    np.testing.assert_array_equal(re["terminate"], g["terminate_eval"])


def test_env_reset_glue(golden):
    """_reset_ref_state_init + _compute_observations(env_ids) (humanoid_phc.py:665-731, 901-961)."""
    g = golden("env_reset")
    s = golden("env_step")
    mt = _tables(s)
    n = g["root_states"].shape[0]
    st = dict(start_times=np.zeros(n, np.float32), start_offsets=np.zeros(n, np.float32),
              global_offset=np.ascontiguousarray(g["global_offset_in"], np.float32),
              progress=np.full(n, 7, np.int16), root_states=np.zeros((n, 13), np.float32),
              dof_state=np.zeros((n, 69, 2), np.float32), dof_targets=np.zeros((n, 69), np.float32),
              rb_state=np.ascontiguousarray(g["rb_state_in"], np.float32), contact_forces=np.ones((n, 24, 3), np.float32),
              obs=np.zeros((n, 934), np.float32), reset=np.ones(n, np.uint8), terminate=np.ones(n, np.uint8))
    ids = g["env_ids"]
    O.reset_envs(_abi.imitation_params(), mt, ids, g["phases"], np.arange(n), st)
    np.testing.assert_array_equal(st["start_times"][ids], g["start_times"][ids])
    np.testing.assert_allclose(st["global_offset"], g["global_offset"], atol=0)
    rs, gr = st["root_states"][ids], g["root_states"][ids]
    np.testing.assert_allclose(rs[:, :3], gr[:, :3], atol=2e-6)
    quat_close(rs[:, 3:7], gr[:, 3:7], 5e-6)
    np.testing.assert_allclose(rs[:, 7:], gr[:, 7:], atol=1e-5)
    cases.assert_expmap_close(st["dof_state"][ids, :, 0], g["dof_pos"][ids])
    np.testing.assert_allclose(st["dof_state"][ids, :, 1], g["dof_vel"][ids], atol=1e-5)
    cases.assert_expmap_close(st["dof_targets"][ids], g["dof_pos"][ids])
    rb, grb = st["rb_state"][ids], g["rb_state"][ids]
    np.testing.assert_allclose(rb[..., :3], grb[..., :3], atol=2e-6)
    quat_close(rb[..., 3:7], grb[..., 3:7], 5e-6)
    np.testing.assert_allclose(rb[..., 7:], grb[..., 7:], atol=1e-5)
    np.testing.assert_allclose(st["obs"][ids], g["obs"][ids], atol=5e-5, rtol=1e-5)
    assert (st["progress"][ids] == 0).all() and (st["contact_forces"][ids] == 0).all()
    others = np.setdiff1d(np.arange(n), ids)
    assert (st["progress"][others] == 7).all()


@pytest.mark.parametrize("kind", ["Default", "Start", "Hybrid"])
def test_state_init_kinds_match_reference(golden, model, kind):
    """StateInit Default / Start / Hybrid (humanoid_phc.py:679-745, 747-780, 937-961) against the
    reference's own _reset_actors run (tests/golden/state_init.npz, tools/gen_golden.py). Hybrid's
    Bernoulli mask and phases come from the fixture: u = phase * p for a reference init, u >= p for
    a Default one (p = 0.5: u / p exact). Default envs' rb rows are the engine's decision (the zero
    pose's rows); the fixture made them with poselib's FK, so the rows and the obs read from them
    are compared too."""
    g = golden("state_init")
    s = golden("env_step")
    np.testing.assert_array_equal(g["motion_lengths"], s["motion_lengths"])
    mt = _tables(s)
    n = 24
    c = lambda x, t=np.float32: np.ascontiguousarray(x, t)  # noqa: E731
    st = dict(start_times=c(g["start_times_in"]), start_offsets=c(g["start_offsets_in"]),
              global_offset=c(g["global_offset_in"]), progress=c(g["progress_in"], np.int16),
              root_states=c(g["root_in"]), dof_state=c(g["dof_in"]), dof_targets=np.zeros((n, 69), np.float32),
              rb_state=c(g["rb_in"]), contact_forces=np.ones((n, 24, 3), np.float32),
              obs=np.zeros((n, 934), np.float32), reset=np.ones(n, np.uint8), terminate=np.ones(n, np.uint8),
              init_root=c(g["init_root"]))
    k = kind.lower()
    ids = g["env_ids"]
    mask, ph = g[k + "_ref_mask"], g[k + "_phases"]
    if kind == "Hybrid":
        assert mask.any() and not mask.all()
        u = np.where(mask, ph * np.float32(0.5), np.float32(0.75)).astype(np.float32)
    else:
        u = np.full(len(ids), 0.3, np.float32)
    p = _abi.imitation_params(state_init=kind, hybrid_init_prob=0.5)
    O.reset_envs(p, mt, ids, u, g["motion_ids"], st, rest_pos=O.rest_positions(model))
    rs, gr = st["root_states"][ids], g[k + "_root"][ids]
    np.testing.assert_allclose(rs[:, :3], gr[:, :3], atol=2e-6)
    quat_close(rs[:, 3:7], gr[:, 3:7], 5e-6)
    np.testing.assert_allclose(rs[:, 7:], gr[:, 7:], atol=1e-5)
    cases.assert_expmap_close(st["dof_state"][ids, :, 0], g[k + "_dof"][ids, :, 0])
    np.testing.assert_allclose(st["dof_state"][ids, :, 1], g[k + "_dof"][ids, :, 1], atol=1e-5)
    cases.assert_expmap_close(st["dof_targets"][ids], g[k + "_dof"][ids, :, 0])
    rb, grb = st["rb_state"][ids], g[k + "_rb"][ids]
    np.testing.assert_allclose(rb[..., :3], grb[..., :3], atol=2e-6)
    quat_close(rb[..., 3:7], grb[..., 3:7], 5e-6)
    np.testing.assert_allclose(rb[..., 7:], grb[..., 7:], atol=1e-5)
    np.testing.assert_array_equal(st["start_times"], g[k + "_start_times"])
    np.testing.assert_array_equal(st["start_offsets"], g[k + "_start_offsets"])
    np.testing.assert_array_equal(st["global_offset"], g[k + "_global_offset"])
    np.testing.assert_array_equal(st["progress"], g[k + "_progress"])
    assert (st["contact_forces"][ids] == 0).all()
    np.testing.assert_allclose(st["obs"][ids], g[k + "_obs"][ids], atol=5e-5, rtol=1e-5)


def test_host_motion_loader_matches_reference(golden, model):
    from humanoid_amd.motion_lib import build_tables
    g = golden("motion_lib")
    clips = [dict(pose_quat_global=g[f"clip{i}_pose_quat_global"], root_trans_offset=g[f"clip{i}_root_trans_offset"],
                  fps=int(g[f"clip{i}_fps"])) for i in range(5)]
    t = build_tables(model, [clips[i] for i in g["sample_idxes"]])
    np.testing.assert_allclose(t.gts, g["gts"], atol=2e-6)
    np.testing.assert_allclose(t.grs, g["grs"], atol=0)
    np.testing.assert_allclose(t.lrs, g["lrs"], atol=1e-6)
    np.testing.assert_allclose(t.gvs, g["gvs"], atol=5e-5)
    # float32 arccos near 1 in poselib's angular velocity is ill-conditioned (~1e-3 rad/s)
    np.testing.assert_allclose(t.gavs, g["gavs"], atol=3e-3)
    np.testing.assert_allclose(t.dvs, g["dvs"], atol=5e-4)
    np.testing.assert_array_equal(t.length_starts, g["length_starts"])
    np.testing.assert_array_equal(t.num_frames, g["num_frames"])
    np.testing.assert_array_equal(t.lengths, g["motion_lengths"])
    np.testing.assert_array_equal(t.dt, g["motion_dt"])


def test_pd_targets(golden, model):
    from humanoid_amd.model import pd_action_offset_scale
    from humanoid_amd.body_sets import frozen_dof_mask
    g = golden("pd_targets")
    off, sc = pd_action_offset_scale(model)
    np.testing.assert_array_equal(off, g["offset"])
    np.testing.assert_array_equal(sc, g["scale"])
    mask = np.array(frozen_dof_mask(), bool)
    pd = off + sc * g["actions"]
    pd[:, mask] = 0
    np.testing.assert_array_equal(pd.astype(np.float32), g["pd_target"])
