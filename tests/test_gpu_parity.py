"""GPU parity: the HIP engine (through its C ABI) against the golden fixtures and the CPU oracle.

Tolerances (float32 kernels vs the reference's float32 torch / the fp64 oracle):
* imitation outputs: 5e-5 abs (+1e-5 rel) on obs/reward, exact on reset/terminate/progress;
  quaternions up to sign within 5e-6 (the slerp is evaluated in torch's float32 order on both);
* physics (both solvers warm-start from their own caches): positions, joint angles and the centre of
  mass 1e-4 m / rad (BASELINE's 1e-4 rad/m), velocities 1e-2 abs + 1e-3 rel (PGS / LTDL in fp32 vs
  fp64 at joint speeds up to ~100 rad/s), over 1-30 policy steps. An element is widened to 4x the
  oracle's own sensitivity to a 1e-6 rad change of the initial joint angles only where that
  sensitivity exceeds the tolerance (see _cond_close), and each test bounds the share of widened
  elements (0-5%). Contact SETS are compared by key (body, partner, candidate) each step; envs
  whose sets differ (a point within rounding of the 0.02 m offset) are excluded, at most 2-5%.
"""
import numpy as np
import pytest

from humanoid_amd import _abi
from humanoid_amd.body_sets import EVAL_BODIES, body_ids
from oracle import oracle as O

import cases

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")


def quat_close(a, b, atol):
    a = np.asarray(a).reshape(-1, 4)
    b = np.asarray(b).reshape(-1, 4)
    d = np.minimum(np.abs(a - b).max(-1), np.abs(a + b).max(-1))
    assert d.max() <= atol, f"max quaternion diff {d.max()}"


def make_engine(he_model, n, **sim):
    from humanoid_amd.engine import Engine
    _require_gpu()
    return Engine(he_model, n, device=0, sim_params=_abi.default_sim_params(**sim))


def tables_from_golden(g):
    from humanoid_amd.motion_lib import MotionTables
    return MotionTables(gts=g["gts"], grs=g["grs"], lrs=g["lrs"], gvs=g["gvs"], gavs=g["gavs"], dvs=g["dvs"],
                        num_frames=g["num_frames"], length_starts=g["length_starts"], lengths=g["motion_lengths"],
                        dt=g["motion_dt"], fps=1.0 / g["motion_dt"])


def cu(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x), device="cuda:0")
    return t if dtype is None else t.to(dtype)


def test_zero_copy_buffers(he_model):
    eng = make_engine(he_model, 8)
    root = eng.root_states
    assert root.shape == (8, 13) and root.is_cuda
    assert eng.dof_state.shape == (8 * 69, 2)
    assert eng.rb_state.shape == (8 * 24, 13)
    assert eng.contact_forces.shape == (8 * 24, 3)
    assert eng.dof_force.shape == (8 * 69,)
    torch.cuda.synchronize()
    r = root.cpu().numpy()
    np.testing.assert_allclose(r[:, 2], 0.89)
    np.testing.assert_allclose(r[:, 6], 1.0)
    # indexed writes from a separate full-size source
    src = torch.zeros(8, 13, device="cuda:0")
    src[:, 2] = 2.5
    ids = torch.tensor([1, 5], dtype=torch.int32, device="cuda:0")
    eng.set_root_state_indexed(src, ids)
    torch.cuda.synchronize()
    z = eng.root_states[:, 2].cpu().numpy()
    assert z[1] == 2.5 and z[5] == 2.5 and z[0] == np.float32(0.89)
    with pytest.raises(Exception):
        eng.set_root_state_indexed(src[:, :12], ids)


def test_product_library_has_no_phase_stamps(he_model):
    """The per-phase cycle stamps live only in the diagnostic twin (libhumanoid_engine_phases.so);
    the product library refuses a stamp buffer instead of silently leaving it zero."""
    import os
    from humanoid_amd.engine import EngineError
    if os.environ.get("HE_ENGINE_LIB"):
        pytest.skip("a variant library is loaded")
    eng = make_engine(he_model, 8)
    buf = torch.zeros(8, 32, dtype=torch.int64, device="cuda:0")
    with pytest.raises(EngineError, match="phase stamps"):
        eng.set_debug_stamps(buf)
    eng.set_debug_stamps(None)


def test_motion_state_matches_golden(he_model, golden):
    g = golden("motion_lib")
    eng = make_engine(he_model, 4)
    eng.load_motions(tables_from_golden(g))
    r = eng.motion_state(cu(g["q_ids"], torch.int64), cu(g["q_times"]), cu(g["q_offset"]))
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in r.items()}
    np.testing.assert_allclose(r["rg_pos"], g["ms_rg_pos"], atol=2e-6)
    np.testing.assert_allclose(r["body_vel"], g["ms_body_vel"], atol=1e-5)
    np.testing.assert_allclose(r["body_ang_vel"], g["ms_body_ang_vel"], atol=1e-5)
    np.testing.assert_allclose(r["dof_vel"], g["ms_dof_vel"], atol=1e-5)
    quat_close(r["rb_rot"], g["ms_rb_rot"], 5e-6)
    cases.assert_expmap_close(r["dof_pos"], g["ms_dof_pos"])


def _load_env_state(eng, g):
    n = g["rb_state"].shape[0]
    eng.rb_state.copy_(cu(g["rb_state"].reshape(n * 24, 13)))
    ds = eng.dof_state.view(n, 69, 2)
    ds[..., 1] = cu(g["dof_vel"])
    eng.dof_force.copy_(cu(g["dof_force"].reshape(-1)))


def test_motion_reload_invalidates_metadata_cache(he_model, golden):
    """The imitation kernel keeps each env's motion metadata (length, dt, frame count, start) from its
    last step, keyed by the motion id (he_engine meta cache). A motion-table reload must not reuse
    it: after a step on the golden tables, a reload with the motions' order reversed (same ids, other
    clips), then a step, equals that step on a fresh engine that only ever saw the reversed tables."""
    from humanoid_amd.motion_lib import MotionTables
    g = golden("env_step")
    n = g["rb_state"].shape[0]
    t = tables_from_golden(g)
    M = len(t.num_frames)
    if M < 2:
        pytest.skip("the golden env step has one motion")
    rev = np.arange(M)[::-1]
    lens, starts = np.asarray(t.num_frames), np.asarray(t.length_starts)
    order = np.concatenate([np.arange(starts[m], starts[m] + lens[m]) for m in rev])
    F = lambda x: np.asarray(x)[order]  # noqa: E731
    t2 = MotionTables(gts=F(t.gts), grs=F(t.grs), lrs=F(t.lrs), gvs=F(t.gvs), gavs=F(t.gavs), dvs=F(t.dvs),
                      num_frames=lens[rev], length_starts=np.concatenate([[0], np.cumsum(lens[rev])[:-1]]),
                      lengths=np.asarray(t.lengths)[rev], dt=np.asarray(t.dt)[rev], fps=np.asarray(t.fps)[rev])

    def step(eng):
        _load_env_state(eng, g)
        em = eng.env_motion(cu(g["motion_ids"], torch.int64), cu(g["start_times"]), cu(g["start_offsets"]),
                            cu(g["global_offset"]), cu(g["progress_in"], torch.int16))
        out = [torch.zeros(n, 934, device="cuda:0"), torch.zeros(n, device="cuda:0"), torch.zeros(n, 5, device="cuda:0"),
               torch.zeros(n, dtype=torch.uint8, device="cuda:0"), torch.zeros(n, dtype=torch.uint8, device="cuda:0")]
        eng.imitation_step(_abi.imitation_params(), em, *out)
        torch.cuda.synchronize()
        return [o.cpu().numpy() for o in out]

    e1 = make_engine(he_model, n)
    e1.load_motions(t)
    step(e1)
    e1.load_motions(t2)
    got = step(e1)
    e2 = make_engine(he_model, n)
    e2.load_motions(t2)
    want = step(e2)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


def test_imitation_step_matches_golden_and_oracle(he_model, golden):
    g = golden("env_step")
    n = g["rb_state"].shape[0]
    eng = make_engine(he_model, n)
    eng.load_motions(tables_from_golden(g))
    _load_env_state(eng, g)
    mids = cu(g["motion_ids"], torch.int64)
    st, so = cu(g["start_times"]), cu(g["start_offsets"])
    go, prog = cu(g["global_offset"]), cu(g["progress_in"], torch.int16)
    em = eng.env_motion(mids, st, so, go, prog)
    obs = torch.zeros(n, 934, device="cuda:0")
    rew = torch.zeros(n, device="cuda:0")
    raw = torch.zeros(n, 5, device="cuda:0")
    reset = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    term = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    eng.imitation_step(_abi.imitation_params(), em, obs, rew, raw, reset, term)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(prog.cpu().numpy(), g["progress_out"])
    np.testing.assert_allclose(rew.cpu().numpy(), g["rew"], atol=5e-5, rtol=1e-5)
    np.testing.assert_allclose(raw.cpu().numpy(), g["reward_raw"], atol=5e-5, rtol=1e-5)
    np.testing.assert_array_equal(reset.cpu().numpy(), g["reset"])
    np.testing.assert_array_equal(term.cpu().numpy(), g["terminate"])
    np.testing.assert_allclose(obs.cpu().numpy(), g["obs"], atol=5e-5, rtol=1e-5)
    # eval-mode termination
    prog.copy_(cu(g["progress_in"], torch.int16))
    pe = _abi.imitation_params(eval_mode=True, termination_distance=0.5, reset_body_ids=body_ids(EVAL_BODIES))
    eng.imitation_step(pe, em, obs, rew, raw, reset, term)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(reset.cpu().numpy(), g["reset_eval"])
    np.testing.assert_array_equal(term.cpu().numpy(), g["terminate_eval"])


@pytest.mark.parametrize("n", [65, 4097])
def test_imitation_step_ragged_launch_equals_golden_run(he_model, golden, n):
    """The imitation kernel packs two envs per wave and eight per 256-lane block: a launch of 65 or
    4,097 envs ends in a partial block and a half-filled wave. Env i of such a launch gets the golden
    fixture's env i mod n_g (state, motion, time, progress) and must produce exactly the golden run's
    outputs for that env (obs, reward, raw terms, reset / terminate, progress), bit for bit."""
    g = golden("env_step")
    ng = g["rb_state"].shape[0]

    def run(idx):
        m = len(idx)
        eng = make_engine(he_model, m)
        eng.load_motions(tables_from_golden(g))
        eng.rb_state.copy_(cu(g["rb_state"][idx].reshape(m * 24, 13)))
        eng.dof_state.view(m, 69, 2)[..., 1] = cu(g["dof_vel"][idx])
        eng.dof_force.copy_(cu(g["dof_force"][idx].reshape(-1)))
        prog = cu(g["progress_in"][idx], torch.int16)
        em = eng.env_motion(cu(g["motion_ids"][idx], torch.int64), cu(g["start_times"][idx]),
                            cu(g["start_offsets"][idx]), cu(g["global_offset"][idx]), prog)
        out = [torch.zeros(m, 934, device="cuda:0"), torch.zeros(m, device="cuda:0"), torch.zeros(m, 5, device="cuda:0"),
               torch.zeros(m, dtype=torch.uint8, device="cuda:0"), torch.zeros(m, dtype=torch.uint8, device="cuda:0")]
        eng.imitation_step(_abi.imitation_params(), em, *out)
        torch.cuda.synchronize()
        res = [o.cpu().numpy() for o in out] + [prog.cpu().numpy()]
        del eng
        return res

    ref = run(np.arange(ng))
    idx = np.arange(n) % ng
    got = run(idx)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b[idx])


def test_reset_envs_matches_golden(he_model, golden):
    g = golden("env_reset")
    s = golden("env_step")
    n = g["root_states"].shape[0]
    eng = make_engine(he_model, n)
    eng.load_motions(tables_from_golden(s))
    eng.rb_state.copy_(cu(g["rb_state_in"].reshape(n * 24, 13)))
    mids = torch.arange(n, device="cuda:0", dtype=torch.int64)
    st = torch.zeros(n, device="cuda:0")
    so = torch.zeros(n, device="cuda:0")
    go = cu(g["global_offset_in"])
    prog = torch.full((n,), 7, dtype=torch.int16, device="cuda:0")
    em = eng.env_motion(mids, st, so, go, prog)
    obs = torch.zeros(n, 934, device="cuda:0")
    reset = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    term = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    ids = cu(g["env_ids"], torch.int32)
    eng.reset_envs(_abi.imitation_params(), em, ids, cu(g["phases"]), obs, reset, term)
    torch.cuda.synchronize()
    I = g["env_ids"]
    np.testing.assert_array_equal(st.cpu().numpy()[I], g["start_times"][I])
    np.testing.assert_array_equal(go.cpu().numpy(), g["global_offset"])
    rs = eng.root_states.cpu().numpy()[I]
    gr = g["root_states"][I]
    np.testing.assert_allclose(rs[:, :3], gr[:, :3], atol=2e-6)
    quat_close(rs[:, 3:7], gr[:, 3:7], 5e-6)
    np.testing.assert_allclose(rs[:, 7:], gr[:, 7:], atol=1e-5)
    ds = eng.dof_state.view(n, 69, 2).cpu().numpy()[I]
    cases.assert_expmap_close(ds[..., 0], g["dof_pos"][I])
    np.testing.assert_allclose(ds[..., 1], g["dof_vel"][I], atol=1e-5)
    cases.assert_expmap_close(eng.dof_targets.cpu().numpy()[I], g["dof_pos"][I])
    rb = eng.rb_state.view(n, 24, 13).cpu().numpy()[I]
    grb = g["rb_state"][I]
    np.testing.assert_allclose(rb[..., :3], grb[..., :3], atol=2e-6)
    quat_close(rb[..., 3:7], grb[..., 3:7], 5e-6)
    np.testing.assert_allclose(rb[..., 7:], grb[..., 7:], atol=1e-5)
    np.testing.assert_allclose(obs.cpu().numpy()[I], g["obs"][I], atol=5e-5, rtol=1e-5)
    p = prog.cpu().numpy()
    assert (p[I] == 0).all() and (p[np.setdiff1d(np.arange(n), I)] == 7).all()
    assert (reset.cpu().numpy()[I] == 0).all()


def _state_init_case(he_model, model, golden, n=24):
    """An engine over the env_step golden motions, the envs advanced 3 policy steps under random
    actions, and the oracle state dict mirroring the engine's (init_root included)."""
    from humanoid_amd.model import pd_action_offset_scale
    g = golden("env_step")
    eng = make_engine(he_model, n)
    tables = tables_from_golden(g)
    eng.load_motions(tables)
    off, sc = pd_action_offset_scale(model)
    eng.set_pd_params(off, sc, None)
    rng = np.random.default_rng(40)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    eng.root_states.copy_(cu(root))
    # the initial root states as the reference keeps them: the creation pose, zero velocity
    init = root.copy()
    init[:, 7:] = 0.0
    eng.initial_root_states.copy_(cu(init))
    st = cu(g["start_times"]); so = torch.zeros(n, device="cuda:0"); go = cu(g["global_offset"])
    prog = torch.zeros(n, dtype=torch.int16, device="cuda:0")
    em = eng.env_motion(torch.arange(n, device="cuda:0"), st, so, go, prog)
    for _ in range(3):
        eng.step_actions(cu(rng.uniform(-0.3, 0.3, (n, 69)).astype(np.float32)), 2)
    torch.cuda.synchronize()
    return eng, em, (st, so, go, prog), O.MotionTables.from_tables(tables), init


def _oracle_state(eng, bk, n, init):
    st, so, go, prog = bk
    return dict(start_times=st.cpu().numpy().copy(), start_offsets=so.cpu().numpy().copy(),
                global_offset=go.cpu().numpy().copy(), progress=prog.cpu().numpy().copy(),
                root_states=eng.root_states.cpu().numpy().copy(), dof_state=eng.dof_state.view(n, 69, 2).cpu().numpy().copy(),
                dof_targets=eng.dof_targets.cpu().numpy().copy(), rb_state=eng.rb_state.view(n, 24, 13).cpu().numpy().copy(),
                contact_forces=eng.contact_forces.view(n, 24, 3).cpu().numpy().copy(),
                obs=np.zeros((n, 934), np.float32), reset=np.zeros(n, np.uint8), terminate=np.zeros(n, np.uint8),
                init_root=init)


def _assert_reset_rows(eng, bk, st_o, ids, n, obs):
    st, so, go, prog = bk
    rs = eng.root_states.cpu().numpy()[ids]
    np.testing.assert_allclose(rs[:, :3], st_o["root_states"][ids, :3], atol=2e-6)
    quat_close(rs[:, 3:7], st_o["root_states"][ids, 3:7], 5e-6)
    np.testing.assert_allclose(rs[:, 7:], st_o["root_states"][ids, 7:], atol=1e-5)
    ds = eng.dof_state.view(n, 69, 2).cpu().numpy()[ids]
    cases.assert_expmap_close(ds[..., 0], st_o["dof_state"][ids, :, 0])
    np.testing.assert_allclose(ds[..., 1], st_o["dof_state"][ids, :, 1], atol=1e-5)
    cases.assert_expmap_close(eng.dof_targets.cpu().numpy()[ids], st_o["dof_targets"][ids])
    rb = eng.rb_state.view(n, 24, 13).cpu().numpy()[ids]
    np.testing.assert_allclose(rb[..., :3], st_o["rb_state"][ids, :, :3], atol=2e-6)
    quat_close(rb[..., 3:7], st_o["rb_state"][ids, :, 3:7], 5e-6)
    np.testing.assert_allclose(rb[..., 7:], st_o["rb_state"][ids, :, 7:], atol=1e-5)
    np.testing.assert_array_equal(st.cpu().numpy(), st_o["start_times"])
    np.testing.assert_array_equal(so.cpu().numpy(), st_o["start_offsets"])
    np.testing.assert_array_equal(go.cpu().numpy(), st_o["global_offset"])
    np.testing.assert_array_equal(prog.cpu().numpy()[ids], 0)
    assert (eng.contact_forces.view(n, 24, 3).cpu().numpy()[ids] == 0).all()
    og, oo = obs.cpu().numpy()[ids], st_o["obs"][ids]
    np.testing.assert_allclose(og, oo, atol=5e-5, rtol=1e-5)


@pytest.mark.parametrize("state_init", ["Default", "Hybrid"])
def test_state_init_default_and_hybrid_match_oracle(he_model, model, golden, state_init):
    """StateInit.Default and .Hybrid (humanoid_phc.py:679-692, 733-745; config.py:114, 139) through
    he_reset_envs after 3 policy steps: Default writes the initial root state, zero dofs and targets,
    the zero pose's body rows and leaves the motion bookkeeping; Hybrid splits the envs by the draw
    u < hybrid_init_prob (reference init at phase u / p, else Default). Against the oracle's reset from
    the engine's own pre-reset state; both kinds occur in the Hybrid case.
    Self-consistency (engine vs the builder's oracle); reference parity of these kinds is
    test_state_init_matches_reference_golden."""
    n = 24
    eng, em, bk, mt, init = _state_init_case(he_model, model, golden, n)
    p = _abi.imitation_params(state_init=state_init, hybrid_init_prob=0.5)
    st_o = _oracle_state(eng, bk, n, init)
    ids = np.arange(0, n, 2).astype(np.int32)
    u = np.random.default_rng(41).uniform(0, 1, len(ids)).astype(np.float32)
    obs = torch.zeros(n, 934, device="cuda:0")
    reset = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    term = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    eng.reset_envs(p, em, cu(ids, torch.int32), cu(u), obs, reset, term)
    O.reset_envs(p, mt, ids, u, np.arange(n), st_o, rest_pos=O.rest_positions(model))
    torch.cuda.synchronize()
    _assert_reset_rows(eng, bk, st_o, ids, n, obs)
    dflt = ids[u >= 0.5] if state_init == "Hybrid" else ids
    assert len(dflt) > 0
    np.testing.assert_array_equal(eng.dof_state.view(n, 69, 2).cpu().numpy()[dflt], 0.0)
    if state_init == "Hybrid":
        assert 0 < len(dflt) < len(ids), "both kinds of reset must occur"


def test_state_init_hybrid_device_reset_matches_oracle(he_model, model, golden):
    """The device reset of he_imitation_reset_step (the env step's) under StateInit.Hybrid: the draw
    is the splitmix hash of (seed, step, env), resolved as in he_reset_envs. Envs are made to fail
    (bodies thrown off their reference), their reset rows checked against the oracle's reset with
    the same draws; AMP history rows of Default-reset envs equal their current row
    (_init_amp_obs_default, humanoid_phc.py:801-803).
    Self-consistency: the reference raises for Default + AMP (humanoid_phc.py:794-795)."""
    n = 24
    eng, em, bk, mt, init = _state_init_case(he_model, model, golden, n)
    S = 4
    amp = torch.zeros(n, S, 196, device="cuda:0")
    demo = torch.zeros(n, S, 196, device="cuda:0")
    eng.set_amp(amp, demo)
    p = _abi.imitation_params(state_init="Hybrid", hybrid_init_prob=0.5)
    # every env far from its reference: all terminate (progress > 1) and reset
    bk[3].fill_(5)
    eng.root_states[:, 2] += 1.0
    eng.simulate(1)
    torch.cuda.synchronize()
    rb = eng.rb_state.view(n, 24, 13).cpu().numpy().copy()
    st_o = _oracle_state(eng, bk, n, init)
    im = O.imitation_step(p, mt, rb, st_o["dof_state"][..., 1], eng.dof_force.view(n, 69).cpu().numpy(),
                          st_o["progress"], np.arange(n), st_o["start_times"], st_o["start_offsets"],
                          st_o["global_offset"])
    obs = torch.zeros(n, 934, device="cuda:0"); rew = torch.zeros(n, device="cuda:0")
    raw = torch.zeros(n, 5, device="cuda:0")
    reset = torch.zeros(n, dtype=torch.uint8, device="cuda:0"); term = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    seed, step = 99, 3
    eng.imitation_reset_step(p, em, obs, rew, raw, reset, term, seed=seed, step_index=step)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(reset.cpu().numpy(), im["reset"])
    ids = np.nonzero(im["reset"])[0].astype(np.int32)
    assert len(ids) == n
    st_o["progress"] = im["progress"]
    u = np.array([O.hash_uniform(seed, step, int(e)) for e in ids], np.float32)
    O.reset_envs(p, mt, ids, u, np.arange(n), st_o, rest_pos=O.rest_positions(model))
    _assert_reset_rows(eng, bk, st_o, ids, n, obs)
    dflt = ids[u >= 0.5]
    ref = ids[u < 0.5]
    assert len(dflt) > 0 and len(ref) > 0
    a = amp.cpu().numpy()
    for k in range(1, S):  # Default: the history is the current row
        np.testing.assert_array_equal(a[dflt, k], a[dflt, 0])
    assert not np.allclose(a[ref, 1], a[ref, 0])  # reference inits: rows from the motion


@pytest.mark.parametrize("kind", ["Default", "Start", "Hybrid"])
def test_state_init_matches_reference_golden(he_model, golden, kind):
    """StateInit Default / Start / Hybrid against the reference itself: tests/golden/state_init.npz
    holds HumanoidPHC._reset_actors (humanoid_phc.py:679-745) + the _reset_env_tensors bookkeeping +
    _compute_observations(env_ids), run by tools/gen_golden.py. Hybrid's torch.bernoulli mask and
    the reference inits' sample_time_interval phases are in the fixture; the engine's one draw per
    env u reproduces them (u = phase * p for a reference init, u >= p for a Default one; p = 0.5, so
    u / p is exact). Default envs' rb rows: the engine writes the zero pose's rows, and the fixture
    feeds the reference's observation the same rows made by poselib's FK (the
    Default-reset decision), so obs parity covers that choice's arithmetic, not the choice."""
    g = golden("state_init")
    s = golden("env_step")
    n = 24
    np.testing.assert_array_equal(g["motion_lengths"], s["motion_lengths"])  # one motion library
    eng = make_engine(he_model, n)
    eng.load_motions(tables_from_golden(s))
    eng.root_states.copy_(cu(g["root_in"]))
    eng.dof_state.copy_(cu(g["dof_in"].reshape(n * 69, 2)))
    eng.rb_state.copy_(cu(g["rb_in"].reshape(n * 24, 13)))
    eng.initial_root_states.copy_(cu(g["init_root"]))
    st, so, go = cu(g["start_times_in"]), cu(g["start_offsets_in"]), cu(g["global_offset_in"])
    prog = cu(g["progress_in"], torch.int16)
    em = eng.env_motion(cu(g["motion_ids"], torch.int64), st, so, go, prog)
    p = _abi.imitation_params(state_init=kind, hybrid_init_prob=0.5)
    k = kind.lower()
    ids = g["env_ids"].astype(np.int32)
    mask, ph = g[k + "_ref_mask"], g[k + "_phases"]
    if kind == "Hybrid":
        assert mask.any() and not mask.all()
        u = np.where(mask, ph * np.float32(0.5), np.float32(0.75)).astype(np.float32)
    else:
        u = np.full(len(ids), 0.3, np.float32)  # Start: t = 0; Default: no motion sample
    obs = torch.zeros(n, 934, device="cuda:0")
    reset = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    term = torch.ones(n, dtype=torch.uint8, device="cuda:0")
    eng.contact_forces.fill_(1.0)
    eng.reset_envs(p, em, cu(ids, torch.int32), cu(u), obs, reset, term)
    torch.cuda.synchronize()
    I = ids
    rs, gr = eng.root_states.cpu().numpy()[I], g[k + "_root"][I]
    np.testing.assert_allclose(rs[:, :3], gr[:, :3], atol=2e-6)
    quat_close(rs[:, 3:7], gr[:, 3:7], 5e-6)
    np.testing.assert_allclose(rs[:, 7:], gr[:, 7:], atol=1e-5)
    ds, gd = eng.dof_state.view(n, 69, 2).cpu().numpy()[I], g[k + "_dof"][I]
    cases.assert_expmap_close(ds[..., 0], gd[..., 0])
    np.testing.assert_allclose(ds[..., 1], gd[..., 1], atol=1e-5)
    cases.assert_expmap_close(eng.dof_targets.cpu().numpy()[I], gd[..., 0])  # set_dof_position_target (:763-767)
    rb, grb = eng.rb_state.view(n, 24, 13).cpu().numpy()[I], g[k + "_rb"][I]
    np.testing.assert_allclose(rb[..., :3], grb[..., :3], atol=2e-6)
    quat_close(rb[..., 3:7], grb[..., 3:7], 5e-6)
    np.testing.assert_allclose(rb[..., 7:], grb[..., 7:], atol=1e-5)
    np.testing.assert_array_equal(st.cpu().numpy(), g[k + "_start_times"])
    np.testing.assert_array_equal(so.cpu().numpy(), g[k + "_start_offsets"])
    np.testing.assert_array_equal(go.cpu().numpy(), g[k + "_global_offset"])
    np.testing.assert_array_equal(prog.cpu().numpy(), g[k + "_progress"])
    assert (eng.contact_forces.view(n, 24, 3).cpu().numpy()[I] == 0).all()
    assert (reset.cpu().numpy()[I] == 0).all() and (term.cpu().numpy()[I] == 0).all()
    np.testing.assert_allclose(obs.cpu().numpy()[I], g[k + "_obs"][I], atol=5e-5, rtol=1e-5)


class CondStats:
    """Counts the elements whose tolerance was widened (see _cond_close) over a whole test."""

    def __init__(self):
        self.widened = 0
        self.total = 0
        self.by_name = {}

    @property
    def frac(self):
        return self.widened / max(self.total, 1)


def _cond_close(name, g, o, s, atol, rtol=0.0, k=4.0, stats=None):
    """|gpu - oracle| <= atol + rtol*|oracle| elementwise, widened to + k * sens only for the
    elements whose oracle sensitivity `sens` exceeds atol.

    sens is the oracle's own change of that element when the initial joint angles move by 1e-6 rad
    (fp32 rounding level), the maximum over the probes `s` (independent perturbations). An element
    whose fp64 answer moves by more than the tolerance under rounding-level noise is ill-conditioned
    -- a toe resting on four box corners settles its yaw wherever friction holds it, a many-contact
    solve of a tumbling body is sensitive -- and no fp32 engine can match it tighter. Everything
    else gets the plain tolerance; `stats` counts the widened elements so that the caller bounds
    their share."""
    n = g.shape[0]
    probes = s if isinstance(s, (list, tuple)) else [s]
    g, o = g.reshape(n, -1), o.reshape(n, -1)
    sens = np.max([np.abs(p.reshape(n, -1) - o) for p in probes], axis=0)
    ill = sens > atol
    allow = atol + rtol * np.abs(o) + np.where(ill, k * sens, 0.0)
    bad = np.abs(g - o) > allow
    if stats is not None:
        stats.widened += int(ill.sum())
        stats.total += ill.size
        stats.by_name[name] = (int(ill.sum()), ill.size)
    assert not bad.any(), (f"{name}: {bad.any(-1).sum()} envs out of tolerance; worst excess "
                           f"{(np.abs(g - o) - allow).max():.3e} (|gpu - oracle| max {np.abs(g - o).max():.3e})")


def contact_keys(cache):
    """Per env: the sorted contact keys (body, partner, point) of the last solve -- the keys of its
    normal and joint-limit rows -- from a warm-start cache [N, HE_CACHE_WORDS] (engine buffer or
    oracle array)."""
    n, keys, _ = _abi.cache_rows(cache)
    return [tuple(sorted(int(k) for k in keys[e, :n[e]] if (k >> 14) == 0)) for e in range(keys.shape[0])]


def torsion_weights(weights, cache):
    """Per env: {row key: friction bound weight} of the torsional rows, from the oracle's row-weight
    diagnostic (oracle.set_row_weight_out) [N, HE_MAX_ROWS] and its warm-start cache (same row order)."""
    n, keys, _ = _abi.cache_rows(cache)
    return [{int(keys[e, r]): float(weights[e, r]) for r in range(n[e]) if (keys[e, r] >> 14) == 3}
            for e in range(keys.shape[0])]


def friction_states(cache, mu, tw=None):
    """Per env: the stick / slip state of every friction row of the last solve, from a warm-start
    cache: sorted (key, s) with s = +1 / -1 when the impulse sits on its bound (within 1e-5 of it:
    the clamp acted, sliding), 0 inside (sticking); patches with no normal impulse left out. A
    tangential row's bound is mu (sum of its patch's normal impulses); a torsional row's is its
    weight mu r_patch times that sum, the weight from `tw` (torsion_weights of the oracle's solve:
    the patch radius is not in the cache; without `tw` the torsional rows are left out). A friction
    row crossing its bound is a discontinuity of the step like a contact entering the set: where the
    fp32 engine and the fp64 oracle land on different sides, their trajectories part by the slip, so
    such envs are excluded like contact-set mismatches."""
    n, keys, lam = _abi.cache_rows(cache)
    mu = np.broadcast_to(np.asarray(mu, np.float32), (keys.shape[0],))
    out = []
    for e in range(keys.shape[0]):
        st = []
        ks = [int(k) for k in keys[e, :n[e]]]
        for r, key in enumerate(ks):
            b0, b1, sub, kind = _abi.key_fields(key)
            if kind == 0 or (kind == 3 and (tw is None or key not in tw[e])):
                continue
            if sub == _abi.KEY_PATCH:  # the body's terrain patch: its normal rows
                ln = sum(float(lam[e, j]) for j, k2 in enumerate(ks)
                         if (k2 >> 14) == 0 and (k2 & 31) == b0 and ((k2 >> 5) & 31) == 1)
            else:  # a self pair: its own normal row
                ln = sum(float(lam[e, j]) for j, k2 in enumerate(ks) if k2 == (key & 0x3FFF))
            if ln <= 1e-5:
                continue
            w = float(mu[e]) if kind < 3 else tw[e][key]
            bound = w * ln * (1.0 - 1e-5)
            st.append((key, int(np.sign(lam[e, r])) if abs(lam[e, r]) >= bound else 0))
        out.append(tuple(sorted(st)))
    return out


def _obs_tol(oo):
    """Per-element obs tolerance: 5e-5 + 1e-5 rel, and for the velocity blocks (self lin/ang vel
    214:358, task vel/ang-vel differences 574:718) 2e-6 of the 3-vector's norm: a body spinning at
    the 100 rad/s clamp is rotated into the heading frame in fp32 by two different instruction
    orders (kernel vs C oracle), so each component carries ~1e-6 x |v| of rounding."""
    tol = 5e-5 + 1e-5 * np.abs(oo)
    for a, b in ((214, 358), (574, 718)):
        blk = oo[:, a:b].reshape(oo.shape[0], -1, 3)
        nrm = np.repeat(np.linalg.norm(blk, axis=-1), 3, axis=-1)
        tol[:, a:b] = np.maximum(tol[:, a:b], 5e-5 + 2e-6 * nrm)
    return tol


def _physics_compare(he_model, root, dof, targets, calls=2, steps=1, pos_tol=1e-4, vel_tol=1e-2, max_skip=0.02,
                     max_widened=0.05, env_props=None, max_slip=0.0, nprobes=None, **sim):
    """Engine vs oracle for `steps` policy steps (`calls` gym.simulate() each) from the same state,
    both warm-starting from their own caches. The oracle's sensitivity probes (_cond_close) carry
    rounding-level noise (cases.probe_physics_step: state and Delassus operator) into every policy
    step, as the fp32 engine rounds in
    every step, not only at the start. Envs whose contact SETS (keys: body, partner, candidate) ever
    differ are excluded (a point within rounding of the 0.02 m offset, or a tie in the deepest-first
    reduction), at most `max_skip` of them; with max_slip > 0 so are envs whose stick / slip states
    ever differ (friction_states), at most `max_slip` together with those (otherwise the count is
    reported); at most `max_widened` of the compared elements may need the sensitivity widening
    (_cond_close), taken over 3 probes (8 past 5 steps)."""
    n = root.shape[0]
    eng = make_engine(he_model, n, **sim)
    props = {}
    if env_props is not None:  # config 5: mass scale [N,24], friction [N], terrain kind [N]
        ms, fr, tk = env_props
        eng.set_env_properties(cu(ms), cu(fr), cu(tk))
        props = dict(mass_scale=ms, friction=fr, terrain_kind=tk)
        sim = dict(sim, terrain=1)
    eng.root_states.copy_(cu(root))
    eng.dof_state.copy_(cu(dof.reshape(n * 69, 2)))
    eng.dof_targets.copy_(cu(targets))
    r_o, d_o, c_o = root.copy(), dof.copy(), O.new_cache(n)
    # sensitivity probes: joint angles moved by 1e-6 rad (three independent draws)
    # more probes over longer horizons: a friction row that crosses its bound in some of them shows
    # the element's discontinuity, which three draws can miss
    nprobes = nprobes or (3 if steps <= 5 else 8)
    probes = [[root.copy(), dof.copy(), None, O.new_cache(n)] for _ in range(nprobes)]
    sp = _abi.default_sim_params(**sim)
    mismatch = np.zeros(n, bool)
    slip = np.zeros(n, bool)
    for step in range(steps):
        eng.simulate(calls)
        rw = np.zeros((n, _abi.MAX_ROWS), np.float32)  # the oracle's row bound weights (torsion stick / slip)
        O.set_row_weight_out(rw)
        try:
            out = O.physics_step(eng.he_model, sp, r_o, d_o, targets, calls, cache=c_o, **props)
        finally:
            O.set_row_weight_out(None)
        for k, pr in enumerate(probes):
            pr[2] = cases.probe_physics_step(eng.he_model, sp, pr[0], pr[1], targets, calls, pr[3], 123 + 1000 * k + step,
                                             **props)
        torch.cuda.synchronize()
        cg = eng.contact_cache.cpu().numpy()
        kg = contact_keys(cg)
        ko = contact_keys(c_o)
        mismatch |= np.array([a != b for a, b in zip(kg, ko)])
        mu = props["friction"] if "friction" in props else sp.friction
        tw = torsion_weights(rw, c_o)
        slip |= np.array([a != b for a, b in zip(friction_states(cg, mu, tw), friction_states(c_o, mu, tw))])
        mismatch |= eng.num_contacts.cpu().numpy() != out["num_contacts"]
        mismatch |= eng.dropped_contacts.cpu().numpy() != out["dropped"]
    excl = mismatch | (slip if max_slip > 0 else False)
    ok = ~excl
    print(f"contact-set mismatch: {mismatch.sum()}/{n} envs, stick/slip mismatch: {(slip & ~mismatch).sum()}/{n}"
          f"{'' if max_slip > 0 else ' (reported, not excluded)'}")
    assert mismatch.mean() <= max_skip, f"contact-set mismatch in {mismatch.sum()}/{n} envs"
    assert excl.mean() <= max(max_skip, max_slip), f"{excl.sum()}/{n} envs excluded"
    rg = eng.root_states.cpu().numpy()
    dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
    rbg = eng.rb_state.view(n, 24, 13).cpu().numpy()
    # quaternions up to sign: align gpu and probe to the oracle's hemisphere
    def align(q, ref):
        return np.where((q * ref).sum(-1, keepdims=True) < 0, -q, q)
    R = [p[0] for p in probes]
    D = [p[1] for p in probes]
    OS = [p[2] for p in probes]
    st = CondStats()
    kw = dict(stats=st)
    _cond_close("root pos", rg[ok, :3], r_o[ok, :3], [r[ok, :3] for r in R], pos_tol, **kw)
    _cond_close("root quat", align(rg[ok, 3:7], r_o[ok, 3:7]), r_o[ok, 3:7],
                [align(r[ok, 3:7], r_o[ok, 3:7]) for r in R], pos_tol, **kw)
    _cond_close("dof pos", dg[ok, :, 0], d_o[ok, :, 0], [d[ok, :, 0] for d in D], pos_tol, **kw)
    _cond_close("root vel", rg[ok, 7:], r_o[ok, 7:], [r[ok, 7:] for r in R], vel_tol, 1e-3, **kw)
    _cond_close("dof vel", dg[ok, :, 1], d_o[ok, :, 1], [d[ok, :, 1] for d in D], vel_tol, 1e-3, **kw)
    _cond_close("body pos", rbg[ok, :, :3], out["rb_state"][ok, :, :3], [o_["rb_state"][ok, :, :3] for o_ in OS],
                pos_tol, **kw)
    com_g = cases.center_of_mass(_model(), rbg[ok])
    com_o = cases.center_of_mass(_model(), out["rb_state"][ok])
    com_s = [cases.center_of_mass(_model(), o_["rb_state"][ok]) for o_ in OS]
    _cond_close("CoM", com_g, com_o, com_s, pos_tol, **kw)
    _cond_close("dof force", eng.dof_force.view(n, 69).cpu().numpy()[ok], out["dof_force"][ok],
                [o_["dof_force"][ok] for o_ in OS], 0.5, 1e-3, **kw)
    print(f"sensitivity-widened elements: {st.widened}/{st.total} ({100 * st.frac:.2f}%) {st.by_name}")
    assert st.frac <= max_widened, f"{st.widened}/{st.total} elements needed the widening: {st.by_name}"
    return eng, out


def _model():
    from humanoid_amd.model import load_default_model
    return load_default_model()


def test_physics_airborne_matches_oracle(he_model):
    rng = np.random.default_rng(1)
    root, dof = cases.random_state(64, rng, height=(3.0, 4.0))
    targets = rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, self_collision=0, max_skip=0.0, max_widened=0.0)


def test_physics_standing_matches_oracle(he_model, model):
    rng = np.random.default_rng(2)
    root, dof = cases.standing_state(model, 64, rng, xy_jitter=1.0)
    targets = np.zeros((64, 69), np.float32)
    _physics_compare(he_model, root, dof, targets, steps=5, max_skip=0.0, max_widened=0.05)


def test_env_results_independent_of_env_count_and_position(he_model, model):
    """Envs never interact: an env's step is a function of its own state, targets and
    warm-start cache only, whatever the launch's env count and wherever the env sits in it. Eight
    distinct states (standing, lying, airborne actuated, contact-rich) are stepped 3 policy steps
    alone (N = 1 each), inside a ragged launch of 65 envs (one past a wave multiple) and inside a
    launch of 32,768 envs (configs[3]'s eight ranks' worth on one GPU, the largest size tested):
    root, dof, rigid-body rows, contact forces, dof forces and the warm-start cache bit-identical."""
    rng = np.random.default_rng(29)
    r1, d1 = cases.standing_state(model, 2, rng, xy_jitter=1.0)
    r2, d2 = cases.lying_state(2, rng)
    r3, d3 = cases.random_state(2, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
    r4, d4 = cases.random_state(2, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    root = np.concatenate([r1, r2, r3, r4])
    dof = np.concatenate([d1, d2, d3, d4])
    tg = rng.uniform(-0.5, 0.5, (8, 69)).astype(np.float32)
    tg[:2] = 0.0

    def run(n, slots):
        fill_r, fill_d = cases.random_state(n, np.random.default_rng(n), height=(0.85, 1.2), ang=0.8, vel=0.5)
        fill_t = np.random.default_rng(n + 1).uniform(-0.5, 0.5, (n, 69)).astype(np.float32)
        fill_r[slots], fill_d[slots], fill_t[slots] = root, dof, tg
        eng = make_engine(he_model, n)
        eng.root_states.copy_(cu(fill_r))
        eng.dof_state.copy_(cu(fill_d.reshape(n * 69, 2)))
        eng.dof_targets.copy_(cu(fill_t))
        for _ in range(3):
            eng.simulate(2)
        torch.cuda.synchronize()
        sl = torch.as_tensor(slots, device=eng.device)
        out = {k: getattr(eng, k).reshape(n, -1)[sl].cpu().numpy().copy()
               for k in ("root_states", "dof_state", "rb_state", "contact_forces", "dof_force", "contact_cache")}
        del eng
        return out

    alone = {k: [] for k in ("root_states", "dof_state", "rb_state", "contact_forces", "dof_force", "contact_cache")}
    for i in range(8):
        fill_r, fill_d = root[i:i + 1], dof[i:i + 1]
        eng = make_engine(he_model, 1)
        eng.root_states.copy_(cu(fill_r))
        eng.dof_state.copy_(cu(fill_d.reshape(69, 2)))
        eng.dof_targets.copy_(cu(tg[i:i + 1]))
        for _ in range(3):
            eng.simulate(2)
        torch.cuda.synchronize()
        for k in alone:
            alone[k].append(getattr(eng, k).reshape(1, -1).cpu().numpy().copy())
        del eng
    alone = {k: np.concatenate(v) for k, v in alone.items()}
    ragged = run(65, np.array([0, 1, 31, 32, 33, 62, 63, 64]))
    large = run(32768, np.array([0, 4095, 4096, 8191, 16384, 20000, 32766, 32767]))
    assert np.isfinite(alone["root_states"]).all()
    for k in alone:
        assert np.array_equal(alone[k], ragged[k]), f"{k}: N = 65 differs from N = 1"
        assert np.array_equal(alone[k], large[k]), f"{k}: N = 32768 differs from N = 1"


def test_physics_trajectories_30_steps(he_model, model):
    """north_star: joint-angle and CoM trajectories within 1e-4 rad / m, over 30 policy steps (1 s,
    60 substeps, both solvers warm-starting from their own caches): airborne actuated bodies (self
    collision on) and the PD stand-still on the plane."""
    rng = np.random.default_rng(11)
    root, dof = cases.random_state(32, rng, height=(6.0, 7.0), ang=0.4, vel=0.5)
    targets = rng.uniform(-0.5, 0.5, (32, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, steps=30, max_skip=0.0, max_widened=0.01)
    root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
    _physics_compare(he_model, root, dof, np.zeros((32, 69), np.float32), steps=30, max_skip=0.0, max_widened=0.05)


def test_physics_contact_rich_matches_oracle(he_model):
    rng = np.random.default_rng(3)
    root, dof = cases.random_state(96, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    r2, d2 = cases.lying_state(32, rng)
    root = np.concatenate([root, r2])
    dof = np.concatenate([dof, d2])
    targets = rng.uniform(-0.5, 0.5, (128, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets)


def test_physics_solver_tolerance_matches_oracle(he_model):
    """PGS (solver_type 0) only: the optional convergence stop (solver_tolerance = 1e-5 m/s: a sweep that moves no row's
    velocity by more ends the solve) on contact-rich states, 5 steps: the same stop in both."""
    rng = np.random.default_rng(13)
    root, dof = cases.random_state(64, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    targets = rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, steps=5, solver_tolerance=1e-5, solver_type=0, solver_iterations=8)


def test_cold_solve_matches_oracle(he_model, model):
    """PGS (solver_type 0): warm_start = 0 is cold in every physics step of a launch, as in the oracle (the
    kernel used to warm-start the second physics step from the first's impulses): standing bodies
    under random targets, 4 sweeps, 5 policy steps."""
    rng = np.random.default_rng(14)
    root, dof = cases.standing_state(model, 48, rng, xy_jitter=1.0)
    targets = rng.uniform(-0.2, 0.2, (48, 69)).astype(np.float32)
    # 4 cold sweeps are the least converged solve, the one that amplifies rounding most (r03 held it at
    # 2e-4: one joint angle of 3312 landed at 1.003e-4); at north_star's 1e-4 with 8 sensitivity
    # probes it passes on the round-4 build (tests/diag/cold_tol.py, profiles/r04/cold_tol.log). The
    # defect this test guards against (a warm start inside the launch) moves the joint angles by
    # >= 1e-3 in 33 of these 48 envs (oracle warm vs cold, median env max 2.3e-3).
    _physics_compare(he_model, root, dof, targets, steps=5, warm_start=0, solver_iterations=4, solver_type=0, max_skip=0.0,
                     nprobes=8,
                     pos_tol=1e-4)


def test_physics_domain_randomised_terrain(he_model, model):
    """Config 5 extension: per-env mass scale, friction and terrain kind vs the oracle, 3 steps,
    positions and velocities."""
    n = 48
    rng = np.random.default_rng(4)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    root[:, 2] += 0.1
    ms = rng.uniform(0.8, 1.2, (n, 24)).astype(np.float32)
    fr = rng.uniform(0.5, 1.25, n).astype(np.float32)
    tk = (np.arange(n) % 3).astype(np.int32)
    # a 0.1 m drop onto slopes and step edges (feet straddling an edge tip over): the divergent
    # contact-set stress case (0% widened on the r02 final box; bound 1%)
    _physics_compare(he_model, root, dof, np.zeros((n, 69), np.float32), steps=3, env_props=(ms, fr, tk),
                     max_widened=0.01)


def test_knee_limit_matches_oracle(he_model, model):
    """Knee-y driven at +-5 rad targets (humanoid_phc.py:441-446): the joint angle stops inside pi on
    the GPU too, and the trajectory follows the oracle's (limit rows, the blocked-joint effort rule)."""
    n = 8
    rng = np.random.default_rng(7)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5
    targets = np.zeros((n, 69), np.float32)
    targets[:, [4, 16]] = np.where(np.arange(n) % 2 == 0, 5.0, -5.0)[:, None]
    eng, _ = _physics_compare(he_model, root, dof, targets, steps=20, self_collision=0, max_skip=0.0)
    q = eng.dof_state.view(n, 69, 2).cpu().numpy()[..., 0]
    ang = np.linalg.norm(q.reshape(n, 23, 3), axis=-1)
    assert ang.max() < np.pi and ang[:, [1, 5]].min() > np.pi - 0.05  # knees (joints 2, 6) on the limit
    # dof_force carries the limit force with the drive's: along the knee's axis the two
    # cancel to the inertial remainder, as in the oracle (compared above at 0.5 N m)
    f = eng.dof_force.view(n, 69).cpu().numpy().reshape(n, 23, 3)
    qa = q.reshape(n, 23, 3)
    for j in (1, 5):
        along = (f[:, j] * qa[:, j]).sum(1) / np.linalg.norm(qa[:, j], axis=1)
        assert (np.abs(along) < 50.0).all(), along


@pytest.mark.parametrize("cap", [16, 40])
def test_contact_overflow_counted_and_reduced(he_model, cap):
    """Lying bodies past the capacity: the engine reports the overflow per env exactly as the oracle,
    keeps the same (deepest-first, row-budgeted) contact set, and the state matches. cap 16 caps the
    slots (25-40 contacts generated: every env overflows by construction); cap 40 (the default)
    leaves the 63-row budget as the limit (patch friction: 2-5 of 32 envs in the oracle)."""
    rng = np.random.default_rng(5)
    root, dof = cases.lying_state(32, rng)
    # lowered to 0.08-0.10 m: limbs start deep in the plane, 25-40 contacts generated per env
    root[:, 2] = 0.08 + rng.uniform(0, 0.02, 32).astype(np.float32)
    targets = np.zeros((32, 69), np.float32)
    eng, out = _physics_compare(he_model, root, dof, targets, steps=1, max_skip=0.05, max_widened=0.05,
                                max_contacts=cap)
    assert (out["dropped"] > 0).sum() >= (8 if cap == 16 else 1), "the case must overflow"


def test_env_step_fused_matches_oracle(he_model, model, golden):
    """he_step_actions + he_imitation_reset_step (= he_env_step): PD targets from actions, physics,
    reward/reset/obs and the device reset of flagged envs (hash phases). The imitation + reset half
    is checked tightly against the oracle run on the GPU's own post-physics state; the physics half
    against the oracle physics at the position tolerance."""
    from humanoid_amd.model import pd_action_offset_scale
    from humanoid_amd.body_sets import frozen_dof_mask
    g = golden("env_step")
    n = 24
    tables = tables_from_golden(g)
    eng = make_engine(he_model, n)
    eng.load_motions(tables)
    off, sc = pd_action_offset_scale(model)
    frozen = np.array(frozen_dof_mask(), np.int32)
    eng.set_pd_params(off, sc, frozen)
    rng = np.random.default_rng(5)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    eng.root_states.copy_(cu(root))
    eng.dof_state.copy_(cu(dof.reshape(n * 69, 2)))
    st = cu(g["start_times"]); so = torch.zeros(n, device="cuda:0"); go = torch.zeros(n, 3, device="cuda:0")
    prog = torch.zeros(n, dtype=torch.int16, device="cuda:0")
    mids = torch.arange(n, device="cuda:0", dtype=torch.int64)
    em = eng.env_motion(mids, st, so, go, prog)
    p = _abi.imitation_params()
    obs = torch.zeros(n, 934, device="cuda:0"); rew = torch.zeros(n, device="cuda:0")
    raw = torch.zeros(n, 5, device="cuda:0")
    reset = torch.zeros(n, dtype=torch.uint8, device="cuda:0"); term = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    actions = rng.uniform(-1.5, 1.5, (n, 69)).astype(np.float32)
    seed = 1234
    mt = O.MotionTables.from_tables(tables)
    sp = _abi.default_sim_params()
    tgt = off + sc * np.clip(actions, -1, 1)
    tgt[:, frozen.astype(bool)] = 0
    n_reset = 0
    for step in range(4):
        r_pre = eng.root_states.cpu().numpy().copy()
        d_pre = eng.dof_state.view(n, 69, 2).cpu().numpy().copy()
        c_pre = eng.contact_cache.cpu().numpy().copy()
        st_o = st.cpu().numpy().copy(); so_o = so.cpu().numpy().copy(); go_o = go.cpu().numpy().copy()
        prog_o = prog.cpu().numpy().copy()
        eng.step_actions(cu(actions), 2)
        torch.cuda.synchronize()
        np.testing.assert_allclose(eng.dof_targets.cpu().numpy(), tgt, atol=1e-6)
        # the oracle starts from the engine's own warm-start cache (its signature is r_pre's pose)
        probes = []
        for k in range(3):  # oracle sensitivity probes (see _cond_close)
            r_s, d_s = r_pre.copy(), d_pre.copy()
            cases.probe_physics_step(eng.he_model, sp, r_s, d_s, tgt.astype(np.float32), 2, c_pre.copy(), 100 * step + k)
            probes.append((r_s, d_s))
        c_o = c_pre.copy()
        out = O.physics_step(eng.he_model, sp, r_pre, d_pre, tgt.astype(np.float32), 2, cache=c_o)
        same = np.array([a == b for a, b in zip(contact_keys(eng.contact_cache.cpu().numpy()), contact_keys(c_o))])
        assert same.mean() >= 0.9
        # saturating actions (targets up to +-pi, knees +-5 rad): the effort limit scales the drive
        # continuously, so joint angles are held at the physics tolerance too
        _cond_close("root pos", eng.root_states.cpu().numpy()[same, :3], r_pre[same, :3],
                    [r[same, :3] for r, _ in probes], 1e-4)
        _cond_close("dof pos", eng.dof_state.view(n, 69, 2).cpu().numpy()[same, :, 0], d_pre[same, :, 0],
                    [d[same, :, 0] for _, d in probes], 1e-4)
        # oracle imitation + reset on the GPU's post-physics state
        rb = eng.rb_state.view(n, 24, 13).cpu().numpy().copy()
        dstate = eng.dof_state.view(n, 69, 2).cpu().numpy().copy()
        rstate = eng.root_states.cpu().numpy().copy()
        df = eng.dof_force.view(n, 69).cpu().numpy().copy()
        cf = eng.contact_forces.view(n, 24, 3).cpu().numpy().copy()
        im = O.imitation_step(p, mt, rb, dstate[..., 1], df, prog_o, np.arange(n), st_o, so_o, go_o)
        state = dict(start_times=st_o, start_offsets=so_o, global_offset=go_o, progress=im["progress"],
                     root_states=rstate, dof_state=dstate, dof_targets=tgt.astype(np.float32).copy(), rb_state=rb,
                     contact_forces=cf, obs=im["obs"], reset=np.zeros(n, np.uint8), terminate=np.zeros(n, np.uint8))
        ids = np.nonzero(im["reset"])[0]
        n_reset += len(ids)
        if len(ids):
            ph = np.array([O.hash_uniform(seed, step, int(e)) for e in ids], np.float32)
            O.reset_envs(p, mt, ids, ph, np.arange(n), state)
        eng.imitation_reset_step(p, em, obs, rew, raw, reset, term, seed=seed, step_index=step)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(reset.cpu().numpy(), im["reset"])
        np.testing.assert_array_equal(term.cpu().numpy(), im["terminate"])
        np.testing.assert_allclose(rew.cpu().numpy(), im["rew"], atol=5e-5, rtol=1e-5)
        np.testing.assert_allclose(raw.cpu().numpy(), im["reward_raw"], atol=5e-5, rtol=1e-5)
        og, oo = obs.cpu().numpy(), state["obs"]
        bad = np.abs(og - oo) > _obs_tol(oo)
        assert not bad.any(), (f"obs mismatch at (env, col) {np.argwhere(bad)[:8].tolist()}: gpu {og[bad][:8]} "
                               f"oracle {oo[bad][:8]}; step {step} reset ids {ids.tolist()} "
                               f"start gpu {st.cpu().numpy()[np.argwhere(bad)[:1, 0]]} oracle "
                               f"{state['start_times'][np.argwhere(bad)[:1, 0]]} prog {im['progress'][np.argwhere(bad)[:1, 0]]}")
        np.testing.assert_array_equal(prog.cpu().numpy(), state["progress"])
        np.testing.assert_array_equal(st.cpu().numpy(), state["start_times"])
        if len(ids):
            np.testing.assert_allclose(eng.root_states.cpu().numpy()[ids, :3], state["root_states"][ids, :3], atol=2e-6)
            cases.assert_expmap_close(eng.dof_state.view(n, 69, 2).cpu().numpy()[ids, :, 0], state["dof_state"][ids, :, 0])
            cases.assert_expmap_close(eng.dof_targets.cpu().numpy()[ids], state["dof_targets"][ids])
            assert (eng.contact_forces.view(n, 24, 3).cpu().numpy()[ids] == 0).all()
    assert n_reset > 0, "test should exercise the device reset path"


@pytest.mark.parametrize("fused", [1, 0])
def test_env_step_single_call_equals_two_calls(he_model, model, golden, fused):
    """he_env_step -- as one launch (the imitation step in the physics kernel's epilogue) and as two
    -- is exactly he_step_actions followed by he_imitation_reset_step, bit for bit: obs, reward,
    reset / terminate flags, the state and the warm-start cache, over 12 steps of random actions
    under which bodies fall and the device resets them (their cache signature is invalidated, so the
    next solve is cold). The two-launch form is held to the oracle by test_env_step_fused_matches_oracle."""
    from humanoid_amd.model import pd_action_offset_scale
    g = golden("env_step")
    n = 24
    outs = []
    n_reset = 0
    for single in (True, False):
        eng = make_engine(he_model, n)
        eng.set_fused_step(fused)
        eng.load_motions(tables_from_golden(g))
        off, sc = pd_action_offset_scale(model)
        eng.set_pd_params(off, sc, None)
        root, dof = cases.standing_state(model, n)
        eng.root_states.copy_(cu(root))
        st = cu(g["start_times"]); so = torch.zeros(n, device="cuda:0"); go = torch.zeros(n, 3, device="cuda:0")
        prog = torch.zeros(n, dtype=torch.int16, device="cuda:0")
        em = eng.env_motion(torch.arange(n, device="cuda:0"), st, so, go, prog)
        bufs = [torch.zeros(n, 934, device="cuda:0"), torch.zeros(n, device="cuda:0"), torch.zeros(n, 5, device="cuda:0"),
                torch.zeros(n, dtype=torch.uint8, device="cuda:0"), torch.zeros(n, dtype=torch.uint8, device="cuda:0")]
        rng = np.random.default_rng(31)
        trace = []
        for k in range(12):
            a = cu(rng.uniform(-1.0, 1.0, (n, 69)).astype(np.float32))
            if single:
                eng.env_step(_abi.imitation_params(), em, a, *bufs, seed=7, step_index=k)
            else:
                eng.step_actions(a, 2)
                eng.imitation_reset_step(_abi.imitation_params(), em, *bufs, seed=7, step_index=k)
            torch.cuda.synchronize()
            rs = bufs[3].cpu().numpy().astype(bool)
            cache = eng.contact_cache.cpu().numpy()
            r = eng.root_states.cpu().numpy()
            if single:
                n_reset += int(rs.sum())
                # a reset env's cache no longer matches its (new) root pose: the next solve is cold
                if rs.any():
                    assert (cache[rs, :7] != r[rs, :7]).any(axis=1).all()
            trace.append([b.cpu().numpy() for b in bufs] + [eng.rb_state.cpu().numpy(), r, cache,
                                                           eng.dof_state.cpu().numpy()])
        outs.append(trace)
    assert n_reset > 0, "the run must exercise the device reset"
    for ta, tb in zip(*outs):
        for x, y in zip(ta, tb):
            np.testing.assert_array_equal(x, y)


def test_model_with_more_boxes_than_corner_lanes_is_refused(he_model):
    """Box corners take 8-lane groups above the 24 body lanes (he_topo.h HE_MAX_BOXES = 5): a model
    with a sixth box geom is refused at he_set_model with the reason, not simulated wrong."""
    from humanoid_amd.engine import Engine, EngineError
    from humanoid_amd.model import GEOM_BOX
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    m = type(he_model).from_buffer_copy(he_model)
    boxes = [b for b in range(24) if m.geom_type[b] == GEOM_BOX]
    assert len(boxes) == 4  # SMPL: ankles and toes
    for b in (0, 13):  # two more bodies become boxes
        m.geom_type[b] = GEOM_BOX
    with pytest.raises(EngineError, match="box geoms"):
        Engine(m, 4, device=0)
    m = type(he_model).from_buffer_copy(he_model)
    m.geom_type[5] = 7
    with pytest.raises(EngineError, match="geom type 7"):
        Engine(m, 4, device=0)


def test_limit_backstop_matches_oracle(he_model, model):
    """The integration's limit backstop (limit_clamp) on the GPU: joints 5 mrad inside the limit
    moving outward at 60 rad/s with rows that cannot act (no sweeps), and the same with the rows
    (which then hold first); both as the oracle, the clamped joints at pi - 0.01 on their side."""
    n = 16
    rng = np.random.default_rng(3)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=0.5)
    root[:, 2] += 1.5
    axis = rng.standard_normal((n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    j = rng.integers(0, 23, n)
    for e in range(n):
        dof[e, 3 * j[e]:3 * j[e] + 3, 0] = (axis[e] * (np.pi - 0.025)).astype(np.float32)
        dof[e, 3 * j[e]:3 * j[e] + 3, 1] = (axis[e] * 60.0).astype(np.float32)
    targets = np.zeros((n, 69), np.float32)
    sim = dict(self_collision=0, kp_scale=0.0, kd_scale=0.0)
    eng, _ = _physics_compare(he_model, root, dof, targets, calls=1, steps=1, max_skip=0.0,
                              solver_iterations=0, solver_type=0, warm_start=0, substeps=1, **sim)
    q = eng.dof_state.view(n, 69, 2).cpu().numpy()[..., 0].reshape(n, 23, 3)
    t = np.linalg.norm(q[np.arange(n), j].astype(np.float64), axis=1)
    np.testing.assert_allclose(t, np.pi - 0.01, atol=2e-6)
    assert ((q[np.arange(n), j] * axis).sum(1) > 0).all()
    # with the rows (one policy step: 60 rad/s joints spread a 1e-4 m difference within ~3 steps)
    _physics_compare(he_model, root, dof, targets, calls=2, steps=1, max_skip=0.0, **sim)


def test_explicit_bias_matches_oracle(he_model, model):
    """bias_midpoint = 0 (the velocity-dependent bias explicit, at u0) on the GPU against
    the oracle: airborne actuated bodies (one policy step) and the PD stand-still (10 steps)."""
    rng = np.random.default_rng(21)
    root, dof = cases.random_state(64, rng, height=(3.0, 4.0))
    targets = rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, self_collision=0, bias_midpoint=0, solver_type=0, solver_iterations=8,
                     max_skip=0.0,
                     max_widened=0.0)
    root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
    _physics_compare(he_model, root, dof, np.zeros((32, 69), np.float32), steps=10, bias_midpoint=0, solver_type=0,
                     solver_iterations=8,
                     max_skip=0.0, max_widened=0.05)


def test_tgs_small_step_mode_matches_oracle(he_model, model):
    """TGS's small-step form on the PGS step (DESIGN §5 "TGS"): substeps 8 (1/480 s) with one Gauss-Seidel
    sweep each -- PhysX TGS's 4 position iterations per 1/120 s step, each re-integrating dt/4, 0
    velocity iterations (isaacgym_env.py:16-18) -- against the oracle under the same parameters:
    airborne actuated bodies (one policy step) and the PD stand-still (10 steps)."""
    tgs = dict(substeps=8, solver_iterations=1, solver_type=0)
    rng = np.random.default_rng(41)
    root, dof = cases.random_state(64, rng, height=(3.0, 4.0))
    targets = rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32)
    _physics_compare(he_model, root, dof, targets, self_collision=0, max_skip=0.0, max_widened=0.0, **tgs)
    root, dof = cases.standing_state(model, 32, rng, xy_jitter=1.0)
    _physics_compare(he_model, root, dof, np.zeros((32, 69), np.float32), steps=10, max_skip=0.0,
                     max_widened=0.05, **tgs)


def test_world_angular_velocity_clamp_matches_oracle(he_model, model):
    """max_angular_velocity on each link's WORLD angular velocity (PxRigidBody) and
    max_joint_velocity on the joint rates, both active: airborne bodies spun up to 60-80 rad/s with
    the caps lowered to 40 / 30 rad/s, one policy step, against the oracle; no link leaves the cap."""
    rng = np.random.default_rng(24)
    n = 64
    root, dof = cases.random_state(n, rng, height=(3.0, 4.0), vel=0.0)
    root[:, 10:13] = rng.normal(0, 20.0, (n, 3)).astype(np.float32)
    dof[..., 1] = rng.normal(0, 25.0, (n, 69)).astype(np.float32)
    targets = rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32)
    eng, out = _physics_compare(he_model, root, dof, targets, self_collision=0, max_angular_velocity=40.0,
                                max_joint_velocity=30.0, max_skip=0.0, max_widened=0.0)
    rb = eng.rb_state.view(n, 24, 13).cpu().numpy()
    w = np.linalg.norm(rb[..., 10:13].astype(np.float64), axis=-1)
    # the rows report the state after the last integration, whose world rates use the integrated
    # rotations: within the cap up to the rotation over one physics step
    assert w.max() < 40.0 * 1.5, w.max()


def _random_action_gpu(he_model, model, n, amp, steps, airborne=False, **sim):
    from humanoid_amd.model import pd_action_offset_scale
    off, sc = pd_action_offset_scale(model)
    rng = np.random.default_rng(8)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    if airborne:
        root[:, 2] += 200.0
        sim.setdefault("self_collision", 0)
    eng = make_engine(he_model, n, **sim)
    eng.root_states.copy_(cu(root))
    eng.dof_state.copy_(cu(dof.reshape(n * 69, 2)))
    off_t, sc_t = cu(np.asarray(off, np.float32)), cu(np.asarray(sc, np.float32))
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(8)
    vmax = torch.zeros(n, device="cuda:0")
    for _ in range(steps):
        a = (torch.rand(n, 69, device="cuda:0", generator=gen) * 2.0 - 1.0) * amp
        eng.dof_targets.copy_(off_t + sc_t * a)
        eng.simulate(2)
        vmax = torch.maximum(vmax, torch.linalg.norm(eng.root_states[:, 7:10], dim=1))
    torch.cuda.synchronize()
    rg = eng.root_states.cpu().numpy()
    dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
    assert np.isfinite(rg).all() and np.isfinite(dg).all()
    me = O.momentum_energy(eng.he_model, _abi.default_sim_params(), rg, dg)
    M = float(np.sum(model.mass))
    ke = me[:, 6] - 0.5 * (me[:, :3] ** 2).sum(1) / M
    return vmax.cpu().numpy(), ke, dg


def test_midpoint_bias_tames_the_runaway_on_gpu(he_model, model):
    """PGS (solver_type 0): DESIGN §5's runaway regime through the engine: airborne bodies under random targets U(+-1) of
    the PD scale renewed every policy step for 3 s. With the bias explicit the median internal
    kinetic energy runs away (the oracle's CPU test: ~50 kJ); with the default midpoint bias it stays
    at the dt-refined level (oracle ~1.0 kJ)."""
    _require_gpu()
    _, ke_exp, _ = _random_action_gpu(he_model, model, 256, 1.0, 90, airborne=True, bias_midpoint=0, solver_type=0,
                                      solver_iterations=8)
    _, ke_mid, _ = _random_action_gpu(he_model, model, 256, 1.0, 90, airborne=True, solver_type=0,
                                      solver_iterations=8)
    res = (float(np.median(ke_exp)), float(np.median(ke_mid)))
    print(f"median internal KE after 3 s (explicit, midpoint): {res}")
    assert res[0] > 1e4, res
    assert res[1] < 1.5e3, res


@pytest.mark.parametrize("amp", [0.5, 0.75, 1.0])
def test_saturated_random_actions_stay_physical_on_gpu(he_model, model, amp):
    """VERDICT r02 item 1 at full size, swept over the action amplitude: 4096 standing envs under
    U(+-amp) random actions (new every policy step) for 2 s, under the default step (TGS, the
    reference's solver). The median internal kinetic energy stays at the dt-refined level (U(+-1):
    oracle TGS 0.79 kJ, 1/480 s PGS steps 0.80 kJ, the explicit bias 22 kJ) and no joint passes its
    angle cap.

    Root speeds: round 4's PGS step let a limb wedge 5-7 cm inside its own thigh and launched it at
    17.4 m/s (DESIGN §5 "the runaway tail"); the TGS step's contact rows are solved per position
    iteration against separations that advance with the iterations' motion, and the 4096-env oracle
    study at U(+-0.75) / U(+-1) has no root over 10 m/s (max 7.8 / 9.0). The bar is round 3's: at most
    0.1 % of envs past 10 m/s and none past 15 m/s, at every amplitude."""
    _require_gpu()
    n = 4096
    vmax, ke, dg = _random_action_gpu(he_model, model, n, amp, 60)
    q = np.linalg.norm(dg[..., 0].reshape(n, 23, 3), axis=-1)
    print(f"U(+-{amp}): envs over 10 m/s: {int((vmax > 10).sum())}/{n}, over 15 m/s {int((vmax > 15).sum())}, "
          f"max root speed {vmax.max():.2f} m/s (env {int(vmax.argmax())}), median internal KE {np.median(ke):.1f} J, "
          f"max joint angle {q.max():.4f}")
    assert vmax.max() < 15.0, vmax.max()
    assert int((vmax > 10).sum()) <= n // 1000, int((vmax > 10).sum())
    assert np.median(ke) < 1.5e3
    assert q.max() <= np.pi - 0.01 + 1e-5  # the limit backstop's cap (limit_clamp) at most
