"""The reference-facing host layer: the ``isaacgym`` facade
(``humanoid_amd.isaacgym``) and the ``HumanoidPHC`` / ``PHCPufferEnv`` mirrors.

CPU tests check the API surface and its error behaviour; GPU tests drive the facade the way
``humanoid_phc.py`` does and check it against direct engine calls, and pin the PHCPufferEnv
bookkeeping (terminals / truncations / masks / episode info, ``clean_pufferl/env.py:124-183``)
against a line-by-line host restatement fed with the same per-step engine outputs."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import cases


# ----------------------------------------------------------------------------------- CPU
def test_env_config_solver_iterations():
    """solver_iterations counts TGS position iterations under solver_type 1 (isaacgym_env.py:17: 4)
    and PGS sweeps under 0; unset, each solver's default; an explicit TGS count other than 4 warns
    (it meant PGS sweeps before round 5)."""
    import warnings
    from humanoid_amd.env import EnvConfig
    assert EnvConfig().resolved_solver_iterations() == 4
    assert EnvConfig(solver_type=0).resolved_solver_iterations() == 8
    assert EnvConfig(solver_type=0, solver_iterations=6).resolved_solver_iterations() == 6
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert EnvConfig(solver_iterations=4).resolved_solver_iterations() == 4
    with pytest.warns(UserWarning, match="TGS position iterations"):
        assert EnvConfig(solver_iterations=8).resolved_solver_iterations() == 8


def test_gymapi_surface_and_errors():
    from humanoid_amd.isaacgym import gymapi, gymtorch
    from humanoid_amd.model import DEFAULT_MODEL_JSON
    gym = gymapi.acquire_gym()
    assert gym is gymapi.acquire_gym()
    sp = gymapi.SimParams()
    assert sp.physx.num_position_iterations == 4 and sp.gravity.z == -9.81  # isaacgym_env.py:18-33
    with pytest.raises(NotImplementedError):
        gym.create_sim(-1, -1, gymapi.SIM_PHYSX, sp)  # no CPU pipeline
    with pytest.raises(NotImplementedError):
        gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)  # no viewer
    sim = gym.create_sim(0, -1, gymapi.SIM_PHYSX, sp)
    opts = gymapi.AssetOptions()
    opts.angular_damping, opts.max_angular_velocity = 0.01, 100.0
    asset = gym.load_asset(sim, "/", DEFAULT_MODEL_JSON, opts)
    assert gym.get_asset_rigid_body_count(asset) == 24 and gym.get_asset_dof_count(asset) == 69
    assert gym.find_asset_rigid_body_index(asset, "L_Knee") == 2
    props = gym.get_asset_dof_properties(asset)
    assert props.dtype == gymapi.DofPropertiesDtype and props.shape == (69,)
    props["stiffness"] *= 2.0  # numpy structured array semantics, as humanoid_phc.py:276-280
    with pytest.raises(RuntimeError):
        gym.prepare_sim(sim)  # no actors yet
    with pytest.raises(ValueError):
        gymtorch.unwrap_tensor(torch.zeros(4, 4).t())  # wrapper.py:52 contiguous check


# ----------------------------------------------------------------------------------- GPU
def _facade_sim(n, self_collision=True, pose_fn=None):
    from humanoid_amd.isaacgym import gymapi
    from humanoid_amd.model import DEFAULT_MODEL_JSON
    gym = gymapi.acquire_gym()
    sp = gymapi.SimParams()
    sim = gym.create_sim(0, -1, gymapi.SIM_PHYSX, sp)
    opts = gymapi.AssetOptions()
    opts.angular_damping, opts.max_angular_velocity = 0.01, 100.0
    opts.default_dof_drive_mode = gymapi.DOF_MODE_NONE
    asset = gym.load_asset(sim, "/", DEFAULT_MODEL_JSON, opts)
    plane = gymapi.PlaneParams()
    gym.add_ground(sim, plane)
    dof_prop = gym.get_asset_dof_properties(asset)
    dof_prop["driveMode"] = gymapi.DOF_MODE_POS
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-5, -5, 0), gymapi.Vec3(5, 5, 5), 4)
        gym.begin_aggregate(env, 160, 160, True)
        pose = (gymapi.Transform(gymapi.Vec3(0.1 * i, 0.0, 0.89), gymapi.Quat(0, 0, 0, 1)) if pose_fn is None
                else pose_fn(gymapi, i))
        h = gym.create_actor(env, asset, pose, f"humanoid_{i}", i, 0 if self_collision else 1, 0)
        gym.enable_actor_dof_force_sensors(env, h)
        assert abs(sum(p.mass for p in gym.get_actor_rigid_body_properties(env, h)) - 74.0) < 0.1
        gym.set_actor_dof_properties(env, h, dof_prop)
        sprops = gym.get_actor_rigid_shape_properties(env, h)
        gym.set_actor_rigid_shape_properties(env, h, sprops)
        gym.end_aggregate(env)
    gym.prepare_sim(sim)
    return gym, sim


@pytest.mark.gpu
def test_facade_matches_direct_engine(he_model):
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.isaacgym import gymtorch
    n = 16
    gym, sim = _facade_sim(n)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    assert root.shape == (n, 13) and dof.shape == (n * 69, 2) and rb.shape == (n * 24, 13)
    rng = np.random.default_rng(5)
    r0, d0 = cases.random_state(n, rng, height=(0.9, 1.1))
    src_r = torch.from_numpy(r0).cuda()
    src_d = torch.from_numpy(d0.reshape(n * 69, 2)).cuda()
    ids = torch.arange(n, dtype=torch.int32, device="cuda")
    gym.set_actor_root_state_tensor_indexed(sim, gymtorch.unwrap_tensor(src_r), gymtorch.unwrap_tensor(ids), n)
    gym.set_dof_state_tensor_indexed(sim, gymtorch.unwrap_tensor(src_d), gymtorch.unwrap_tensor(ids), n)
    tgt = torch.from_numpy(rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32)).cuda()
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tgt))
    gym.simulate(sim)
    gym.simulate(sim)
    gym.fetch_results(sim, True)
    gym.refresh_actor_root_state_tensor(sim)
    gym.refresh_dof_state_tensor(sim)
    eng = Engine(he_model, n, device=0, sim_params=_abi.default_sim_params())
    eng.root_states.copy_(src_r)
    eng.dof_state.copy_(src_d)
    eng.dof_targets.copy_(tgt)
    eng.simulate(2)
    torch.cuda.synchronize()
    assert torch.equal(root, eng.root_states) and torch.equal(dof, eng.dof_state)
    # the views alias engine memory: a write through the view is seen by the engine
    root[0, 2] = 5.0
    assert float(sim.engine.root_states[0, 2]) == 5.0


@pytest.mark.gpu
def test_facade_creation_poses_are_the_default_init_pose():
    """_initial_humanoid_root_states (humanoid_phc.py:522-523) = the root states after prepare_sim
    with zero velocities: actors created at their own height and heading must land there, in both
    the root state tensor and the engine's Default-init buffer (HE_BUF_INIT_ROOT_STATE)."""
    from humanoid_amd.isaacgym import gymtorch
    n = 6

    def pose(gymapi, i):
        yaw = 0.3 * i
        return gymapi.Transform(gymapi.Vec3(0.2 * i, -0.1 * i, 1.0 + 0.05 * i),
                                gymapi.Quat(0, 0, np.sin(yaw / 2), np.cos(yaw / 2)))

    gym, sim = _facade_sim(n, pose_fn=pose)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim)).cpu().numpy()
    init = sim.engine.initial_root_states.cpu().numpy()
    want = np.zeros((n, 13), np.float32)
    for i in range(n):
        yaw = 0.3 * i
        want[i, :7] = [0.2 * i, -0.1 * i, 1.0 + 0.05 * i, 0, 0, np.sin(yaw / 2), np.cos(yaw / 2)]
    np.testing.assert_allclose(root, want, atol=1e-6)
    np.testing.assert_allclose(init, want, atol=1e-6)


def _clip_dict(model, k=4, frames=90):
    from humanoid_amd import synthetic
    return {f"clip{i}": synthetic.make_clip(model, np.random.default_rng(100 + i), num_frames=frames)
            for i in range(k)}


def _reference_bookkeeping(seq, n, log_interval):
    """clean_pufferl/env.py:124-183 restated on host lists (the reference's own code path)."""
    ep_ret = np.zeros(n, np.float32)
    ep_len = np.zeros(n, np.int32)
    infos = {"episode_return": [], "episode_length": [], "truncated_rate": []}
    raw_sum = np.zeros(5, np.float64)
    out = []
    for tick, (rew, reset, term, raw) in enumerate(seq, 1):
        raw_sum += raw.mean(0)
        terminals = np.zeros(n, bool)
        truncs = np.zeros(n, bool)
        ridx = np.nonzero(reset)[0]
        if len(ridx):
            infos["episode_return"] += ep_ret[ridx].tolist()
            infos["episode_length"] += ep_len[ridx].tolist()
            ep_ret[ridx] = 0
            ep_len[ridx] = 0
            tidx = np.nonzero(term)[0]
            terminals[tidx] = True
            infos["truncated_rate"] += [0.0] * len(tidx)
            tr = ridx[~np.isin(ridx, tidx)]
            truncs[tr] = True
            infos["truncated_rate"] += [1.0] * len(tr)
        ep_ret[~reset] += rew[~reset]
        ep_len[~reset] += 1
        info = []
        if tick % log_interval == 0:
            info = [{k: float(np.mean(v)) if v else float("nan") for k, v in infos.items()}]
            for v in infos.values():
                v.clear()
            info[0].update({"rew_body_pos": raw_sum[0] / log_interval, "rew_power": raw_sum[4] / log_interval})
            raw_sum[:] = 0
        out.append((terminals, truncs, info))
    return out


@pytest.mark.gpu
def test_puffer_env_bookkeeping_matches_reference_logic(model):
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    n, li = 64, 5
    cfg = EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=3, log_interval=li)
    pe = PHCPufferEnv(cfg)
    obs, info = pe.reset()
    assert obs.shape == (n, 934) and torch.isfinite(obs).all() and info == []
    rng = np.random.default_rng(0)
    seq, got = [], []
    for t in range(25):
        a = rng.uniform(-1.5, 1.5, (n, 69)).astype(np.float32)  # clip_actions clamps
        obs, rew, terminals, truncs, info = pe.step(a)
        e = pe.env
        seq.append((rew.cpu().numpy(), e.reset_buf.cpu().numpy().copy(), e.extras["terminate"].cpu().numpy(),
                    e.extras["reward_raw"].cpu().numpy()))
        got.append((terminals.cpu().numpy().copy(), truncs.cpu().numpy().copy(), pe.masks.cpu().numpy().copy(), info))
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    ref = _reference_bookkeeping(seq, n, li)
    n_resets = sum(int(s[1].sum()) for s in seq)
    assert n_resets > 0, "the action stream should make some envs fall"
    for (tg, trg, mg, ig), (tr, trr, ir) in zip(got, ref):
        assert (tg == tr).all() and (trg == trr).all() and (mg == ~trr).all()
        assert len(ig) == len(ir)
        for a, b in zip(ig, ir):
            for k in ("episode_return", "episode_length", "truncated_rate", "rew_body_pos", "rew_power"):
                assert (np.isnan(a[k]) and np.isnan(b[k])) or abs(a[k] - b[k]) <= 1e-4 * max(1.0, abs(b[k])), (k, a, b)


@pytest.mark.gpu
def test_humanoid_phc_reset_and_step(model):
    from humanoid_amd.env import EnvConfig, HumanoidPHC
    n = 32
    env = HumanoidPHC(EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=1))
    obs = env.reset()
    assert obs.shape == (n, 934) and torch.isfinite(obs).all()
    # after the reference-state init the simulated bodies sit on the reference motion
    assert int(env.progress_buf.abs().sum()) == 0
    obs, rew, reset, extras = env.step(torch.zeros(n, 69, device=env.device))
    assert rew.shape == (n,) and reset.dtype == torch.bool and set(extras) >= {"terminate", "reward_raw"}
    assert (env.progress_buf == 1).all() and torch.isfinite(rew).all()
    assert bool(((rew >= 0) & (rew <= 1)).all())  # 4 weighted exp terms, power is 0 while progress <= 3
    ids = torch.arange(0, n, 2, device=env.device)
    env.reset(ids)
    assert (env.progress_buf[ids] == 0).all() and (env.progress_buf[1::2] == 1).all()
    n_unique = env.toggle_eval_mode()
    assert n_unique == 4 and env.flag_im_eval
    hist = env.untoggle_eval_mode(["clip1"])
    assert hist.shape == (4,) and float(hist[1]) == 1.0
    env.resample_motions()
    assert torch.isfinite(env.obs_buf).all()


@pytest.mark.gpu
def test_puffer_env_amp_obs(model):
    """use_amp_obs (config.py:98): the AMP buffers ride along the device step (clean_pufferl/env.py:94,
    206-207; humanoid_phc.py:154-157, 665-676): [N, 1960] view, history shifted each step for envs
    that continue, demo rows written for every reset env."""
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    n = 64
    cfg = EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=5, use_amp_obs=True)
    pe = PHCPufferEnv(cfg)
    assert pe.amp_observation_space.shape == (1960,) and pe.amp_obs.shape == (n, 1960)
    pe.reset()
    demo = pe.fetch_amp_obs_demo()
    assert demo.shape == (n, 1960)
    # after the full reset every env's history comes from its motion and demo = buffer
    assert torch.equal(demo, pe.amp_obs) and torch.isfinite(demo).all()
    rng = np.random.default_rng(1)
    prev = pe.amp_obs.view(n, 10, 196).clone()
    n_reset = 0
    for _ in range(12):
        pe.step(rng.uniform(-1.5, 1.5, (n, 69)).astype(np.float32))
        cur = pe.amp_obs.view(n, 10, 196)
        reset = pe.env.reset_buf
        keep = ~reset
        assert torch.equal(cur[keep, 1:], prev[keep, :-1])
        assert torch.equal(pe.env.extras["amp_obs"], pe.amp_obs)
        if reset.any():
            n_reset += int(reset.sum())
            assert torch.equal(demo.view(n, 10, 196)[reset], cur[reset])
        prev = cur.clone()
    assert n_reset > 0
    assert torch.isfinite(pe.amp_obs).all()


# ------------------------------------------------------------- config branches (A11 mirror)
def test_env_config_branches_raise_before_the_gpu():
    """The obs / robot options the fused kernels do not implement raise (NotImplementedError), an
    unknown state_init raises as the reference does (ValueError, humanoid_phc.py:679-686) -- before
    any GPU work, so this runs on the CPU. (All four StateInit values are implemented.)"""
    from humanoid_amd.env import EnvConfig, HumanoidPHC, RobotConfig
    from humanoid_amd import _abi
    assert set(_abi.STATE_INIT) == {"Default", "Start", "Random", "Hybrid"}
    with pytest.raises(ValueError, match="Unsupported state initialization"):
        HumanoidPHC(EnvConfig(num_envs=4, state_init="Middle"))
    for kw in (dict(has_upright_start=False), dict(has_shape_obs=True), dict(reduce_action=True), dict(has_mesh=True)):
        with pytest.raises(NotImplementedError, match="RobotConfig"):
            HumanoidPHC(EnvConfig(num_envs=4, robot=RobotConfig(**kw)))
    RobotConfig(has_smpl_pd_offset=True).check()  # supported (pd_action_offset_scale)


@pytest.mark.gpu
def test_state_init_default_through_the_env(model):
    """state_init=Default through HumanoidPHC / PHCPufferEnv: the full reset puts every env at its
    creation pose with zero dofs (humanoid_phc.py:688-692) and the motion start times stay at their
    loaded values; under random actions the fused device resets bring failed envs back there."""
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    n = 32
    pe = PHCPufferEnv(EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=5, state_init="Default"))
    pe.reset()
    e = pe.env
    init = e.engine.initial_root_states.clone()
    assert (e.engine.root_states == init).all()
    assert (e.engine.dof_state == 0).all()
    rng = np.random.default_rng(2)
    resets = 0
    for _ in range(20):
        pe.step(rng.uniform(-1, 1, (n, 69)).astype(np.float32))
        r = e.reset_buf.clone()
        resets += int(r.sum())
        if r.any():
            assert (e.engine.root_states[r] == init[r]).all()
            assert (e.engine.dof_state.view(n, 69, 2)[r] == 0).all()
    assert resets > 0
    pe.close()


@pytest.mark.gpu
def test_state_init_start_and_obs_noise(model):
    """state_init=Start: every reset (the full reset and the fused device resets of PHCPufferEnv)
    starts the motion at time 0 (humanoid_phc.py:850-851); add_obs_noise adds N(0, 0.1) to the
    observations while training (humanoid_phc.py:956)."""
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    n = 32
    pe = PHCPufferEnv(EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=5, state_init="Start"))
    pe.reset()
    e = pe.env
    assert (e._motion_start_times == 0).all()
    rng = np.random.default_rng(1)
    resets = 0
    for _ in range(20):
        pe.step(rng.uniform(-1, 1, (n, 69)).astype(np.float32))
        r = e.reset_buf.clone()
        resets += int(r.sum())
        assert (e._motion_start_times[r] == 0).all()
    assert resets > 0
    pe.close()
    clean = PHCPufferEnv(EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=5))
    noisy = PHCPufferEnv(EnvConfig(num_envs=n, motion_file=_clip_dict(model), seed=5, add_obs_noise=True))
    o0, _ = clean.reset()
    o1, _ = noisy.reset()
    d = (o1 - o0).float()
    assert abs(float(d.std()) - 0.1) < 0.01 and abs(float(d.mean())) < 0.01
    clean.close()
    noisy.close()
