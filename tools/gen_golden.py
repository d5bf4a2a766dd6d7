"""Generate the golden fixtures under ``tests/golden/`` by running the reference's own code.

Build-container only (``/root/reference`` does not exist on the GPU box). The reference's
pure-torch modules are imported from ``/root/reference/packages/puffer-phc``; only the absent
third-party imports (``isaacgym``, ``gym``, ``tyro``, ``smpl_sim``) are replaced by empty stub
modules so that ``humanoid_phc.py`` can be imported. No reference method that touches the
simulator is called: the env-level fixtures call ``HumanoidPHC._compute_reward``,
``_compute_reset``, ``_compute_observations``, ``_reset_ref_state_init``,
``_build_pd_action_offset_scale`` and ``_action_to_pd_targets`` on an instance created with
``__new__`` whose state tensors are plain CPU tensors filled by this script.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
        PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py amp     (one part only)
Writes: tests/golden/{quat_prims,skeleton,motion_lib,imitation_funcs,env_step,env_reset,pd_targets,amp,
        state_init}.npz
"""
import os
import sys
import tempfile
import types
from types import SimpleNamespace

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/packages/puffer-phc"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Sub:
        def __getitem__(self, x):
            return x

    mod("smpl_sim")
    mod("smpl_sim.smpllib")
    mod("smpl_sim.smpllib.smpl_parser", SMPL_Parser=object)
    gymapi = mod("isaacgym.gymapi")
    gymtorch = mod("isaacgym.gymtorch")
    mod("isaacgym", gymapi=gymapi, gymtorch=gymtorch)
    sys.modules.setdefault("gymtorch", gymtorch)
    spaces = mod("gym.spaces")
    mod("gym", spaces=spaces)
    conf = mod("tyro.conf", Suppress=_Sub(), Fixed=_Sub())
    mod("tyro", conf=conf)
    sys.path.insert(0, REF)


install_stubs()

from puffer_phc import torch_utils as TU  # noqa: E402
from puffer_phc.envs import common as C  # noqa: E402
from puffer_phc.poselib_skeleton import SkeletonTree  # noqa: E402
from puffer_phc import motion_lib as ML  # noqa: E402
from puffer_phc.config import EnvConfig  # noqa: E402
from puffer_phc.envs.humanoid_phc import HumanoidPHC  # noqa: E402
from puffer_phc.envs.state_init import StateInit  # noqa: E402
from puffer_phc import body_sets as BS  # noqa: E402

from humanoid_amd.model import parse_mjcf  # noqa: E402
from humanoid_amd import synthetic  # noqa: E402

XML = os.path.join(REF, "puffer_phc/assets/smpl_humanoid.xml")


def t2n(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def rand_quat(g, n):
    q = torch.randn(n, 4, generator=g)
    return q / q.norm(dim=-1, keepdim=True)


# --------------------------------------------------------------------------------- quats
def gen_quat_prims():
    g = torch.Generator().manual_seed(1)
    n = 256
    q = rand_quat(g, n)
    # edge cases: identity, -identity, w ~ +-1, w ~ 0, 180 deg about axes, tiny angles
    edge = torch.tensor([
        [0, 0, 0, 1], [0, 0, 0, -1], [1e-6, 0, 0, 1], [0, 1e-7, 0, -1], [1, 0, 0, 0], [0, 1, 0, 0],
        [0, 0, 1, 0], [0.7071068, 0, 0, 0.7071068], [0, 0, 0.7071068, -0.7071068],
        [3e-5, -2e-5, 1e-5, 1.0], [0.5, 0.5, 0.5, 0.5], [-0.5, 0.5, -0.5, 0.5],
    ], dtype=torch.float32)
    edge = edge / edge.norm(dim=-1, keepdim=True)
    q = torch.cat([q, edge])
    r = torch.cat([rand_quat(g, n), rand_quat(g, edge.shape[0])])
    v = torch.randn(q.shape[0], 3, generator=g) * 2
    e = torch.randn(q.shape[0], 3, generator=g) * 1.5
    e[:4] = torch.tensor([[0, 0, 0], [1e-7, 0, 0], [3.14159, 0, 0], [0, 0, 6.5]])
    t = torch.rand(q.shape[0], 1, generator=g)
    t[:3] = torch.tensor([[0.0], [1.0], [0.5]])
    r_close = q + 1e-4 * torch.randn(q.shape, generator=g)
    r_close = r_close / r_close.norm(dim=-1, keepdim=True)
    r_close[::2] = -r_close[::2]  # exercise slerp's negative-dot branch
    ang, axis = TU.quat_to_angle_axis(q)
    out = dict(
        q=q, r=r, v=v, e=e, t=t, r_close=r_close,
        quat_mul=TU.quat_mul(q, r), quat_conjugate=TU.quat_conjugate(q),
        my_quat_rotate=TU.my_quat_rotate(q, v), quat_to_tan_norm=TU.quat_to_tan_norm(q),
        angle=ang, axis=axis, quat_to_exp_map=TU.quat_to_exp_map(q),
        exp_map_to_quat=TU.exp_map_to_quat(e),
        slerp=TU.slerp(q, r, t), slerp_close=TU.slerp(q, r_close, t),
        calc_heading=TU.calc_heading(q), calc_heading_quat=TU.calc_heading_quat(q),
        calc_heading_quat_inv=TU.calc_heading_quat_inv(q),
        normalize_angle=TU.normalize_angle(e[:, 0] * 3),
    )
    np.savez_compressed(os.path.join(OUT, "quat_prims.npz"), **{k: t2n(v) for k, v in out.items()})


# --------------------------------------------------------------------------------- skeleton
def gen_skeleton():
    tree = SkeletonTree.from_mjcf(XML)
    np.savez_compressed(os.path.join(OUT, "skeleton.npz"), parents=t2n(tree.parent_indices),
                        local_translation=t2n(tree.local_translation),
                        node_names=np.array(tree.node_names))
    return tree


# --------------------------------------------------------------------------------- motion lib
CLIP_FRAMES = [40, 31, 24, 12]


def make_clips():
    model = parse_mjcf(XML)
    rng = np.random.default_rng(7)
    clips = {}
    for i, nf in enumerate(CLIP_FRAMES):
        c = synthetic.make_clip(model, rng, num_frames=nf)
        clips[f"clip{i}"] = c
    clips["standstill"] = synthetic.make_standstill_clip(model, num_frames=20)
    return clips


def to_ref_schema(clips):
    out = {}
    for k, c in clips.items():
        d = dict(c)
        d["root_trans_offset"] = torch.from_numpy(np.asarray(c["root_trans_offset"], np.float32))
        out[k] = d
    return out


def build_motion_lib(tree, clips, sample_idxes, device="cpu"):
    fd, path = tempfile.mkstemp(suffix=".pkl")
    os.close(fd)
    import joblib
    joblib.dump(to_ref_schema(clips), path)
    cfg = SimpleNamespace(motion_file=path, device=device, fix_height=ML.FixHeightMode.full_fix,
                          min_length=5, max_length=300, im_eval=False, num_thread=1, smpl_type="smpl",
                          step_dt=1 / 30, is_deterministic=True)
    lib = ML.MotionLibSMPL(cfg, "/nonexistent_smpl_dir")
    n = len(sample_idxes)
    lib.load_motions(skeleton_trees=[tree] * n, gender_betas=torch.zeros(n, 17),
                     limb_weights=torch.zeros(n, 10), random_sample=False,
                     sample_idxes=torch.tensor(sample_idxes))
    os.unlink(path)
    return lib


def gen_motion_lib(tree):
    clips = make_clips()
    keys = list(clips.keys())
    sample = [0, 1, 2, 3, 4, 0, 2]
    lib = build_motion_lib(tree, clips, sample)
    g = torch.Generator().manual_seed(3)
    K = 96
    ids = torch.randint(0, len(sample), (K,), generator=g)
    lens = lib._motion_lengths[ids]
    times = torch.rand(K, generator=g) * (lens + 0.2) - 0.1
    # exact frame multiples like the env produces: progress*dt + start (float32 ops)
    prog = torch.randint(0, 40, (K // 2,), generator=g).to(torch.int16)
    start = ((torch.rand(K // 2, generator=g) * lens[: K // 2]) / (1 / 30)).long() * (1 / 30)
    times[: K // 2] = prog * (1 / 30) + start + torch.zeros(K // 2)
    offset = torch.randn(K, 3, generator=g) * 0.3
    res = lib.get_motion_state(ids, times, offset)
    res_no = lib.get_motion_state(ids, times, None)
    # sample_time_interval with a recorded phase stream
    torch.manual_seed(11)
    phases = torch.rand(K)
    torch.manual_seed(11)
    st = lib.sample_time_interval(ids)
    out = dict(
        clip_keys=np.array(keys), sample_idxes=np.array(sample),
        gts=lib.gts, grs=lib.grs, lrs=lib.lrs, gvs=lib.gvs, gavs=lib.gavs, dvs=lib.dvs,
        length_starts=lib.length_starts, num_frames=lib._motion_num_frames,
        motion_lengths=lib._motion_lengths, motion_dt=lib._motion_dt, motion_fps=lib._motion_fps,
        q_ids=ids, q_times=times, q_offset=offset, phases=phases, sample_time_interval=st,
        num_steps=lib.get_motion_num_steps(),
    )
    for k, v in res.items():
        out["ms_" + k] = v
    for k in ("rg_pos", "root_pos"):
        out["msno_" + k] = res_no[k]
    # the clips themselves (inputs for the host loader parity test)
    for i, (k, c) in enumerate(clips.items()):
        out[f"clip{i}_pose_quat_global"] = c["pose_quat_global"]
        out[f"clip{i}_root_trans_offset"] = c["root_trans_offset"]
        out[f"clip{i}_fps"] = np.array(c["fps"])
    np.savez_compressed(os.path.join(OUT, "motion_lib.npz"), **{k: t2n(v) for k, v in out.items()})
    return clips, lib


# --------------------------------------------------------------------------------- obs/reward
def gen_imitation_funcs():
    g = torch.Generator().manual_seed(5)
    N, B = 64, 24

    def state(scale=1.0):
        return (torch.randn(N, B, 3, generator=g) * scale, rand_quat(g, N * B).view(N, B, 4),
                torch.randn(N, B, 3, generator=g), torch.randn(N, B, 3, generator=g))

    bp, br, bv, bav = state()
    bp[..., 2] += 0.9
    rp = bp + torch.randn(N, B, 3, generator=g) * torch.linspace(0.01, 0.5, N).view(N, 1, 1)
    rr = rand_quat(g, N * B).view(N, B, 4)
    rr[: N // 2] = br[: N // 2] + 0.05 * torch.randn(N // 2, B, 4, generator=g)
    rr = rr / rr.norm(dim=-1, keepdim=True)
    rv = bv + torch.randn(N, B, 3, generator=g)
    rav = bav + torch.randn(N, B, 3, generator=g)
    specs = {"k_pos": 100.0, "k_rot": 10.0, "k_vel": 0.1, "k_ang_vel": 0.1,
             "w_pos": 0.5, "w_rot": 0.3, "w_vel": 0.1, "w_ang_vel": 0.1}
    rew, raw = C.compute_imitation_reward(bp[:, 0], br[:, 0], bp, br, bv, bav, rp, rr, rv, rav, specs)
    progress = torch.randint(0, 5, (N,), generator=g).to(torch.int16)
    pass_time = torch.rand(N, generator=g) < 0.2
    reset_buf = torch.zeros(N, dtype=torch.bool)
    contact = torch.zeros(N, B, 3)
    cids = torch.tensor([7, 3, 8, 4])
    td = torch.full((B,), 0.25)
    reset, term = C.compute_humanoid_im_reset(reset_buf, progress, contact, cids, bp, rp, pass_time, True, td, False)
    ev = torch.tensor(BS.build_body_ids_tensor(BS.BODY_NAMES, BS.EVAL_BODIES, "cpu"))
    td5 = torch.full((len(ev),), 0.5)
    reset_e, term_e = C.compute_humanoid_im_reset(reset_buf, progress, contact, cids, bp[:, ev], rp[:, ev],
                                                  pass_time, True, td5, True)
    self_obs = C.compute_humanoid_observations_smpl_max(bp, br, bv, bav, None, None, True, True, True, False, False)
    task_obs = C.compute_imitation_observations_v6(bp[:, 0], br[:, 0], bp, br, bv, bav, rp, rr, rv, rav, 1, True)
    out = dict(body_pos=bp, body_rot=br, body_vel=bv, body_ang_vel=bav, ref_pos=rp, ref_rot=rr, ref_vel=rv,
               ref_ang_vel=rav, rew=rew, reward_raw=raw, progress=progress, pass_time=pass_time,
               reset=reset, terminate=term, reset_eval=reset_e, terminate_eval=term_e, eval_ids=ev,
               self_obs=self_obs, task_obs=task_obs)
    np.savez_compressed(os.path.join(OUT, "imitation_funcs.npz"), **{k: t2n(v) for k, v in out.items()})


# --------------------------------------------------------------------------------- env glue
def fake_env(lib, tree, N):
    env = HumanoidPHC.__new__(HumanoidPHC)
    cfg = EnvConfig(device_type="cpu", num_envs=N)
    env.cfg = cfg
    env.isaac_base = SimpleNamespace(dt=1 / 30, control_freq_inv=2)
    env.num_bodies, env.num_dof = 24, 69
    env.all_env_ids = torch.arange(N)
    env._motion_lib = lib
    env._motion_train_lib = lib
    env.ref_motion_cache = {}
    env.flag_test = False
    env.flag_im_eval = False
    env.flag_debug = True
    env._config_env()
    env._dof_offsets = np.linspace(0, 69, 24).astype(int)
    env.humanoid_shapes = torch.zeros(N, 17)
    env.humanoid_limb_and_weights = torch.zeros(N, 10)
    env._root_states = torch.zeros(N, 13)
    env._humanoid_root_states = env._root_states.view(N, 1, 13)[..., 0, :]
    env._dof_state = torch.zeros(N * 69, 2)
    env._dof_pos = env._dof_state.view(N, 69, 2)[..., 0]
    env._dof_vel = env._dof_state.view(N, 69, 2)[..., 1]
    env._rigid_body_state = torch.zeros(N * 24, 13)
    rbs = env._rigid_body_state.view(N, 24, 13)
    env._rigid_body_pos = rbs[..., 0:3]
    env._rigid_body_rot = rbs[..., 3:7]
    env._rigid_body_vel = rbs[..., 7:10]
    env._rigid_body_ang_vel = rbs[..., 10:13]
    env._contact_forces = torch.zeros(N, 24, 3)
    env.dof_force_tensor = torch.zeros(N, 69)
    env.obs_buf = torch.zeros(N, 934)
    env.rew_buf = torch.zeros(N)
    env.reward_raw = torch.zeros(N, 5)
    env.progress_buf = torch.zeros(N, dtype=torch.short)
    env.reset_buf = torch.ones(N, dtype=torch.bool)
    env._terminate_buf = torch.ones(N, dtype=torch.bool)
    env.extras = {}
    env._global_offset = torch.zeros(N, 3)
    env._motion_start_times = torch.zeros(N)
    env._motion_start_times_offset = torch.zeros(N)
    env._sampled_motion_ids = torch.arange(N) % lib._motion_lengths.shape[0]
    env.ref_dof_pos = torch.zeros(N, 69)
    return env


def gen_env(tree, clips):
    g = torch.Generator().manual_seed(9)
    N = 24
    sample = [i % 5 for i in range(N)]
    lib = build_motion_lib(tree, clips, sample)
    env = fake_env(lib, tree, N)
    env._sampled_motion_ids = torch.arange(N)
    lens = lib._motion_lengths
    env._motion_start_times[:] = ((torch.rand(N, generator=g) * lens) / (1 / 30)).long() * (1 / 30)
    env._motion_start_times_offset[:] = torch.where(torch.rand(N, generator=g) < 0.2,
                                                    torch.rand(N, generator=g) * 0.05, torch.zeros(N))
    env._global_offset[:] = torch.randn(N, 3, generator=g) * 0.1 * (torch.rand(N, 1, generator=g) < 0.5)
    env.progress_buf[:] = torch.randint(0, 30, (N,), generator=g).to(torch.short)
    # sim state = reference state at the step's time + per-env noise (some envs fall)
    t_next = (env.progress_buf + 1) * env.isaac_base.dt + env._motion_start_times + env._motion_start_times_offset
    ms = lib.get_motion_state(env._sampled_motion_ids, t_next, env._global_offset)
    noise = torch.linspace(0.0, 0.2, N).view(N, 1, 1)
    env._rigid_body_pos[:] = ms["rg_pos"] + noise * torch.randn(N, 24, 3, generator=g)
    rot = ms["rb_rot"] + 0.5 * noise * torch.randn(N, 24, 4, generator=g)
    env._rigid_body_rot[:] = rot / rot.norm(dim=-1, keepdim=True)
    env._rigid_body_vel[:] = ms["body_vel"] + 5 * noise * torch.randn(N, 24, 3, generator=g)
    env._rigid_body_ang_vel[:] = ms["body_ang_vel"] + 5 * noise * torch.randn(N, 24, 3, generator=g)
    env._dof_vel[:] = torch.randn(N, 69, generator=g)
    env.dof_force_tensor[:] = torch.randn(N, 69, generator=g) * 50
    inputs = dict(
        motion_ids=env._sampled_motion_ids.clone(), start_times=env._motion_start_times.clone(),
        start_offsets=env._motion_start_times_offset.clone(), global_offset=env._global_offset.clone(),
        progress_in=env.progress_buf.clone(), rb_state=env._rigid_body_state.view(N, 24, 13).clone(),
        dof_vel=env._dof_vel.clone(), dof_force=env.dof_force_tensor.clone(),
        gts=lib.gts, grs=lib.grs, lrs=lib.lrs, gvs=lib.gvs, gavs=lib.gavs, dvs=lib.dvs,
        length_starts=lib.length_starts, num_frames=lib._motion_num_frames,
        motion_lengths=lib._motion_lengths, motion_dt=lib._motion_dt,
    )
    # --- HumanoidPHC.step post-physics half (humanoid_phc.py:138-152)
    env.progress_buf += 1
    env._compute_reward()
    env._compute_reset()
    env._compute_observations()
    outputs = dict(progress_out=env.progress_buf, rew=env.rew_buf, reward_raw=env.reward_raw,
                   reset=env.reset_buf, terminate=env._terminate_buf, obs=env.obs_buf)
    # --- eval-mode reset variant (humanoid_phc.py:1426-1437)
    env2 = fake_env(lib, tree, N)
    for k in ("_sampled_motion_ids", "_motion_start_times", "_motion_start_times_offset", "_global_offset",
              "progress_buf", "dof_force_tensor"):
        getattr(env2, k).copy_(getattr(env, k))
    env2._rigid_body_state.copy_(env._rigid_body_state)
    env2._dof_state.copy_(env._dof_state)
    env2.flag_im_eval = True
    env2.set_termination_distances(0.5)
    env2._reset_bodies_id = env2._eval_track_bodies_id
    env2._compute_reset()
    outputs["reset_eval"] = env2.reset_buf
    outputs["terminate_eval"] = env2._terminate_buf
    out = {**inputs, **outputs}
    np.savez_compressed(os.path.join(OUT, "env_step.npz"), **{k: t2n(v) for k, v in out.items()})

    # --- reset path: _reset_ref_state_init + _reset_env_tensors bookkeeping + obs (humanoid_phc.py:665-731)
    env3 = fake_env(lib, tree, N)
    env3._sampled_motion_ids = torch.arange(N)
    env3.cfg.state_init = StateInit.Random
    env3._global_offset[:] = inputs["global_offset"]
    env3._rigid_body_state.copy_(env._rigid_body_state)
    env3.progress_buf[:] = 7
    env_ids = torch.tensor([0, 3, 4, 9, 10, 17, 23])
    torch.manual_seed(21)
    phases = torch.rand(len(env_ids))
    torch.manual_seed(21)
    env3._reset_ref_state_init(env_ids)
    env3.progress_buf[env_ids] = 0
    env3._compute_observations(env_ids)
    out = dict(env_ids=env_ids, phases=phases, global_offset_in=inputs["global_offset"],
               rb_state_in=env._rigid_body_state.view(N, 24, 13),
               root_states=env3._root_states, dof_pos=env3._dof_pos, dof_vel=env3._dof_vel,
               rb_state=env3._rigid_body_state.view(N, 24, 13), start_times=env3._motion_start_times,
               global_offset=env3._global_offset, obs=env3.obs_buf)
    np.savez_compressed(os.path.join(OUT, "env_reset.npz"), **{k: t2n(v) for k, v in out.items()})


def gen_pd():
    env = HumanoidPHC.__new__(HumanoidPHC)
    env.cfg = EnvConfig(device_type="cpu", num_envs=4)
    env._dof_offsets = np.linspace(0, 69, 24).astype(int)
    model = parse_mjcf(XML)
    env.dof_limits_lower = torch.tensor(model.dof_lower, dtype=torch.float32)
    env.dof_limits_upper = torch.tensor(model.dof_upper, dtype=torch.float32)
    env._build_pd_action_offset_scale()
    g = torch.Generator().manual_seed(4)
    a = torch.rand(32, 69, generator=g) * 2 - 1
    pd = env._action_to_pd_targets(a)
    for n in ("L_Hand", "R_Hand", "L_Toe", "R_Toe"):  # humanoid_phc.py:116-125
        i = BS.DOF_NAMES.index(n) * 3
        pd[:, i:i + 3] = 0
    np.savez_compressed(os.path.join(OUT, "pd_targets.npz"), offset=t2n(env._pd_action_offset),
                        scale=t2n(env._pd_action_scale), actions=t2n(a), pd_target=t2n(pd))


# --------------------------------------------------------------------------------- StateInit kinds
def zero_pose_rows(tree, init_root):
    """Rigid-body rows of the zero local pose at the given root states (the engine's Default-reset
    rows, an engine decision: the reference leaves the rb tensor to refresh), by the
    reference's own forward kinematics (poselib SkeletonState)."""
    from puffer_phc.poselib_skeleton import SkeletonState
    n = init_root.shape[0]
    r = torch.zeros(n, 24, 4)
    r[..., 3] = 1.0
    r[:, 0] = init_root[:, 3:7]
    sk = SkeletonState.from_rotation_and_root_translation(tree, r, init_root[:, 0:3], is_local=True)
    rows = torch.zeros(n, 24, 13)
    rows[..., 0:3] = sk.global_translation
    rows[..., 3:7] = sk.global_rotation
    return rows


def gen_state_init(tree, clips):
    """_reset_actors for StateInit Default / Start / Hybrid (humanoid_phc.py:679-745) followed by the
    _reset_env_tensors bookkeeping (:747-780) and _compute_observations(env_ids) (:937-961), on one
    pre-reset state. Hybrid's Bernoulli mask and the reference inits' phases are recorded (the
    torch RNG draws of torch.bernoulli and sample_time_interval after manual_seed). For Default envs
    the rb rows fed to the observation are the zero pose's rows at the initial root state (see
    zero_pose_rows): the reference reads whatever refresh returns there."""
    g = torch.Generator().manual_seed(13)
    N = 24
    lib = build_motion_lib(tree, clips, [i % 5 for i in range(N)])
    lens = lib._motion_lengths[torch.arange(N)]
    st0 = ((torch.rand(N, generator=g) * lens) / (1 / 30)).long() * (1 / 30)
    so0 = torch.where(torch.rand(N, generator=g) < 0.3, torch.rand(N, generator=g) * 0.05, torch.zeros(N))
    go0 = torch.randn(N, 3, generator=g) * 0.1
    prog0 = torch.randint(0, 30, (N,), generator=g).to(torch.short)
    root0 = torch.zeros(N, 13)
    root0[:, 0:2] = torch.rand(N, 2, generator=g) * 2 - 1
    root0[:, 2] = 0.9 + 0.2 * torch.rand(N, generator=g)
    q = torch.randn(N, 4, generator=g)
    root0[:, 3:7] = q / q.norm(dim=-1, keepdim=True)
    root0[:, 7:13] = torch.randn(N, 6, generator=g)
    dof0 = torch.randn(N, 69, 2, generator=g) * 0.3
    rb0 = torch.randn(N, 24, 13, generator=g)
    rb0[..., 3:7] = rb0[..., 3:7] / rb0[..., 3:7].norm(dim=-1, keepdim=True)
    init_root = torch.zeros(N, 13)  # creation poses (start xy jitter, z 0.89, a heading), zero velocity
    init_root[:, 0:2] = torch.rand(N, 2, generator=g) * 2 - 1
    init_root[:, 2] = 0.89
    yaw = (torch.rand(N, generator=g) * 2 - 1) * np.pi
    init_root[:, 5] = torch.sin(yaw / 2)
    init_root[:, 6] = torch.cos(yaw / 2)
    env_ids = torch.tensor([1, 2, 5, 8, 11, 12, 14, 19, 22, 23])
    out = dict(motion_ids=torch.arange(N), start_times_in=st0, start_offsets_in=so0, global_offset_in=go0,
               progress_in=prog0, root_in=root0, dof_in=dof0, rb_in=rb0, init_root=init_root, env_ids=env_ids,
               hybrid_init_prob=torch.tensor(0.5), motion_lengths=lib._motion_lengths, length_starts=lib.length_starts)
    for kind, seed in ((StateInit.Default, 31), (StateInit.Start, 32), (StateInit.Hybrid, 33)):
        env = fake_env(lib, tree, N)
        env._sampled_motion_ids = torch.arange(N)
        env._motion_start_times[:] = st0
        env._motion_start_times_offset[:] = so0
        env._global_offset[:] = go0
        env.progress_buf[:] = prog0
        env._root_states[:] = root0
        env._dof_state.view(N, 69, 2)[:] = dof0
        env._rigid_body_state.view(N, 24, 13)[:] = rb0
        env._initial_humanoid_root_states = init_root.clone()
        env._initial_dof_pos = torch.zeros(N, 69)
        env._initial_dof_vel = torch.zeros(N, 69)
        env.cfg.state_init = kind
        env.cfg.hybrid_init_prob = 0.5
        seen = {"default": torch.zeros(0, dtype=torch.long), "ref": torch.zeros(0, dtype=torch.long)}
        rd, rr = env._reset_default, env._reset_ref_state_init

        def rec_default(ids, rd=rd, seen=seen):
            seen["default"] = ids.clone()
            return rd(ids)

        def rec_ref(ids, rr=rr, seen=seen):
            seen["ref"] = ids.clone()
            return rr(ids)

        env._reset_default, env._reset_ref_state_init = rec_default, rec_ref
        # the draws the reference makes, in its order (torch.bernoulli, then sample_time_interval)
        torch.manual_seed(seed)
        mask = torch.ones(len(env_ids), dtype=torch.bool)
        phases = torch.zeros(len(env_ids))
        if kind == StateInit.Hybrid:
            mask = torch.bernoulli(torch.full((len(env_ids),), 0.5)) == 1.0
            phases[mask] = torch.rand(int(mask.sum()))
        elif kind == StateInit.Default:
            mask[:] = False
        torch.manual_seed(seed)
        env._reset_actors(env_ids)
        assert torch.equal(seen["ref"], env_ids[mask]) and torch.equal(seen["default"], env_ids[~mask])
        env.progress_buf[env_ids] = 0  # _reset_env_tensors (:775-780)
        env.reset_buf[env_ids] = 0
        env._terminate_buf[env_ids] = 0
        env._contact_forces[env_ids] = 0
        d = seen["default"]
        if len(d):
            env._rigid_body_state.view(N, 24, 13)[d] = zero_pose_rows(tree, init_root[d])
        env._compute_observations(env_ids)
        name = str(kind).split(".")[-1].lower()
        out.update({f"{name}_ref_mask": mask, f"{name}_phases": phases, f"{name}_root": env._root_states.clone(),
                    f"{name}_dof": env._dof_state.view(N, 69, 2).clone(),
                    f"{name}_rb": env._rigid_body_state.view(N, 24, 13).clone(),
                    f"{name}_start_times": env._motion_start_times.clone(),
                    f"{name}_start_offsets": env._motion_start_times_offset.clone(),
                    f"{name}_global_offset": env._global_offset.clone(), f"{name}_progress": env.progress_buf.clone(),
                    f"{name}_obs": env.obs_buf.clone()})
    np.savez_compressed(os.path.join(OUT, "state_init.npz"), **{k: t2n(v) for k, v in out.items()})


# --------------------------------------------------------------------------------- AMP obs (§8f-4)
def amp_dof_subset():
    # the index list HumanoidPHC._config_robot builds (humanoid_phc.py:186-194); that method also
    # creates gym assets, so the list is formed here from the same body sets
    idx = [np.arange(i * 3, (i + 1) * 3) for i, n in enumerate(BS.DOF_NAMES) if n not in BS.REMOVE_NAMES]
    return torch.from_numpy(np.concatenate(idx))


def gen_amp(tree, clips):
    """build_amp_observations_smpl (common.py:191-267) on random states, and the env-level AMP
    buffer flow: _update_hist_amp_obs + _compute_amp_observations after a step
    (humanoid_phc.py:154-157, 1125-1176, 1341-1350), then _init_amp_obs for a reset subset
    (:665-676, 791-838)."""
    g = torch.Generator().manual_seed(13)
    subset = amp_dof_subset()
    # -- function level
    N = 48
    root_pos = torch.randn(N, 3, generator=g) * 0.5
    root_pos[:, 2] += 0.9
    root_rot = rand_quat(g, N)
    root_vel = torch.randn(N, 3, generator=g)
    root_ang_vel = torch.randn(N, 3, generator=g) * 2
    dof_pos = torch.randn(N, 69, generator=g) * 1.2
    dof_pos[0] = 0.0                                   # exp map of zero: the default-axis branch
    dof_pos[1, :9] = 1e-7                              # below min_theta
    dof_pos[2, :3] = torch.tensor([3.14159, 0.0, 0.0])  # ~pi
    dof_pos[3, :3] = torch.tensor([0.0, 4.5, 0.0])      # > pi: normalize_angle wraps
    dof_pos[4, :3] = torch.tensor([0.0, 0.0, -7.0])     # > 2 pi
    dof_vel = torch.randn(N, 69, generator=g) * 3
    key_pos = root_pos[:, None, :] + torch.randn(N, 4, 3, generator=g) * 0.6
    shape = torch.zeros(N, 11)
    limb = torch.zeros(N, 10)
    amp = C.build_amp_observations_smpl(root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_pos,
                                        shape, limb, subset, True, True, True, False, False, True)
    out = dict(root_pos=root_pos, root_rot=root_rot, root_vel=root_vel, root_ang_vel=root_ang_vel,
               dof_pos=dof_pos, dof_vel=dof_vel, key_pos=key_pos, dof_subset=subset, amp_obs=amp)
    # -- env level
    NE, S = 24, 10
    sample = [i % 5 for i in range(NE)]
    lib = build_motion_lib(tree, clips, sample)
    env = fake_env(lib, tree, NE)
    env.cfg.use_amp_obs = True
    env.cfg.num_amp_obs_steps = S
    env.cfg.state_init = StateInit.Random
    env.dof_subset = subset
    env._reset_default_env_ids = []
    env._num_amp_obs_per_step = 13 + 23 * 6 + 69 + 3 * len(BS.KEY_BODIES) - (6 + 3) * 4  # :471-476
    env._amp_obs_buf = torch.randn(NE, S, env._num_amp_obs_per_step, generator=g)
    env._curr_amp_obs_buf = env._amp_obs_buf[:, 0]
    env._hist_amp_obs_buf = env._amp_obs_buf[:, 1:]
    env._amp_obs_demo_buf = torch.randn(NE, S, env._num_amp_obs_per_step, generator=g)
    lens = lib._motion_lengths
    env._motion_start_times[:] = ((torch.rand(NE, generator=g) * lens) / (1 / 30)).long() * (1 / 30)
    env._global_offset[:] = torch.randn(NE, 3, generator=g) * 0.1
    env.progress_buf[:] = torch.randint(0, 30, (NE,), generator=g).to(torch.short)
    t = env.progress_buf * env.isaac_base.dt + env._motion_start_times
    ms = lib.get_motion_state(env._sampled_motion_ids, t, env._global_offset)
    env._rigid_body_pos[:] = ms["rg_pos"] + 0.05 * torch.randn(NE, 24, 3, generator=g)
    rot = ms["rb_rot"] + 0.05 * torch.randn(NE, 24, 4, generator=g)
    env._rigid_body_rot[:] = rot / rot.norm(dim=-1, keepdim=True)
    env._rigid_body_vel[:] = ms["body_vel"] + torch.randn(NE, 24, 3, generator=g)
    env._rigid_body_ang_vel[:] = ms["body_ang_vel"] + torch.randn(NE, 24, 3, generator=g)
    env._dof_pos[:] = ms["dof_pos"] + 0.05 * torch.randn(NE, 69, generator=g)
    env._dof_vel[:] = ms["dof_vel"] + torch.randn(NE, 69, generator=g)
    out.update(env_motion_ids=env._sampled_motion_ids, env_start_times=env._motion_start_times.clone(),
               env_global_offset=env._global_offset.clone(), env_progress=env.progress_buf.clone(),
               env_rb_state=env._rigid_body_state.view(NE, 24, 13).clone(),
               env_dof_state=env._dof_state.view(NE, 69, 2).clone(), amp_buf_in=env._amp_obs_buf.clone(),
               amp_demo_in=env._amp_obs_demo_buf.clone(), num_amp_obs_steps=np.array(S))
    # step: HumanoidPHC.step's AMP tail (:154-157). The un-indexed branch of _update_hist_amp_obs
    # (:1341-1347) assigns between overlapping views of one buffer. The reference's comment there
    # records that its torch raised on that and it falls back to .clone(), i.e. a history shift; the
    # CPU torch of this container raises nothing and smears row 0 over every history row. The
    # indexed branch (:1349) gathers the source first, which is the shift for any torch, so the
    # fixture is taken through it with every env id.
    env._update_hist_amp_obs(env.all_env_ids)
    env._compute_amp_observations()
    out["amp_buf_step"] = env._amp_obs_buf.clone()
    # reset of a subset: _reset_ref_state_init (the env state) then _init_amp_obs (:665-676)
    env_ids = torch.tensor([1, 2, 5, 11, 16, 23])
    torch.manual_seed(31)
    phases = torch.rand(len(env_ids))
    torch.manual_seed(31)
    env._reset_ref_state_init(env_ids)
    env.progress_buf[env_ids] = 0
    env._init_amp_obs(env_ids)
    out.update(reset_ids=env_ids, reset_phases=phases, amp_buf_reset=env._amp_obs_buf.clone(),
               amp_demo_reset=env._amp_obs_demo_buf.clone(), reset_start_times=env._motion_start_times.clone(),
               env_rb_state_reset=env._rigid_body_state.view(NE, 24, 13).clone(),
               env_dof_state_reset=env._dof_state.view(NE, 69, 2).clone(),
               gts=lib.gts, grs=lib.grs, lrs=lib.lrs, gvs=lib.gvs, gavs=lib.gavs, dvs=lib.dvs,
               length_starts=lib.length_starts, num_frames=lib._motion_num_frames,
               motion_lengths=lib._motion_lengths, motion_dt=lib._motion_dt)
    np.savez_compressed(os.path.join(OUT, "amp.npz"), **{k: t2n(v) for k, v in out.items()})


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(1)
    if sys.argv[1:] == ["amp"]:
        tree = SkeletonTree.from_mjcf(XML)
        gen_amp(tree, make_clips())
        return
    if sys.argv[1:] == ["state_init"]:
        tree = SkeletonTree.from_mjcf(XML)
        gen_state_init(tree, make_clips())
        return
    gen_quat_prims()
    tree = gen_skeleton()
    clips, _ = gen_motion_lib(tree)
    gen_imitation_funcs()
    gen_env(tree, clips)
    gen_pd()
    gen_amp(tree, clips)
    gen_state_init(tree, clips)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
