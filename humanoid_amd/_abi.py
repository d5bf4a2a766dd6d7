"""ctypes mirrors of ``include/humanoid_engine.h`` and helpers to fill them.

Pure data-contract code: the product shim (``engine.py``) and the test-side oracle wrapper
(``oracle/oracle.py``) both use these layouts.
"""
import ctypes as C

import numpy as np

from .model import HumanoidModel

NB, ND, NG = 24, 69, 75
MAX_PAIRS = 256
OBS_SELF, OBS_TASK, OBS_DIM = 358, 576, 934

(BUF_ROOT_STATE, BUF_DOF_STATE, BUF_RB_STATE, BUF_CONTACT_FORCE, BUF_DOF_FORCE, BUF_DOF_TARGET, BUF_NUM_CONTACTS,
 BUF_DROPPED_CONTACTS, BUF_CONTACT_CACHE, BUF_INIT_ROOT_STATE, BUF_PHYS_ORDER, BUF_PHYS_COST) = range(12)
# StateInit (envs/state_init.py) -> he_imitation_params.state_init
STATE_INIT = {"Default": 0, "Start": 1, "Random": 2, "Hybrid": 3}
CACHE_WORDS, CACHE_KEYS, CACHE_LAMBDA = 104, 8, 40  # he_sim_params warm-start cache layout (row keys, impulses)
MAX_CONTACTS, MAX_ROWS = 40, 63
KEY_PATCH = 15  # row key sub-index of a body's terrain-patch friction rows


def cache_rows(cache):
    """Rows of warm-start caches [N, CACHE_WORDS] (include/humanoid_engine.h): row counts [N],
    16-bit row keys [N, MAX_ROWS] (int64, -1 past the count) and impulses [N, MAX_ROWS]."""
    c = np.ascontiguousarray(cache, np.float32)
    n = c[:, 7].view(np.int32).copy()
    kw = c[:, CACHE_KEYS:CACHE_KEYS + (MAX_ROWS + 1) // 2].view(np.uint32)
    keys = np.stack([kw & 0xFFFF, kw >> 16], -1).reshape(c.shape[0], -1)[:, :MAX_ROWS].astype(np.int64)
    lam = c[:, CACHE_LAMBDA:CACHE_LAMBDA + MAX_ROWS].copy()
    keys[np.arange(MAX_ROWS)[None, :] >= n[:, None]] = -1
    return n, keys, lam


def key_fields(key):
    """(body0, body1, sub, kind) of a 16-bit row key: body1 -1 terrain, -2 joint limit; kind 0
    normal, 1 / 2 tangential, 3 torsional."""
    key = int(key)
    return key & 31, ((key >> 5) & 31) - 2, (key >> 10) & 15, key >> 14
DTYPE_F32, DTYPE_I32 = 1, 2


class HeModel(C.Structure):
    _fields_ = [
        ("num_bodies", C.c_int32), ("num_dof", C.c_int32), ("num_pairs", C.c_int32), ("reserved", C.c_int32),
        ("parents", C.c_int32 * NB), ("geom_type", C.c_int32 * NB),
        ("local_pos", (C.c_float * 3) * NB), ("mass", C.c_float * NB), ("com", (C.c_float * 3) * NB),
        ("inertia", (C.c_float * 6) * NB), ("geom_params", (C.c_float * 10) * NB), ("geom_radius", C.c_float * NB),
        ("stiffness", C.c_float * ND), ("damping", C.c_float * ND), ("armature", C.c_float * ND),
        ("effort", C.c_float * ND), ("pairs", (C.c_int32 * 2) * MAX_PAIRS),
        ("dof_lower", C.c_float * ND), ("dof_upper", C.c_float * ND),
    ]


class HeSimParams(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("gravity", C.c_float * 3), ("contact_offset", C.c_float), ("friction", C.c_float),
        ("baumgarte", C.c_float), ("max_depenetration_velocity", C.c_float), ("angular_damping", C.c_float),
        ("max_angular_velocity", C.c_float), ("solver_iterations", C.c_int32), ("self_collision", C.c_int32),
        ("max_contacts", C.c_int32), ("kp_scale", C.c_float), ("kd_scale", C.c_float), ("terrain", C.c_int32),
        ("terrain_slope", C.c_float), ("step_height", C.c_float), ("step_length", C.c_float),
        ("joint_limits", C.c_int32), ("limit_margin", C.c_float), ("warm_start", C.c_int32), ("solver_tolerance", C.c_float),
        ("bias_midpoint", C.c_int32), ("substeps", C.c_int32), ("max_joint_velocity", C.c_float),
        ("solver_type", C.c_int32),
    ]


class HeImitationParams(C.Structure):
    _fields_ = [
        ("k_pos", C.c_float), ("k_rot", C.c_float), ("k_vel", C.c_float), ("k_ang_vel", C.c_float),
        ("w_pos", C.c_float), ("w_rot", C.c_float), ("w_vel", C.c_float), ("w_ang_vel", C.c_float),
        ("power_coef", C.c_float), ("use_power_reward", C.c_int32), ("control_dt", C.c_float),
        ("enable_early_termination", C.c_int32), ("eval_mode", C.c_int32), ("reset_body_mask", C.c_int32),
        ("term_dist", C.c_float * NB), ("state_init", C.c_int32), ("hybrid_init_prob", C.c_float),
        ("test_mode", C.c_int32), ("reserved", C.c_int32),
    ]


class HeEnvMotion(C.Structure):
    _fields_ = [("motion_ids", C.c_void_p), ("start_times", C.c_void_p), ("start_offsets", C.c_void_p),
                ("global_offset", C.c_void_p), ("progress", C.c_void_p)]


def make_model(m: HumanoidModel) -> HeModel:
    if m.num_bodies != NB or m.num_dof != ND:
        raise ValueError(f"engine is built for {NB} bodies / {ND} dofs, model has {m.num_bodies}/{m.num_dof}")
    hm = HeModel()
    pairs = m.self_collision_pairs()
    if len(pairs) > MAX_PAIRS:
        raise ValueError("too many self-collision pairs")
    hm.num_bodies, hm.num_dof, hm.num_pairs = NB, ND, len(pairs)
    for b in range(NB):
        hm.parents[b] = int(m.parents[b])
        hm.geom_type[b] = int(m.geom_type[b])
        hm.mass[b] = float(m.mass[b])
        hm.geom_radius[b] = float(m.geom_radius[b])
        for c in range(3):
            hm.local_pos[b][c] = float(m.local_pos[b, c])
            hm.com[b][c] = float(m.com[b, c])
        I = m.inertia[b]
        for c, v in enumerate((I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2])):
            hm.inertia[b][c] = float(v)
        for c in range(10):
            hm.geom_params[b][c] = float(m.geom_params[b, c])
    for d in range(ND):
        hm.stiffness[d] = float(m.stiffness[d])
        hm.damping[d] = float(m.damping[d])
        hm.armature[d] = float(m.armature[d])
        hm.effort[d] = float(m.effort[d])
        hm.dof_lower[d] = float(m.dof_lower[d])
        hm.dof_upper[d] = float(m.dof_upper[d])
    for i, (a, b) in enumerate(pairs):
        hm.pairs[i][0], hm.pairs[i][1] = int(a), int(b)
    return hm


def default_sim_params(**kw) -> HeSimParams:
    """isaacgym_env.py:6-35 and asset options humanoid_phc.py:211-214 (engine defaults)."""
    p = HeSimParams()
    p.dt = 1.0 / 60.0
    p.gravity[:] = (0.0, 0.0, -9.81)
    p.contact_offset = 0.02
    p.friction = 1.0
    p.baumgarte = 0.2
    p.max_depenetration_velocity = 10.0
    p.angular_damping = 0.01
    p.max_angular_velocity = 100.0
    p.solver_iterations = 4  # TGS position iterations per physics step (num_position_iterations, isaacgym_env.py:17)
    p.self_collision = 1
    p.max_contacts = 40
    p.kp_scale = 1.0
    p.kd_scale = 1.0
    p.terrain = 0
    p.terrain_slope = float(np.deg2rad(10.0))
    p.step_height = 0.05
    p.step_length = 0.4
    p.joint_limits = 1  # the MJCF ranges, enforced by PhysX (humanoid_phc.py:305-324)
    p.limit_margin = 0.1
    p.warm_start = 1
    p.solver_tolerance = 0.0
    p.bias_midpoint = 1  # explicit bias pumps energy under per-step random targets
    p.substeps = 2  # gymapi.SimParams.substeps default (not set by isaacgym_env.py:6-35)
    p.max_joint_velocity = 100.0  # PhysX articulation joint maxJointVelocity default
    p.solver_type = 1  # TGS, the reference's solver (isaacgym_env.py:16-18); 0: PGS (pgs_sim_params)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def pgs_sim_params(**kw) -> HeSimParams:
    """The engine's velocity-level PGS step (solver_type 0, 8 warm-started sweeps per 1/120 s physics
    step, the midpoint bias; rounds 1-4's default) instead of the reference's TGS."""
    kw.setdefault("solver_type", 0)
    kw.setdefault("solver_iterations", 8)
    return default_sim_params(**kw)


def imitation_params(reward=None, control_dt=1.0 / 30.0, use_power_reward=True, power_coef=0.0005,
                     enable_early_termination=True, eval_mode=False, termination_distance=0.25,
                     reset_body_ids=None, state_init="Random", hybrid_init_prob=0.5,
                     test_mode=False) -> HeImitationParams:
    """config.py:37-50 (RewardConfig), :97-112, :114, :139 (EnvConfig) defaults. state_init is a
    StateInit name (state_init.py); test_mode = flag_test (reference-state inits at motion time 0)."""
    r = dict(k_pos=100.0, k_rot=10.0, k_vel=0.1, k_ang_vel=0.1, w_pos=0.5, w_rot=0.3, w_vel=0.1, w_ang_vel=0.1)
    if reward:
        r.update({k: v for k, v in reward.items() if k in r})
    p = HeImitationParams(**r)
    p.power_coef = power_coef
    p.use_power_reward = int(use_power_reward)
    p.control_dt = control_dt
    p.enable_early_termination = int(enable_early_termination)
    p.eval_mode = int(eval_mode)
    ids = range(NB) if reset_body_ids is None else reset_body_ids
    mask = 0
    for b in ids:
        mask |= 1 << int(b)
    p.reset_body_mask = mask
    td = np.broadcast_to(np.asarray(termination_distance, np.float32), (NB,))
    for b in range(NB):
        p.term_dist[b] = float(td[b])
    if state_init not in STATE_INIT:
        raise ValueError(f"Unsupported state initialization strategy: {state_init}")
    p.state_init = STATE_INIT[state_init]
    p.hybrid_init_prob = float(hybrid_init_prob)
    p.test_mode = int(bool(test_mode))
    return p


# include/humanoid_rollout.h
ROLLOUT_MAX_FIELDS = 8
ROLLOUT_F32 = 0
ROLLOUT_U8 = 1


class HeRolloutField(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("width", C.c_int32), ("src_kind", C.c_int32)]


class HeRolloutIndex(C.Structure):
    _fields_ = [("num_keys", C.c_int32), ("reserved", C.c_int32), ("capacity", C.c_int64),
                ("scratch_rows", C.c_int64), ("key_count", C.c_void_p), ("key_last", C.c_void_p),
                ("key_offset", C.c_void_p), ("row_env", C.c_void_p), ("row_rank", C.c_void_p),
                ("scratch", C.c_void_p), ("status", C.c_void_p)]


# include/humanoid_engine.h he_eval_buffers
EVAL_SUMS = 8


class HeEvalBuffers(C.Structure):
    _fields_ = [("num_steps", C.c_void_p), ("mpjpe", C.c_void_p), ("body_pos", C.c_void_p),
                ("body_pos_gt", C.c_void_p), ("history", C.c_void_p), ("sums", C.c_void_p),
                ("frame", C.c_int32), ("reserved", C.c_int32)]


AMP_OBS_STEP = 196  # include/humanoid_engine.h HE_AMP_OBS_STEP


class HeAmpBuffers(C.Structure):
    """include/humanoid_engine.h he_amp_buffers (device pointers)."""
    _fields_ = [("amp_obs", C.c_void_p), ("amp_obs_demo", C.c_void_p), ("num_steps", C.c_int32),
                ("reserved", C.c_int32)]
