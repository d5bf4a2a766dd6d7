"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle ``oracle/libhe_oracle.so``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module; the product path (``humanoid_amd``) never does. See ``he_oracle.c`` for what each
function restates (reference file:line) and which parts are pinned by golden vectors.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from humanoid_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhe_oracle.so")
_lib = None


def build(force=False):
    """Incremental make (no-op when up to date); falls back to a prebuilt .so without a compiler."""
    try:
        subprocess.run(["make", "-C", HERE] + (["-B"] if force else []), check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError):
        if not os.path.exists(LIB_PATH):
            raise
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(LIB_PATH)
        _lib.ho_hash_uniform.restype = C.c_float
        _lib.ho_hash_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        _lib.ho_sample_time_interval.restype = C.c_float
        _lib.ho_sample_time_interval.argtypes = [C.c_float, C.c_float]
    return _lib


def set_threads(n):
    """OpenMP threads of the oracle's parallel loops; returns the count in effect."""
    lib().ho_set_threads(int(n))
    return int(lib().ho_get_threads())


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def f32(a):
    return np.ascontiguousarray(a, np.float32)


class HoMotion(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("gts", "grs", "lrs", "gvs", "gavs", "dvs", "length_starts",
                                            "num_frames", "lengths", "dt")]


class MotionTables:
    """Keeps the numpy arrays alive behind the HoMotion struct."""

    def __init__(self, gts, grs, lrs, gvs, gavs, dvs, length_starts, num_frames, lengths, dt):
        self.arrays = dict(gts=f32(gts), grs=f32(grs), lrs=f32(lrs), gvs=f32(gvs), gavs=f32(gavs), dvs=f32(dvs),
                           length_starts=np.ascontiguousarray(length_starts, np.int64),
                           num_frames=np.ascontiguousarray(num_frames, np.int64), lengths=f32(lengths), dt=f32(dt))
        self.struct = HoMotion(**{k: _p(v) for k, v in self.arrays.items()})

    @classmethod
    def from_tables(cls, t):
        return cls(t.gts, t.grs, t.lrs, t.gvs, t.gavs, t.dvs, t.length_starts, t.num_frames, t.lengths, t.dt)


def quat_prims(q, r, v, e, t):
    n = q.shape[0]
    outs = dict(mul=(n, 4), rot=(n, 3), tan_norm=(n, 6), angle=(n,), axis=(n, 3), expmap=(n, 3), exp2q=(n, 4),
                slerp=(n, 4), heading=(n,), hq=(n, 4), hqi=(n, 4))
    res = {k: np.zeros(s, np.float32) for k, s in outs.items()}
    ins = [f32(q), f32(r), f32(v), f32(e), f32(t).reshape(-1)]
    lib().ho_quat_prims(C.c_int(n), *[_p(a) for a in ins], *[_p(res[k]) for k in outs])
    return res


def motion_state(mt: MotionTables, ids, times, offset=None):
    k = len(ids)
    ids = np.ascontiguousarray(ids, np.int64)
    times = f32(times)
    off = None if offset is None else f32(offset)
    out = dict(rg_pos=np.zeros((k, 24, 3), np.float32), rb_rot=np.zeros((k, 24, 4), np.float32),
               body_vel=np.zeros((k, 24, 3), np.float32), body_ang_vel=np.zeros((k, 24, 3), np.float32),
               dof_pos=np.zeros((k, 69), np.float32), dof_vel=np.zeros((k, 69), np.float32))
    lib().ho_motion_state(C.byref(mt.struct), C.c_int(k), _p(ids), _p(times), _p(off),
                          *[_p(out[n]) for n in ("rg_pos", "rb_rot", "body_vel", "body_ang_vel", "dof_pos", "dof_vel")])
    return out


def sample_time_interval(phase, length):
    return lib().ho_sample_time_interval(float(phase), float(length))


def hash_uniform(seed, step, env):
    return lib().ho_hash_uniform(seed, step, env)


def imitation_step(params, mt: MotionTables, rb_state, dof_vel, dof_force, progress, motion_ids, start_times,
                   start_offsets, global_offset):
    n = rb_state.shape[0]
    progress = np.ascontiguousarray(progress, np.int16).copy()
    out = dict(obs=np.zeros((n, 934), np.float32), rew=np.zeros(n, np.float32),
               reward_raw=np.zeros((n, 5), np.float32), reset=np.zeros(n, np.uint8), terminate=np.zeros(n, np.uint8))
    ins = [f32(rb_state), f32(dof_vel), f32(dof_force)]
    lib().ho_imitation_step(C.byref(params), C.byref(mt.struct), C.c_int(n), *[_p(a) for a in ins], _p(progress),
                            _p(np.ascontiguousarray(motion_ids, np.int64)), _p(f32(start_times)), _p(f32(start_offsets)),
                            _p(f32(global_offset)), _p(out["obs"]), _p(out["rew"]), _p(out["reward_raw"]),
                            _p(out["reset"]), _p(out["terminate"]))
    out["progress"] = progress
    return out


def rest_positions(model):
    """[24,3] body origins of the zero pose in the root frame (the joint offsets summed along each
    chain): the Default state init's rigid-body rows (he_engine.cpp he_set_model)."""
    rest = np.zeros((24, 3), np.float32)
    for b in range(1, 24):
        rest[b] = rest[model.parents[b]] + np.asarray(model.local_pos[b], np.float32)
    return rest


def reset_envs(params, mt: MotionTables, env_ids, phases, motion_ids, state, rest_pos=None):
    """state: dict of numpy arrays (modified in place): start_times, start_offsets, global_offset, progress,
    root_states [N,13], dof_state [N,69,2], dof_targets [N,69], rb_state [N,24,13], contact_forces [N,24,3],
    obs [N,934], reset [N] u8, terminate [N] u8, and for the Default / Hybrid state init init_root [N,13]
    (with rest_pos [24,3], rest_positions(model)). `phases` are the resets' uniform draws, resolved by
    params.state_init as in the engine."""
    ids = np.ascontiguousarray(env_ids, np.int32)
    names = ("start_times", "start_offsets", "global_offset", "progress", "root_states", "dof_state", "dof_targets",
             "rb_state", "contact_forces", "obs", "reset", "terminate")
    for n in names:
        assert state[n].flags.c_contiguous
    init_root = state.get("init_root")
    if params.state_init in (0, 3) and (init_root is None or rest_pos is None):
        raise ValueError("the Default / Hybrid state init needs state['init_root'] and rest_pos")
    ir = None if init_root is None else f32(init_root)
    rp = None if rest_pos is None else f32(rest_pos)
    lib().ho_reset_envs(C.byref(params), C.byref(mt.struct), C.c_int(len(ids)), _p(ids), _p(f32(phases)),
                        _p(np.ascontiguousarray(motion_ids, np.int64)), *[_p(state[n]) for n in names], _p(ir), _p(rp))
    return state


def new_cache(n):
    """Empty warm-start cache [N, HE_CACHE_WORDS] (float32 words, include/humanoid_engine.h)."""
    return np.zeros((n, _abi.CACHE_WORDS), np.float32)


def set_probe_noise(seed=0, rel=0.0):
    """Sensitivity probes only: rounding-level noise rel on the Delassus operator and the contact
    right-hand side of the following physics_step calls (he_oracle_physics.c); rel 0 turns it off."""
    lib().ho_set_probe_noise(C.c_uint64(int(seed)), C.c_double(float(rel)))


def set_drop_gap_out(arr=None):
    """Diagnostics only: float32 [N] that the following physics_step calls fill with the smallest gap
    among each env's dropped contacts of the last substep (inf: none dropped); None turns it off."""
    lib().ho_set_drop_gap_out(None if arr is None else arr.ctypes.data_as(C.POINTER(C.c_float)))


def set_row_weight_out(arr=None):
    """Diagnostics only: float32 [N, HE_MAX_ROWS] that the following physics_step calls fill with the
    friction bound weight of every solver row of each env's last substep (mu tangential, mu r_patch
    torsional, 0 normal / limit), in the warm-start cache's row order; None turns it off."""
    lib().ho_set_row_weight_out(None if arr is None else arr.ctypes.data_as(C.POINTER(C.c_float)))


def set_two_anchor(on):
    """Diagnostics only (tests/diag/anchor_study.py): PhysX-style two-anchor patch friction in the
    oracle's solver rows instead of the engine's centroid pair + torsional row."""
    lib().ho_set_two_anchor(int(bool(on)))


def set_tgs_sequential(on):
    """Diagnostic: TGS positions integrated once per position iteration (each with that iteration's
    velocity) instead of once with the iterations' mean velocity (the engine's form)."""
    lib().ho_set_tgs_sequential(int(bool(on)))


def set_row_gap_out(arr=None):
    """Diagnostics only: float32 [N, HE_MAX_ROWS] filled with the gap of every solver row's contact of
    each env's last substep (m; a joint-limit row: its angle gap), in the cache's row order."""
    lib().ho_set_row_gap_out(None if arr is None else arr.ctypes.data_as(C.POINTER(C.c_float)))


def physics_step(model: "_abi.HeModel", sim: "_abi.HeSimParams", root_states, dof_state, targets, substeps=2,
                 mass_scale=None, friction=None, terrain_kind=None, cache=None):
    """In-place on root_states [N,13] / dof_state [N,69,2] (float32 arrays) and on the warm-start
    `cache` [N, HE_CACHE_WORDS] (None = cold solves). Returns outputs, including the contacts
    dropped past the capacity and the solve's residual (last substep)."""
    n = root_states.shape[0]
    assert root_states.dtype == np.float32 and root_states.flags.c_contiguous
    assert dof_state.dtype == np.float32 and dof_state.flags.c_contiguous
    if cache is not None:
        assert cache.dtype == np.float32 and cache.flags.c_contiguous and cache.shape == (n, _abi.CACHE_WORDS)
    out = dict(rb_state=np.zeros((n, 24, 13), np.float32), contact_forces=np.zeros((n, 24, 3), np.float32),
               dof_force=np.zeros((n, 69), np.float32), num_contacts=np.zeros(n, np.int32),
               dropped=np.zeros(n, np.int32), residual=np.zeros(n, np.float32), sweeps=np.zeros(n, np.int32))
    ms = None if mass_scale is None else f32(mass_scale)
    fr = None if friction is None else f32(friction)
    tk = None if terrain_kind is None else np.ascontiguousarray(terrain_kind, np.int32)
    lib().ho_physics_step(C.byref(model), C.byref(sim), C.c_int(n), _p(root_states), _p(dof_state), _p(f32(targets)),
                          C.c_int(substeps), _p(out["rb_state"]), _p(out["contact_forces"]), _p(out["dof_force"]),
                          _p(out["num_contacts"]), _p(ms), _p(fr), _p(tk), _p(cache), _p(out["dropped"]),
                          _p(out["residual"]), _p(out["sweeps"]))
    return out


def forward_kinematics(model, root_states, dof_state):
    n = root_states.shape[0]
    rb = np.zeros((n, 24, 13), np.float32)
    lib().ho_forward_kinematics(C.byref(model), C.c_int(n), _p(f32(root_states)), _p(f32(dof_state)), _p(rb))
    return rb


def momentum_energy(model, sim, root_states, dof_state):
    n = root_states.shape[0]
    out = np.zeros((n, 8), np.float64)
    lib().ho_momentum_energy(C.byref(model), C.byref(sim), C.c_int(n), _p(f32(root_states)), _p(f32(dof_state)), _p(out))
    return out


def dynamics_terms(model, sim, root_states, dof_state):
    """The oracle's joint-space inertia H [N,75,75] (CRBA, no armature) and bias [N,75] (RNEA: gravity,
    Coriolis / gyroscopic) at the given states, as its physics step forms them."""
    n = root_states.shape[0]
    H = np.zeros((n, 75, 75), np.float64)
    bias = np.zeros((n, 75), np.float64)
    lib().ho_dynamics_terms(C.byref(model), C.byref(sim), C.c_int(n), _p(f32(root_states)), _p(f32(dof_state)),
                            _p(H), _p(bias))
    return H, bias


def point_jacobian(model, root_states, dof_state, body, x, d):
    """J^T [N,75] of a terrain contact row on body[e] at world point x[e] along d[e] (row_jacobian)."""
    n = root_states.shape[0]
    z = np.zeros((n, 75), np.float64)
    lib().ho_point_jacobian(C.byref(model), C.c_int(n), _p(f32(root_states)), _p(f32(dof_state)),
                            _p(np.ascontiguousarray(body, np.int32)), _p(np.ascontiguousarray(x, np.float64)),
                            _p(np.ascontiguousarray(d, np.float64)), _p(z))
    return z


def jr_inv(th):
    """The inverse right Jacobian of SO(3) at rotation vector th [3] (the joint-limit rows' map from a
    ball joint's child-frame rate to its exp-map coordinate rates)."""
    out = np.zeros((3, 3), np.float64)
    lib().ho_jr_inv(_p(np.ascontiguousarray(th, np.float64)), _p(out))
    return out


def imitation_from_ref(params, pos, rot, vel, ang, rpos, rrot, rvel, rang, progress, pass_time):
    n = pos.shape[0]
    out = dict(rew=np.zeros(n, np.float32), reward_raw=np.zeros((n, 4), np.float32), reset=np.zeros(n, np.uint8),
               terminate=np.zeros(n, np.uint8), self_obs=np.zeros((n, 358), np.float32),
               task_obs=np.zeros((n, 576), np.float32))
    ins = [f32(a) for a in (pos, rot, vel, ang, rpos, rrot, rvel, rang)]
    lib().ho_imitation_from_ref(C.byref(params), C.c_int(n), *[_p(a) for a in ins],
                                _p(np.ascontiguousarray(progress, np.int16)), _p(np.ascontiguousarray(pass_time, np.uint8)),
                                *[_p(out[k]) for k in ("rew", "reward_raw", "reset", "terminate", "self_obs", "task_obs")])
    return out


# ---------------------------------------------------------------- rollout handoff (he_oracle_rollout.c)
def gae(dones, values, rewards, gamma, gae_lambda):
    """c_gae.pyx:11-32 compute_gae restated in C (float32, the Cython operation order)."""
    d, v, r = f32(dones).ravel(), f32(values).ravel(), f32(rewards).ravel()
    n = r.size
    out = np.zeros(n, np.float32)
    lib().ho_gae(C.c_int64(n), _p(d), _p(v), _p(r), C.c_float(gamma), C.c_float(gae_lambda), _p(out))
    return out


def sort_keys(env_id, step):
    """structs.py:128-129: sorted(range(n), key=(env_id, step)) (stable)."""
    e = np.ascontiguousarray(env_id, np.int64)
    s = np.ascontiguousarray(step, np.int64)
    out = np.zeros(e.size, np.int64)
    lib().ho_sort_keys(C.c_int64(e.size), _p(e), _p(s), _p(out))
    return out


class HostExperience:
    """structs.py:22-179 Experience restated over NumPy (store / sort_training_data / flatten_batch) plus
    the core.py:213-258 GAE block: the host checker for humanoid_amd.experience.Experience."""

    def __init__(self, batch_size, bptt_horizon, num_minibatches, minibatch_rows, obs_dim, atn_dim):
        self.batch_size, self.bptt, self.num_mb, self.rows = batch_size, bptt_horizon, num_minibatches, minibatch_rows
        self.obs = np.zeros((batch_size, obs_dim), np.float32)
        self.actions = np.zeros((batch_size, atn_dim), np.float32)
        self.values, self.logprobs, self.rewards, self.dones, self.truncateds = (
            np.zeros(batch_size, np.float32) for _ in range(5))
        self.sort_keys = []
        self.ptr = 0
        self.step = 0

    @property
    def full(self):
        return self.ptr >= self.batch_size

    def store(self, obs, value, action, logprob, reward, done, trunc, env_id, mask):  # structs.py:108-126
        ptr = self.ptr
        indices = np.where(mask)[0][: self.batch_size - ptr]
        end = ptr + len(indices)
        self.obs[ptr:end] = obs[indices]
        self.values[ptr:end] = value[indices]
        self.actions[ptr:end] = action[indices]
        self.logprobs[ptr:end] = logprob[indices]
        self.rewards[ptr:end] = reward[indices]
        self.dones[ptr:end] = done[indices]
        self.truncateds[ptr:end] = trunc[indices]
        self.sort_keys.extend([(env_id[i], self.step) for i in indices])
        self.ptr = end
        self.step += 1

    def sort_training_data(self):  # structs.py:128-142
        keys = np.array(self.sort_keys, np.int64).reshape(-1, 2)
        idxs = sort_keys(keys[:, 0], keys[:, 1])
        self.b_idxs = idxs.reshape(self.rows, self.num_mb, self.bptt).transpose(1, 0, 2)
        self.b_flat = self.b_idxs.reshape(self.num_mb, -1)
        self.sort_keys = []
        return idxs

    def flatten_batch(self):  # structs.py:144-160
        b = self.b_idxs
        self.b_obs, self.b_actions = self.obs[b], self.actions[b]
        self.b_logprobs, self.b_dones, self.b_truncated = self.logprobs[b], self.dones[b], self.truncateds[b]
        self.b_values = self.values[self.b_flat]

    def compute_advantages(self, idxs, gamma, gae_lambda, extra=None):  # core.py:213-258
        r = self.rewards[idxs] if extra is None else self.rewards[idxs] + f32(extra)
        adv = gae(self.dones[idxs], self.values[idxs], r, gamma, gae_lambda)
        self.b_advantages = adv.reshape(self.rows, self.num_mb, self.bptt).transpose(1, 0, 2).reshape(self.num_mb, -1)
        self.b_returns = self.b_advantages + self.b_values
        self.returns = adv + self.values
        return adv


# ------------------------------------------------------------------------- AMP obs (§8f-4)
def amp_joints():
    """Joint indices of the AMP dof subset (humanoid_phc.py:186-194) and key bodies (body_sets.py:45)."""
    from humanoid_amd import body_sets as BS
    joints = [i for i, n in enumerate(BS.DOF_NAMES) if n not in BS.REMOVE_NAMES]
    return np.array(joints, np.int32), BS.body_ids(BS.KEY_BODIES)


def amp_obs(root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_pos):
    """build_amp_observations_smpl (common.py:191-267) with the reference's constant flags."""
    joints, keys = amp_joints()
    n = root_pos.shape[0]
    out = np.zeros((n, 13 + 9 * len(joints) + 3 * len(keys)), np.float32)
    lib().ho_amp_obs(C.c_int(n), C.c_int(len(joints)), _p(joints), C.c_int(len(keys)),
                     *[_p(f32(a)) for a in (root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_pos)],
                     _p(out))
    return out


def amp_obs_from_sim(rb_state, dof_state):
    """_compute_amp_observations (humanoid_phc.py:1125-1176) on rb rows [N,24,13] / dof [N,69,2]."""
    _, keys = amp_joints()
    rb = np.asarray(rb_state, np.float32)
    return amp_obs(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof_state[..., 0],
                   dof_state[..., 1], rb[:, keys, 0:3])


def amp_obs_from_motion(mt: MotionTables, ids, times):
    """_get_amp_obs (humanoid_phc.py:821-838): motion state without offset -> AMP row."""
    _, keys = amp_joints()
    ms = motion_state(mt, ids, times, None)
    return amp_obs(ms["rg_pos"][:, 0], ms["rb_rot"][:, 0], ms["body_vel"][:, 0], ms["body_ang_vel"][:, 0],
                   ms["dof_pos"], ms["dof_vel"], ms["rg_pos"][:, keys])


def amp_step(buf, rb_state, dof_state):
    """_update_hist_amp_obs + _compute_amp_observations (humanoid_phc.py:154-157): history shift,
    then the current row from the simulated state. buf [N,S,W] is returned updated (a copy)."""
    out = np.array(buf, np.float32, copy=True)
    out[:, 1:] = buf[:, :-1]
    out[:, 0] = amp_obs_from_sim(rb_state, dof_state)
    return out


def amp_init(buf, demo, env_ids, rb_state, dof_state, mt: MotionTables, motion_ids, times, control_dt):
    """_init_amp_obs for reference-state resets (humanoid_phc.py:791-819): row 0 from the reset
    state, rows k >= 1 from the motion at t - k*dt (float32 ops as torch does them), then
    demo[env] = buf[env]. Returns updated copies."""
    buf = np.array(buf, np.float32, copy=True)
    demo = np.array(demo, np.float32, copy=True)
    ids = np.asarray(env_ids, np.int64)
    S = buf.shape[1]
    buf[ids, 0] = amp_obs_from_sim(np.asarray(rb_state)[ids], np.asarray(dof_state)[ids])
    if S > 1:
        steps = np.float32(-control_dt) * (np.arange(S - 1, dtype=np.float32) + np.float32(1))
        t = (np.asarray(times, np.float32)[ids][:, None] + steps[None, :]).astype(np.float32)
        mids = np.repeat(np.asarray(motion_ids, np.int64)[ids], S - 1)
        buf[ids, 1:] = amp_obs_from_motion(mt, mids, t.reshape(-1)).reshape(len(ids), S - 1, -1)
    demo[ids] = buf[ids]
    return buf, demo
