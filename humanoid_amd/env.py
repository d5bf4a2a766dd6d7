"""Host-side mirror of the reference's environment classes on the HIP engine.

``HumanoidPHC`` follows ``puffer_phc/envs/humanoid_phc.py`` (reset / step / motion resampling /
eval toggles, same buffers and ``extras`` keys). ``PHCPufferEnv`` follows
``puffer_phc/clean_pufferl/env.py:40-210`` (terminals / truncations / masks, episode statistics,
info every ``log_interval`` ticks).

Differences, all on the performance side:
* ``HumanoidPHC.step`` is two launches (physics with the action->PD-target map fused in, then the
  fused reward/reset/observation kernel) instead of ~200 eager torch ops;
* ``PHCPufferEnv.step`` resets the flagged envs on the device inside the same launch
  (``he_imitation_reset_step``) and keeps episode statistics on the device, so a step performs no
  host synchronisation except the one-off ``info`` read every ``log_interval`` ticks. Reset
  phases come from a counter-based hash of (seed, tick, env) rather than ``torch.rand``.
There is no CPU path: constructing either class without the engine library or a GPU raises.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _abi
from .body_sets import BODY_NAMES, DOF_NAMES, EVAL_BODIES, body_ids, frozen_dof_mask
from .model import load_default_model, pd_action_offset_scale

NUM_OBS = 934
NUM_ACTIONS = 69


# ------------------------------------------------------------------------------ config (config.py)
@dataclass
class RewardConfig:  # config.py:37-50
    k_pos: float = 100.0
    k_rot: float = 10.0
    k_vel: float = 0.1
    k_ang_vel: float = 0.1
    w_pos: float = 0.5
    w_rot: float = 0.3
    w_vel: float = 0.1
    w_ang_vel: float = 0.1
    imitation_reward_dim: int = 4
    full_body_reward: bool = True
    use_power_reward: bool = True


@dataclass
class RobotConfig:  # config.py:53-86 (the fields the hot path reads)
    humanoid_type: str = "smpl"
    has_self_collision: bool = True
    has_smpl_pd_offset: bool = False  # PD offsets from the SMPL rest pose (humanoid_phc.py:411-440)
    has_upright_start: bool = True    # the clips' upright start (obs heading frame, common.py:106-176)
    has_dof_subset: bool = True       # AMP's 19-joint dof subset (humanoid_phc.py:186-194)
    has_mesh: bool = False
    has_shape_obs: bool = False
    has_shape_obs_disc: bool = False
    has_limb_weight_obs: bool = False
    has_limb_weight_obs_disc: bool = False
    reduce_action: bool = False
    freeze_hand: bool = True
    freeze_toe: bool = True
    bias_offset: bool = False

    def check(self):
        """Raise for the reference options the engine's fused kernels do not implement (their
        defaults are what the engine bakes in); never silently ignore one."""
        unsupported = {"has_upright_start": (self.has_upright_start, True), "has_dof_subset": (self.has_dof_subset, True),
                       "has_mesh": (self.has_mesh, False), "has_shape_obs": (self.has_shape_obs, False),
                       "has_shape_obs_disc": (self.has_shape_obs_disc, False),
                       "has_limb_weight_obs": (self.has_limb_weight_obs, False),
                       "has_limb_weight_obs_disc": (self.has_limb_weight_obs_disc, False),
                       "reduce_action": (self.reduce_action, False)}
        for name, (value, supported) in unsupported.items():
            if bool(value) != supported:
                raise NotImplementedError(f"RobotConfig.{name}={value} is not supported by the engine "
                                          f"(the reference default {supported} is)")
        if self.humanoid_type != "smpl":
            raise ValueError(f"humanoid_type {self.humanoid_type!r}: only 'smpl' (config.py:56)")


@dataclass
class EnvConfig:  # config.py:89-157
    device_type: str = "cuda"
    device_id: int = 0
    motion_file: object = "data/motion/amass_train_take6_upright.pkl"  # path, directory or clip dict
    num_envs: int = 4096
    headless: bool = True
    clip_actions: bool = True
    use_amp_obs: bool = False
    num_amp_obs_steps: int = 10
    enable_early_termination: bool = True
    termination_distance: float = 0.25
    max_episode_length: int = 300
    auto_pmcp: bool = False
    auto_pmcp_soft: bool = True
    kp_scale: float = 1.0
    kd_scale: float = 1.0
    log_interval: int = 32
    rew_power_coef: float = 0.0005
    state_init: str = "Random"   # StateInit (config.py:114): Default, Start, Random, Hybrid
    hybrid_init_prob: float = 0.5  # config.py:139 (Hybrid only)
    add_obs_noise: bool = False    # config.py:120-121, humanoid_phc.py:956
    obs_noise_std: float = 0.1
    min_motion_len: int = 5
    max_motion_len: int = 600
    robot: RobotConfig = field(default_factory=RobotConfig)
    reward: RewardConfig = field(default_factory=RewardConfig)
    # engine extensions (not in the reference config)
    seed: int = 0
    max_contacts: int = 40
    # the physics solver (isaacgym_env.py:16-18 sets PhysX TGS, 4 position iterations): solver_type 1
    # TGS with solver_iterations position iterations per physics step; 0 the engine's PGS step
    # (solver_iterations velocity-level sweeps). None: the solver's own default (TGS 4,
    # PGS 8). Until round 4 the count meant PGS sweeps (default 8); a TGS iteration costs about two
    # sweeps, so an explicit count other than 4 under TGS warns (resolved_solver_iterations).
    solver_type: int = 1
    solver_iterations: Optional[int] = None

    def resolved_solver_iterations(self) -> int:
        if self.solver_iterations is None:
            return 4 if self.solver_type == 1 else 8
        if self.solver_type == 1 and self.solver_iterations != 4:
            import warnings
            warnings.warn(f"solver_iterations={self.solver_iterations} counts TGS position iterations "
                          "(solver_type 1, the reference's 4: isaacgym_env.py:17), not PGS sweeps; set "
                          "solver_type=0 for the PGS step", stacklevel=2)
        return int(self.solver_iterations)

    @property
    def device(self) -> str:
        return "cpu" if self.device_type == "cpu" else f"cuda:{self.device_id}"

    @property
    def num_agents(self) -> int:
        return self.num_envs


class Box:
    """Minimal ``gym.spaces.Box`` stand-in (gym/gymnasium are not dependencies of the engine)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low = np.full(shape, low, dtype)
        self.high = np.full(shape, high, dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def sample(self, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi).astype(self.dtype)


# ------------------------------------------------------------------------------ HumanoidPHC
class HumanoidPHC:
    """``humanoid_phc.py:HumanoidPHC`` on the engine. Buffers have the reference's names, shapes
    and dtypes: obs_buf [N,934] f32, rew_buf [N] f32, reset_buf [N] bool, progress_buf [N] i16,
    reward_raw [N,5] f32, extras {"terminate", "reward_raw"}."""

    def __init__(self, cfg: EnvConfig, motion_data=None):
        import torch
        from .engine import Engine
        from .motion_lib import MotionLibSMPL
        if cfg.device_type != "cuda":
            raise ValueError("the engine runs on the GPU only (device_type='cuda')")
        cfg.robot.check()
        # _reset_actors (humanoid_phc.py:679-686): Random and Start sample the reference motion
        # (_reset_ref_state_init), Default resets to the initial pose (_reset_default), Hybrid mixes
        # them by a Bernoulli(hybrid_init_prob) draw (_reset_hybrid_state_init); all four run in the
        # engine's reset (he_reset_envs, and the device reset of he_env_step)
        if cfg.state_init not in _abi.STATE_INIT:
            raise ValueError(f"Unsupported state initialization strategy: {cfg.state_init}")
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        n = cfg.num_envs
        self.model = load_default_model()
        self.num_bodies, self.num_dof = len(BODY_NAMES), 3 * len(DOF_NAMES)
        self.num_obs, self.num_actions = NUM_OBS, NUM_ACTIONS
        sim = _abi.default_sim_params(self_collision=int(cfg.robot.has_self_collision), kp_scale=cfg.kp_scale,
                                      kd_scale=cfg.kd_scale, max_contacts=cfg.max_contacts,
                                      solver_type=cfg.solver_type,
                                      solver_iterations=cfg.resolved_solver_iterations())
        # start pose z=0.89 + U(-1,1) xy jitter (humanoid_phc.py:340-347)
        rng = np.random.default_rng(cfg.seed)
        self.engine = Engine(self.model, n, device=self.device.index or 0, sim_params=sim,
                             start_xy=rng.uniform(-1.0, 1.0, (n, 2)).astype(np.float32))
        off, sc = pd_action_offset_scale(self.model, bias_offset=cfg.robot.bias_offset,
                                         has_smpl_pd_offset=cfg.robot.has_smpl_pd_offset)
        frozen = np.zeros(self.num_dof, np.int32)
        if cfg.robot.freeze_hand or cfg.robot.freeze_toe:
            frozen = np.array(frozen_dof_mask(freeze_hand=cfg.robot.freeze_hand, freeze_toe=cfg.robot.freeze_toe),
                              np.int32)
        self.engine.set_pd_params(off, sc, frozen, clip_actions=False)  # clipping is the caller's (env.py:110)
        self.single_observation_space = Box(-np.inf, np.inf, (NUM_OBS,))
        self.single_action_space = Box(-1.0, 1.0, (NUM_ACTIONS,))
        self.amp_observation_space = None
        dev = self.device
        if cfg.use_amp_obs:  # AMP buffers (humanoid_phc.py:469-491, 600-611), updated by the engine
            self._num_amp_obs_per_step = _abi.AMP_OBS_STEP
            self.num_amp_obs = cfg.num_amp_obs_steps * self._num_amp_obs_per_step
            self.amp_observation_space = Box(-np.inf, np.inf, (self.num_amp_obs,))
            self._amp_obs_buf = torch.zeros(n, cfg.num_amp_obs_steps, self._num_amp_obs_per_step, device=dev)
            self._curr_amp_obs_buf = self._amp_obs_buf[:, 0]
            self._hist_amp_obs_buf = self._amp_obs_buf[:, 1:]
            self._amp_obs_demo_buf = torch.zeros_like(self._amp_obs_buf)
            self.engine.set_amp(self._amp_obs_buf, self._amp_obs_demo_buf)
        self.obs_buf = torch.zeros(n, NUM_OBS, device=dev)
        self.rew_buf = torch.zeros(n, device=dev)
        self.reward_raw = torch.zeros(n, 5, device=dev)
        self.progress_buf = torch.zeros(n, dtype=torch.int16, device=dev)
        self._reset_u8 = torch.ones(n, dtype=torch.uint8, device=dev)
        self._term_u8 = torch.ones(n, dtype=torch.uint8, device=dev)
        self.reset_buf = self._reset_u8.view(torch.bool)
        self._terminate_buf = self._term_u8.view(torch.bool)
        self.extras = {}
        self._global_offset = torch.zeros(n, 3, device=dev)
        self._motion_start_times = torch.zeros(n, device=dev)
        self._motion_start_times_offset = torch.zeros(n, device=dev)
        self._sampled_motion_ids = torch.arange(n, device=dev)
        self._motion_sample_start_idx = 0
        self.all_env_ids = torch.arange(n, device=dev)
        self.flag_test = False
        self.flag_im_eval = False
        self._eval_recorder = None
        self._gen = torch.Generator(device=dev).manual_seed(cfg.seed)
        self._term_dist = float(cfg.termination_distance)
        self._reset_bodies = list(range(self.num_bodies))
        self._reset_bodies_backup = list(self._reset_bodies)
        self._update_params()
        self._em = self.engine.env_motion(self._sampled_motion_ids, self._motion_start_times,
                                          self._motion_start_times_offset, self._global_offset, self.progress_buf)
        # motion libraries (humanoid_phc.py:620-663)
        data = cfg.motion_file if motion_data is None else motion_data
        self._motion_train_lib = MotionLibSMPL(data, self.model, device=dev, min_length=cfg.min_motion_len,
                                               seed=cfg.seed)
        self._motion_eval_lib = MotionLibSMPL(data, self.model, device=dev, min_length=cfg.min_motion_len,
                                              im_eval=True, seed=cfg.seed)
        self._motion_lib = self._motion_train_lib
        interval = self.num_unique_motions / (n + 50)  # even sampling on the first load (:645-648)
        idx = np.floor(np.arange(0, self.num_unique_motions, interval)).astype(int)[:n]
        self._load(sample_idxes=torch.from_numpy(idx))

    # -- parameters ----------------------------------------------------------------------

    def _obs_noise(self, env_ids=None):
        """humanoid_phc.py:956-959: obs + N(0, obs_noise_std) while training (not in test mode), on the
        rows just computed: every row after a step, only the reset rows after a partial reset
        (obs_buf[env_ids] = obs)."""
        import torch
        if self.cfg.add_obs_noise and not self.flag_test:
            if not hasattr(self, "_noise_gen"):  # its own stream: the reset phases stay the same
                self._noise_gen = torch.Generator(device=self.device).manual_seed(self.cfg.seed + 7919)
            if env_ids is None:
                self.obs_buf.add_(torch.randn(self.obs_buf.shape, device=self.device, generator=self._noise_gen)
                                  * self.cfg.obs_noise_std)
            else:
                ids = env_ids.to(device=self.device, dtype=torch.long)
                self.obs_buf[ids] += torch.randn((len(ids), self.obs_buf.shape[1]), device=self.device,
                                                 generator=self._noise_gen) * self.cfg.obs_noise_std

    def _update_params(self):
        r = dataclasses.asdict(self.cfg.reward)
        self._params = _abi.imitation_params(reward=r, use_power_reward=self.cfg.reward.use_power_reward,
                                             power_coef=self.cfg.rew_power_coef,
                                             enable_early_termination=self.cfg.enable_early_termination,
                                             eval_mode=self.flag_im_eval, termination_distance=self._term_dist,
                                             reset_body_ids=self._reset_bodies,
                                             state_init=self.cfg.state_init,
                                             hybrid_init_prob=self.cfg.hybrid_init_prob, test_mode=self.flag_test)

    def set_termination_distances(self, termination_distances):  # :1338-1339
        self._term_dist = termination_distances
        self._update_params()

    def _load(self, **kw):
        # sampling on the host (motion_lib.py:305-345), ingestion on the device (he_ingest_clips)
        clips, motion_clip = self._motion_lib.select_motions(self.cfg.num_envs, **kw)
        self.engine.ingest_clips(clips, motion_clip)
        if self._eval_recorder is not None:
            self._eval_recorder.set_num_steps(self.get_motion_steps())

    def _attach_eval(self):
        """Eval mode: the next stepping launch also records the frame's metrics (he_set_eval) and the
        reference's eval extras (humanoid_phc.py:158-169; device tensors instead of host copies)."""
        if self.flag_im_eval and self._eval_recorder is not None:
            rec = self._eval_recorder
            rec.attach()
            self.extras["mpjpe"] = rec.mpjpe
            self.extras["body_pos"] = rec.body_pos
            self.extras["body_pos_gt"] = rec.body_pos_gt

    # -- reset / step (:90-172) ----------------------------------------------------------
    def _reset_envs(self, env_ids):
        import torch
        if len(env_ids) == 0:
            return
        # one uniform draw per env; the engine resolves it by the state init (Start / test mode: t = 0,
        # Hybrid: the Bernoulli and the phase, include/humanoid_engine.h)
        phases = torch.rand(len(env_ids), device=self.device, generator=self._gen)
        self.engine.reset_envs(self._params, self._em, env_ids.to(torch.int32), phases, self.obs_buf,
                               self._reset_u8, self._term_u8)
        self._obs_noise(env_ids)

    def reset(self, env_ids=None):
        safe_reset = env_ids is None or len(env_ids) == self.cfg.num_envs
        if env_ids is None:
            env_ids = self.all_env_ids
        self._reset_envs(env_ids)
        if safe_reset:  # one substep, then reset again (:97-101)
            self.engine.simulate(1)
            self._reset_envs(env_ids)
        return self.obs_buf

    def step(self, actions):
        self.engine.step_actions(actions, 2)
        self._attach_eval()
        self.engine.imitation_step(self._params, self._em, self.obs_buf, self.rew_buf, self.reward_raw,
                                   self._reset_u8, self._term_u8)
        self._obs_noise()
        self.extras["terminate"] = self._terminate_buf.clone()
        self.extras["reward_raw"] = self.reward_raw.detach()
        if self.cfg.use_amp_obs:  # the launch above also shifted the history and wrote row 0 (:154-157)
            self.extras["amp_obs"] = self.amp_obs
        return self.obs_buf, self.rew_buf, self.reset_buf, self.extras

    # -- AMP (:1352-1357) --------------------------------------------------------------------
    @property
    def amp_obs(self):
        return self._amp_obs_buf.view(-1, self.num_amp_obs) if self.cfg.use_amp_obs else None

    def fetch_amp_obs_demo(self):
        return self._amp_obs_demo_buf.view(-1, self.num_amp_obs) if self.cfg.use_amp_obs else None

    # -- motion sampling (:1363-1455) ------------------------------------------------------
    def resample_motions(self):
        if self.flag_test:
            self.forward_motion_samples()
            return
        t = self.progress_buf.float() * (1.0 / 30.0) + self._motion_start_times + self._motion_start_times_offset
        self._load(random_sample=True)
        ms = self.engine.motion_state(self._sampled_motion_ids, t, want_dof=False)
        self._global_offset[:, :2] = self.engine.root_states[:, :2] - ms["rg_pos"][:, 0, :2]
        self.reset()

    def begin_seq_motion_samples(self):
        self._motion_sample_start_idx = 0
        self._load(random_sample=False, start_idx=0)
        self.reset()

    def forward_motion_samples(self):
        self._motion_sample_start_idx += self.cfg.num_envs
        self._load(random_sample=False, start_idx=self._motion_sample_start_idx)
        self.reset()

    def toggle_eval_mode(self):
        self.flag_test = True
        self.flag_im_eval = True
        self._term_dist = 0.5
        self._motion_lib = self._motion_eval_lib
        if len(self._reset_bodies) > 15:
            self._reset_bodies = list(body_ids(EVAL_BODIES))
        self._update_params()
        from .eval import EvalRecorder
        self._eval_recorder = EvalRecorder(self.engine, self.cfg.num_envs, self.device)
        self.begin_seq_motion_samples()
        return self._motion_lib._num_unique_motions

    def untoggle_eval_mode(self, failed_keys):
        self.flag_test = False
        self.flag_im_eval = False
        if self._eval_recorder is not None:
            self._eval_recorder.detach()
            self._eval_recorder = None
        for k in ("mpjpe", "body_pos", "body_pos_gt"):
            self.extras.pop(k, None)
        self._term_dist = float(self.cfg.termination_distance)
        self._motion_lib = self._motion_train_lib
        self._reset_bodies = list(self._reset_bodies_backup)
        self._update_params()
        if self.cfg.auto_pmcp:
            self._motion_lib.update_hard_sampling_weight(failed_keys)
        elif self.cfg.auto_pmcp_soft:
            self._motion_lib.update_soft_sampling_weight(failed_keys)
        return self._motion_lib._termination_history.clone()

    @property
    def num_unique_motions(self):
        return self._motion_lib._num_unique_motions

    @property
    def current_motion_ids(self):
        return self._motion_lib._curr_motion_ids

    @property
    def motion_sample_start_idx(self):
        return self._motion_sample_start_idx

    @property
    def motion_data_keys(self):
        return self._motion_lib._motion_data_keys

    def get_motion_steps(self):
        return self._motion_lib.get_motion_num_steps()

    # -- state views (humanoid_phc.py:497-554) ----------------------------------------------
    @property
    def _humanoid_root_states(self):
        return self.engine.root_states

    @property
    def _dof_pos(self):
        return self.engine.dof_state.view(self.cfg.num_envs, self.num_dof, 2)[..., 0]

    @property
    def _dof_vel(self):
        return self.engine.dof_state.view(self.cfg.num_envs, self.num_dof, 2)[..., 1]

    @property
    def _rigid_body_pos(self):
        return self.engine.rb_state.view(self.cfg.num_envs, self.num_bodies, 13)[..., :3]

    @property
    def _contact_forces(self):
        return self.engine.contact_forces.view(self.cfg.num_envs, self.num_bodies, 3)

    def render(self):
        return None

    def close(self):
        self.engine = None


# ------------------------------------------------------------------------------ PHCPufferEnv
class PHCPufferEnv:
    """``clean_pufferl/env.py:PHCPufferEnv`` over :class:`HumanoidPHC`, host-sync-free per step."""

    def __init__(self, cfg: EnvConfig, motion_data=None):
        import torch
        self.render_mode = "native"
        self.cfg = cfg
        self.env = HumanoidPHC(cfg, motion_data=motion_data)
        self.single_observation_space = self.env.single_observation_space
        self.single_action_space = self.env.single_action_space
        self.amp_observation_space = self.env.amp_observation_space if cfg.use_amp_obs else None  # env.py:59
        self.amp_obs = self.env.amp_obs if cfg.use_amp_obs else None  # env.py:94 (a live view)
        dev = self.env.device
        n = cfg.num_envs
        self.observations = self.env.obs_buf
        self.rewards = self.env.rew_buf
        self.terminals = torch.zeros(n, dtype=torch.bool, device=dev)
        self.truncations = torch.zeros(n, dtype=torch.bool, device=dev)
        self.masks = torch.ones(n, dtype=torch.bool, device=dev)
        self.actions = torch.zeros(n, NUM_ACTIONS, dtype=torch.float, device=dev)
        self.episode_returns = torch.zeros(n, dtype=torch.float32, device=dev)
        self.episode_lengths = torch.zeros(n, dtype=torch.int32, device=dev)
        self.episode_count = 0
        self.raw_rewards = torch.zeros(5, dtype=torch.float32, device=dev)
        # device-side accumulators of the reference's per-episode info lists (env.py:80-84)
        self._acc = torch.zeros(5, dtype=torch.float64, device=dev)  # sum_ret, sum_len, n_ep, n_trunc, n_term
        self.tick = 0
        # numpy actions go through two pinned host buffers (alternating, each reused only after its
        # previous host-to-device copy has completed), so the copy is asynchronous and the host runs
        # ahead of the device instead of blocking on a pageable transfer every step
        self._pinned = [torch.empty(n, NUM_ACTIONS, dtype=torch.float32).pin_memory() for _ in range(2)]
        self._pinned_done = [None, None]

    @property
    def num_agents(self):
        return self.cfg.num_envs

    def reset(self, seed=None):
        self.tick = 0
        self.env.reset()
        self.rewards[:] = 0
        self.terminals[:] = False
        self.truncations[:] = False
        self.masks[:] = True
        self.actions[:] = 0
        self.raw_rewards[:] = 0
        self._acc[:] = 0
        return self.observations, []

    def step(self, actions):
        """``actions``: numpy [N,69] (copied to the device, as env.py:112) or a device tensor."""
        import torch
        if isinstance(actions, np.ndarray):
            k = self.tick & 1
            if self._pinned_done[k] is not None:
                self._pinned_done[k].synchronize()
            buf = self._pinned[k]
            buf.numpy()[...] = actions
            self.actions.copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pinned_done[k] = ev
            if self.cfg.clip_actions:  # env.py:110-111, on the device
                self.actions.clamp_(-1, 1)
        else:
            self.actions[:] = actions.clamp(-1, 1) if self.cfg.clip_actions else actions
        e = self.env
        e._attach_eval()
        # physics + reward / reset / observation: one launch up to 2048 envs (he_set_fused_step auto),
        # two above, or with eval recording attached; bit-identical either way
        e.engine.env_step(e._params, e._em, self.actions, e.obs_buf, e.rew_buf, e.reward_raw, e._reset_u8, e._term_u8,
                          seed=self.cfg.seed, step_index=self.tick)
        e._obs_noise()
        # the step's returned copies and the episode bookkeeping (env.py:120-160) in one launch
        rew = torch.empty_like(self.rewards)
        term_copy = torch.empty_like(e._term_u8)
        stream = torch.cuda.current_stream(self.actions.device).cuda_stream
        rc = e.engine.lib.he_episode_step(
            int(self.cfg.num_envs), self.rewards.data_ptr(), e.reward_raw.data_ptr(), e._reset_u8.data_ptr(),
            e._term_u8.data_ptr(), rew.data_ptr(), term_copy.data_ptr(), self.terminals.data_ptr(),
            self.truncations.data_ptr(), self.masks.data_ptr(), self.episode_returns.data_ptr(),
            self.episode_lengths.data_ptr(), self.raw_rewards.data_ptr(), self._acc.data_ptr(), stream)
        if rc != 0:
            from humanoid_amd.engine import EngineError
            raise EngineError(e.engine.lib.he_last_error().decode())
        e.extras["terminate"] = term_copy.view(torch.bool)
        e.extras["reward_raw"] = e.reward_raw.detach()
        if self.cfg.use_amp_obs:
            e.extras["amp_obs"] = e.amp_obs
        info = []
        self.tick += 1
        if self.tick % self.cfg.log_interval == 0:
            info = self.mean_and_log()
            li = self.cfg.log_interval
            rr = (self.raw_rewards / li).tolist()
            reward_info = {"rew_body_pos": rr[0], "rew_body_rot": rr[1], "rew_lin_vel": rr[2], "rew_ang_vel": rr[3],
                           "rew_power": rr[4]}
            self.raw_rewards[:] = 0
            if len(info) > 0:
                info[0].update(reward_info)
            else:
                info.append(reward_info)
        return self.observations, rew, self.terminals, self.truncations, info

    def fetch_amp_obs_demo(self):  # env.py:206-207
        return self.env.fetch_amp_obs_demo()

    def mean_and_log(self):
        s = self._acc.tolist()
        self._acc[:] = 0
        self.episode_count += int(s[2])
        n_ep = s[2]
        nan = float("nan")
        return [{"episode_return": s[0] / n_ep if n_ep else nan, "episode_length": s[1] / n_ep if n_ep else nan,
                 "truncated_rate": s[3] / (s[3] + s[4]) if (s[3] + s[4]) else nan}]

    def render(self):
        return self.env.render()

    def close(self):
        self.env.close()
