"""Eval path on the device.

The reference's eval loop (scripts/phc_train.py:62-244 ``EvalStats`` + :373-421 ``rollout``) copies
``body_pos`` and ``body_pos_gt`` ([N,24,3] each) to the host every step (humanoid_phc.py:158-169),
stacks them for every motion of a batch, and at the end runs smpl_sim's ``compute_metrics_lite``
(un-vendored; smpl_sim 0.0.1 @ git fe22a5d9) over the stacks: per frame MPJPE (global and
root-relative), Procrustes-aligned MPJPE (a 3x3 SVD per frame), velocity and acceleration errors.

Here the imitation kernel records those per-frame metrics in the same launch that computes the
reward (``he_eval_buffers``, include/humanoid_engine.h) and keeps per-env sums on the device, so
a batch costs no position copies; :class:`EvalStats` mirrors the reference's bookkeeping and
reads back [N,8] sums once per batch plus one small vector per step (the reference's own per-step
``.sum()``/``.max()`` decisions, gathered into one read).
"""
from typing import Optional

import numpy as np

from . import _abi

__all__ = ["EvalRecorder", "EvalStats", "METRICS"]

METRICS = ("mpjpe_g", "mpjpe_l", "mpjpe_pa", "vel_dist", "accel_dist")
_COUNT = {"mpjpe_g": 5, "mpjpe_l": 5, "mpjpe_pa": 5, "vel_dist": 6, "accel_dist": 7}


class EvalRecorder:
    """Device buffers behind he_eval_buffers for one engine of N envs."""

    def __init__(self, engine, num_envs: int, device, with_positions: bool = True):
        import torch
        self.engine = engine
        self.n = num_envs
        dev = torch.device(device)
        self.num_steps = torch.zeros(num_envs, dtype=torch.int32, device=dev)
        self.mpjpe = torch.zeros(num_envs, dtype=torch.float32, device=dev)
        self.body_pos = torch.zeros(num_envs, 24, 3, device=dev) if with_positions else None
        self.body_pos_gt = torch.zeros(num_envs, 24, 3, device=dev) if with_positions else None
        self.history = torch.zeros(num_envs, 2, 2, 24, 3, device=dev)
        self.sums = torch.zeros(num_envs, _abi.EVAL_SUMS, dtype=torch.float64, device=dev)
        self.frame = 0

    def set_num_steps(self, num_steps):
        import torch
        self.num_steps.copy_(num_steps.to(self.num_steps.device, dtype=torch.int32))

    def attach(self):
        """he_set_eval with the current frame (call before every stepping launch)."""
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        b = _abi.HeEvalBuffers(p(self.num_steps), p(self.mpjpe), p(self.body_pos), p(self.body_pos_gt),
                               p(self.history), p(self.sums), int(self.frame), 0)
        self.engine.set_eval(b)

    def detach(self):
        self.engine.set_eval(None)


class EvalStats:
    """phc_train.py:62-244 ``EvalStats`` over the device recorder (same constructor, methods,
    ``results`` / ``results_by_motion`` keys). ``vec_env`` is a :class:`humanoid_amd.env.PHCPufferEnv`."""

    def __init__(self, vec_env, failed_save_path=None, verbose: bool = True):
        import torch
        self.task_env = vec_env.env
        self.num_envs = self.task_env.cfg.num_envs
        device = self.task_env.device
        self.failed_save_path = failed_save_path
        self.verbose = verbose
        self.num_unique_motions = self.task_env.toggle_eval_mode()  # attaches the recorder
        self.recorder: EvalRecorder = self.task_env._eval_recorder
        self.terminate_state = torch.zeros(self.num_envs, dtype=torch.bool, device=device)
        self.played_steps_buf = torch.zeros(self.num_envs, dtype=torch.short, device=device)
        self.terminate_memory = []
        self.motion_length = []
        self.played_steps = []
        self.batch_sums = []   # per batch: [N, 8] float64 (host), the per-motion metric sums
        self.mpjpe_all = []    # per batch: per-env mean extras["mpjpe"] over its counted frames (m)
        self.curr_steps = 0
        self.success_rate = 0
        self.failed_keys = []
        self.results = None
        self.results_by_motion = None
        self._new_batch()

    def _new_batch(self):
        """Per-batch constants of post_step_eval's frame-budget rule (phc_train.py:103-118)."""
        import torch
        self._num_steps = self.task_env.get_motion_steps()
        curr_ids = self.task_env.current_motion_ids
        hit = (curr_ids == self.num_unique_motions - 1).nonzero()
        self._bound = int(hit[0, 0]) + 1 if len(hit) else None
        self._idx = torch.arange(self.num_envs, device=self._num_steps.device)
        self.recorder.frame = 0

    def post_step_eval(self):
        """phc_train.py:88-164, one small device->host read per step."""
        import torch
        motion_num_steps = self._num_steps
        next_batch = False
        info = self.task_env.extras
        cs = self.curr_steps
        termination_state = torch.logical_and(cs < motion_num_steps, info["terminate"])
        torch.logical_or(termination_state, self.terminate_state, out=self.terminate_state)
        current_envs = torch.logical_and(~self.terminate_state, cs < motion_num_steps)
        self.played_steps_buf += current_envs.to(torch.short)
        alive = ~self.terminate_state
        neg = torch.full_like(motion_num_steps, -(1 << 30))
        if self._bound is not None:
            inb = self._idx < self._bound
            stats = torch.stack([alive.sum(), (alive & inb).sum(),
                                 torch.where(alive & inb, motion_num_steps, neg).max(), motion_num_steps.max()])
        else:
            stats = torch.stack([alive.sum(), alive.sum(), torch.where(alive, motion_num_steps, neg).max(),
                                 motion_num_steps.max()])
        n_alive, n_alive_b, max_alive, max_all = (int(v) for v in stats.tolist())
        if n_alive > 0:
            if self._bound is not None:
                if n_alive_b > 0:
                    curr_max = max_alive
                else:
                    curr_max = cs - 1
                    self.terminate_state[self._bound:] = True
            else:
                curr_max = max_alive
            if cs >= curr_max:
                curr_max = cs + 1
        else:
            curr_max = max_all
        self.curr_steps += 1

        if self.curr_steps >= curr_max or int(self.terminate_state.sum()) == self.num_envs:
            self.curr_steps = 0
            self.terminate_memory.append(self.terminate_state.cpu().numpy())
            self.motion_length.append(motion_num_steps.cpu().numpy())
            self.played_steps.append(self.played_steps_buf.cpu().numpy())
            self.success_rate = 1 - np.concatenate(self.terminate_memory)[: self.num_unique_motions].mean()
            sums = self.recorder.sums.cpu().numpy().copy()
            self.batch_sums.append(sums)
            with np.errstate(invalid="ignore", divide="ignore"):
                self.mpjpe_all.append(sums[:, 0] / 1000.0 / sums[:, 5])
            if self.task_env.motion_sample_start_idx + self.num_envs >= self.num_unique_motions:
                self.recorder.frame = 0
                return self.get_final_stats(), next_batch
            next_batch = True
            self.task_env.forward_motion_samples()
            self.terminate_state[:] = False
            self.played_steps_buf[:] = 0
            self._new_batch()
        self.recorder.frame = self.curr_steps
        return False, next_batch

    @staticmethod
    def _metrics(sums: np.ndarray):
        """compute_metrics_lite(...) then {m: np.mean(v)}: the mean over every counted frame."""
        if sums.shape[0] == 0:
            return {}
        out = {}
        for k, m in enumerate(METRICS):
            c = sums[:, _COUNT[m]].sum()
            out[m] = float(sums[:, k].sum() / c) if c > 0 else float("nan")
        return out

    def get_final_stats(self):
        """phc_train.py:166-225."""
        terminate_hist = np.concatenate(self.terminate_memory)
        nu = self.num_unique_motions
        all_sums = np.concatenate(self.batch_sums)[:nu]
        succ = ~terminate_hist[:nu]
        metrics_all_print = self._metrics(all_sums)
        metrics_succ_print = self._metrics(all_sums[succ])
        self.failed_keys = self.task_env.motion_data_keys[terminate_hist[:nu]]
        if len(metrics_succ_print) == 0:
            if self.verbose:
                print("No success!!!")
            metrics_succ_print = metrics_all_print
        if self.verbose:
            print("------------------------------------------")
            print(f"Success Rate: {self.success_rate:.10f}")
            print("All: ", " \t".join([f"{k}: {v:.3f}" for k, v in metrics_all_print.items()]))
            print("Succ: ", " \t".join([f"{k}: {v:.3f}" for k, v in metrics_succ_print.items()]))
            print("Failed keys: ", len(self.failed_keys), ",", self.failed_keys)
        self.metrics_all, self.metrics_succ = metrics_all_print, metrics_succ_print
        self.results = {
            "eval/success_rate": float(self.success_rate),
            "eval/mpjpe_all": metrics_all_print["mpjpe_g"],
            "eval/mpjpe_succ": metrics_succ_print["mpjpe_g"],
            "eval/accel_dist": metrics_succ_print["accel_dist"],
            "eval/vel_dist": metrics_succ_print["vel_dist"],
            "eval/mpjpel_all": metrics_all_print["mpjpe_l"],
            "eval/mpjpel_succ": metrics_succ_print["mpjpe_l"],
            "eval/mpjpe_pa": metrics_succ_print["mpjpe_pa"],
        }
        self.results_by_motion = {
            "motion_keys": self.task_env.motion_data_keys.tolist(),
            "motion_length": np.concatenate(self.motion_length)[:nu],
            "played_steps": np.concatenate(self.played_steps)[:nu],
            "success": ~terminate_hist[:nu],
        }
        return True

    def update_env_and_close(self):
        """phc_train.py:227-244 (detaches the recorder with the eval mode)."""
        termination_history = self.task_env.untoggle_eval_mode(self.failed_keys)
        if self.failed_save_path:
            import joblib
            joblib.dump({"failed_keys": self.failed_keys, "termination_history": termination_history},
                        self.failed_save_path)
        return self.results


def recorder_for(env) -> Optional[EvalRecorder]:
    return getattr(env, "_eval_recorder", None)
