"""TEST INFRASTRUCTURE ONLY: host restatement of the reference's eval metrics and bookkeeping, the
checker for the device eval path (humanoid_amd/eval.py, he_eval_buffers).

- ``compute_metrics_lite`` and its helpers restate smpl_sim's ``smpllib/smpl_eval.py`` (smpl_sim
  0.0.1, git fe22a5d9 per /root/reference/uv.lock; un-vendored and not installed here), called at
  scripts/phc_train.py:188-189: per motion, per frame MPJPE on world positions (mpjpe_g), on
  root-relative positions (mpjpe_l), after a Procrustes similarity alignment (mpjpe_pa, the
  VideoPose3D "protocol #2" 3x3 SVD with reflection fix), and the velocity / acceleration errors of
  the frame sequence, all x1000 (mm). PARITY UNPINNED against smpl_sim itself (absent); the
  restatement is checked with closed-form cases in tests/test_eval.py.
- ``HostEvalStats`` restates ``EvalStats.post_step_eval``'s batch bookkeeping (phc_train.py:88-164)
  over host copies of what the reference copies every step, without touching the env.
"""
from collections import defaultdict

import numpy as np


def p_mpjpe(predicted, target):
    """MPJPE after the similarity transform (scale, rotation, translation) mapping predicted onto target."""
    muX = np.mean(target, axis=1, keepdims=True)
    muY = np.mean(predicted, axis=1, keepdims=True)
    X0 = target - muX
    Y0 = predicted - muY
    normX = np.sqrt(np.sum(X0 ** 2, axis=(1, 2), keepdims=True))
    normY = np.sqrt(np.sum(Y0 ** 2, axis=(1, 2), keepdims=True))
    X0 /= normX
    Y0 /= normY
    H = np.matmul(X0.transpose(0, 2, 1), Y0)
    U, s, Vt = np.linalg.svd(H)
    V = Vt.transpose(0, 2, 1)
    R = np.matmul(V, U.transpose(0, 2, 1))
    sign_detR = np.sign(np.expand_dims(np.linalg.det(R), axis=1))  # no reflections
    V[:, :, -1] *= sign_detR
    s[:, -1] *= sign_detR.flatten()
    R = np.matmul(V, U.transpose(0, 2, 1))
    tr = np.expand_dims(np.sum(s, axis=1, keepdims=True), axis=2)
    a = tr * normX / normY
    t = muX - a * np.matmul(muY, R)
    aligned = a * np.matmul(predicted, R) + t
    return np.mean(np.linalg.norm(aligned - target, axis=len(target.shape) - 1), axis=len(target.shape) - 2)


def compute_error_accel(joints_gt, joints_pred):
    accel_gt = joints_gt[:-2] - 2 * joints_gt[1:-1] + joints_gt[2:]
    accel_pred = joints_pred[:-2] - 2 * joints_pred[1:-1] + joints_pred[2:]
    normed = np.linalg.norm(accel_pred - accel_gt, axis=2)
    return np.mean(normed, axis=1)


def compute_error_vel(joints_gt, joints_pred):
    vel_gt = joints_gt[1:] - joints_gt[:-1]
    vel_pred = joints_pred[1:] - joints_pred[:-1]
    normed = np.linalg.norm(vel_pred - vel_gt, axis=2)
    return np.mean(normed, axis=1)


def compute_metrics_lite(pred_pos_all, gt_pos_all):
    """Per-motion lists of [T,24,3] -> dict of per-frame arrays concatenated over motions."""
    metrics = defaultdict(list)
    for idx in range(len(pred_pos_all)):
        jpos_pred = pred_pos_all[idx].copy()
        jpos_gt = gt_pos_all[idx].copy()
        mpjpe_g = np.linalg.norm(jpos_gt - jpos_pred, axis=2).mean(axis=-1) * 1000
        vel_dist = compute_error_vel(jpos_pred, jpos_gt) * 1000
        accel_dist = compute_error_accel(jpos_pred, jpos_gt) * 1000
        jpos_pred = jpos_pred - jpos_pred[:, [0]]
        jpos_gt = jpos_gt - jpos_gt[:, [0]]
        pa_mpjpe = p_mpjpe(jpos_pred, jpos_gt) * 1000
        mpjpe = np.linalg.norm(jpos_pred - jpos_gt, axis=2).mean(axis=-1) * 1000
        metrics["mpjpe_g"].append(mpjpe_g)
        metrics["mpjpe_l"].append(mpjpe)
        metrics["mpjpe_pa"].append(pa_mpjpe)
        metrics["accel_dist"].append(accel_dist)
        metrics["vel_dist"].append(vel_dist)
    return {k: np.concatenate(v) for k, v in metrics.items()}


class HostEvalStats:
    """phc_train.py:62-164 bookkeeping over host copies (no env mutation): feed one step at a time;
    ``step`` returns "continue", "next_batch" or "done" exactly where the reference does."""

    def __init__(self, num_envs, num_unique_motions):
        self.num_envs, self.num_unique = num_envs, num_unique_motions
        self.terminate_state = np.zeros(num_envs, bool)
        self.played_steps_buf = np.zeros(num_envs, np.int16)
        self.terminate_memory, self.motion_length, self.played_steps = [], [], []
        self.gt_pos, self.pred_pos = [], []
        self.pred_pos_all, self.gt_pos_all = [], []
        self.curr_steps = 0
        self.success_rate = 0.0

    def step(self, motion_num_steps, terminate, curr_ids, body_pos, body_pos_gt, motion_sample_start_idx):
        motion_num_steps = np.asarray(motion_num_steps)
        termination_state = (self.curr_steps < motion_num_steps) & np.asarray(terminate, bool)
        self.terminate_state |= termination_state
        current_envs = ~self.terminate_state & (self.curr_steps < motion_num_steps)
        self.played_steps_buf[current_envs] += 1
        if (~self.terminate_state).sum() > 0:
            max_possible_id = self.num_unique - 1
            curr_ids = np.asarray(curr_ids)
            if (max_possible_id == curr_ids).sum() > 0:
                bound = np.flatnonzero(max_possible_id == curr_ids)[0] + 1
                if (~self.terminate_state[:bound]).sum() > 0:
                    curr_max = motion_num_steps[:bound][~self.terminate_state[:bound]].max()
                else:
                    curr_max = self.curr_steps - 1
                    self.terminate_state[bound:] = True
            else:
                curr_max = motion_num_steps[~self.terminate_state].max()
            if self.curr_steps >= curr_max:
                curr_max = self.curr_steps + 1
        else:
            curr_max = motion_num_steps.max()
        self.gt_pos.append(np.asarray(body_pos_gt))
        self.pred_pos.append(np.asarray(body_pos))
        self.curr_steps += 1
        if self.curr_steps >= curr_max or self.terminate_state.sum() == self.num_envs:
            self.curr_steps = 0
            self.terminate_memory.append(self.terminate_state.copy())
            self.motion_length.append(motion_num_steps.copy())
            self.played_steps.append(self.played_steps_buf.copy())
            self.success_rate = 1 - np.concatenate(self.terminate_memory)[: self.num_unique].mean()
            pred = np.stack(self.pred_pos)
            gt = np.stack(self.gt_pos)
            self.pred_pos_all += [pred[: (i - 1), idx] for idx, i in enumerate(motion_num_steps)]
            self.gt_pos_all += [gt[: (i - 1), idx] for idx, i in enumerate(motion_num_steps)]
            self.gt_pos, self.pred_pos = [], []
            if motion_sample_start_idx + self.num_envs >= self.num_unique:
                return "done"
            self.terminate_state[:] = False
            self.played_steps_buf[:] = 0
            return "next_batch"
        return "continue"

    def final_metrics(self):
        """get_final_stats's metrics_all_print / metrics_succ_print (phc_train.py:166-195)."""
        hist = np.concatenate(self.terminate_memory)[: self.num_unique]
        pred_all = self.pred_pos_all[: self.num_unique]
        gt_all = self.gt_pos_all[: self.num_unique]
        succ = np.flatnonzero(~hist).tolist()
        m_all = {m: float(np.mean(v)) for m, v in compute_metrics_lite(pred_all, gt_all).items()}
        m_succ = {m: float(np.mean(v)) for m, v in
                  compute_metrics_lite([pred_all[i] for i in succ], [gt_all[i] for i in succ]).items()}
        if len(m_succ) == 0:
            m_succ = m_all
        return m_all, m_succ, hist
