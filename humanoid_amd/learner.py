"""The per-rank learner slice of BASELINE configs[3], for measurement and the multi-GPU rehearsal.

configs[3] is 8 ranks x 4096 envs with the PPO update and an RCCL gradient all-reduce. The trainer
is the reference's (out of scope). This module restates just enough of it to run one
rank's iteration on the engine, at the reference's sizes:

* :class:`PHCPolicy`: the reference-size network (``policies/phc_policy.py:23-66`` over
  ``discriminator_policy.py:11-111``; ``config.py:157-158``). Actor and critic are each an MLP
  934 -> 2048 -> 1536 -> 1024 -> 1024 -> 512 -> 512 with SiLU, then LayerNorm + SiLU. The actor adds a
  69-wide mean head and a fixed log-std of -2.9. The critic adds a 1-wide value head. That is
  16,984,134 trainable fp32 parameters (67.9 MB), SURVEY §8e.
* :class:`RunningNorm`: ``running_norm.py``, with the update on global batch moments
  (``dist.synced_running_norm_update``; ``phc_train.py:329-332``).
* :func:`collect`: ``clean_pufferl/core.py:130-183`` over :class:`~humanoid_amd.env.PHCPufferEnv`,
  stored into the device :class:`~humanoid_amd.experience.Experience`.
* :func:`train`: ``core.py:207-380``. It runs sort, flatten, GAE, then the clipped PPO objective
  with the clipped value loss and the mean-bound loss. Each minibatch step is
  backward -> gradient all-reduce -> clip -> Adam. The all-reduce sits where a multi-rank trainer
  inserts it: between ``loss.backward()`` (``core.py:366``) and ``clip_grad_norm_`` (``:373``).

The collectives run on device tensors through ``torch.distributed`` (RCCL over xGMI on the GPU
box). Nothing here is on the env step's hot path.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

OBS = 934
ACT = 69


@dataclass
class TrainConfig:
    """``config.py:188-212`` defaults (per rank: 4096 envs x 32 steps = batch 131072)."""
    batch_size: int = 131072
    minibatch_size: int = 32768
    bptt_horizon: int = 8
    update_epochs: int = 4
    learning_rate: float = 1e-4
    gamma: float = 0.98
    gae_lambda: float = 0.2
    clip_coef: float = 0.01
    vf_coef: float = 1.2
    clip_vloss: bool = True
    vf_clip_coef: float = 0.2
    max_grad_norm: float = 10.0
    ent_coef: float = 0.0
    norm_adv: bool = True
    bound_coef: float = 10.0

    @property
    def num_minibatches(self) -> int:
        return self.batch_size // self.minibatch_size

    @property
    def minibatch_rows(self) -> int:
        return self.minibatch_size // self.bptt_horizon


def _nn():
    import torch
    return torch.nn


def layer_init(layer, std: float = math.sqrt(2), bias_const: float = 0.0):
    """pufferlib.pytorch.layer_init: orthogonal weights with gain ``std``, constant bias."""
    import torch
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def _mlp(sizes):
    """phc_policy.py:11-20 ``mlp``: Linear+SiLU between the sizes, a bare Linear at the end."""
    nn = _nn()
    layers = []
    for a, b in zip(sizes[:-2], sizes[1:-1]):
        layers += [layer_init(nn.Linear(a, b)), nn.SiLU()]
    layers.append(layer_init(nn.Linear(sizes[-2], sizes[-1])))
    return layers


class RunningNorm:
    """running_norm.py: (x - mean) / sqrt(var + eps), clipped to +-10; update on batch moments."""

    def __init__(self, shape: int, device, epsilon: float = 1e-5, clip: float = 10.0):
        import torch
        self.running_mean = torch.zeros((1, shape), dtype=torch.float32, device=device)
        self.running_var = torch.ones((1, shape), dtype=torch.float32, device=device)
        self.count = torch.ones(1, dtype=torch.float32, device=device)
        self.epsilon, self.clip = epsilon, clip

    def __call__(self, x):
        import torch
        return torch.clamp((x - self.running_mean) / torch.sqrt(self.running_var + self.epsilon), -self.clip, self.clip)


def make_policy(device, hidden_size: int = 512, layer_sizes=(2048, 1536, 1024, 1024, 512)):
    """The reference-size :class:`PHCPolicy` on ``device``."""
    import torch
    nn = torch.nn

    class PHCPolicy(nn.Module):
        def __init__(self):
            super().__init__()
            sizes = [OBS] + list(layer_sizes) + [hidden_size]
            self.actor_mlp = nn.Sequential(*_mlp(sizes), nn.LayerNorm(hidden_size), nn.SiLU())
            self.critic_mlp = nn.Sequential(*_mlp(sizes), nn.LayerNorm(hidden_size), nn.SiLU(),
                                            layer_init(nn.Linear(hidden_size, 1), std=0.01))
            self.mu = nn.Sequential(layer_init(nn.Linear(hidden_size, ACT), std=0.01))
            # discriminator_policy.py:31-35: a constant log-std, not trained
            self.sigma = nn.Parameter(torch.full((ACT,), -2.9), requires_grad=False)
            self.soft_bound = 0.9  # 0.9 * action_space.high (clip_actions: [-1, 1])
            self.obs_norm = RunningNorm(OBS, device)

        def forward(self, obs, action=None):
            """pufferlib cleanrl Policy over encode/decode (phc_policy.py:45-66): actions sampled
            when ``action`` is None; returns (action, logprob, entropy, value, mean_bound_loss)."""
            x = self.obs_norm(obs)
            mu = self.mu(self.actor_mlp(x))
            std = torch.exp(self.sigma).expand_as(mu)
            probs = torch.distributions.Normal(mu, std)
            if action is None:
                action = probs.sample()
            value = self.critic_mlp(x)
            zero = torch.zeros_like(mu)
            bl = torch.where(mu > self.soft_bound, (mu - self.soft_bound) ** 2, zero)
            bl = torch.where(mu < -self.soft_bound, (mu + self.soft_bound) ** 2, bl)  # bound_loss (:107-111)
            return action, probs.log_prob(action).sum(-1), probs.entropy().sum(-1), value, bl.mean()

    return PHCPolicy().to(device)


def num_trainable(policy) -> int:
    return sum(p.numel() for p in policy.parameters() if p.requires_grad)


def make_experience(num_envs: int, cfg: TrainConfig, device):
    from .experience import Experience
    return Experience(batch_size=cfg.batch_size, bptt_horizon=cfg.bptt_horizon, minibatch_size=cfg.minibatch_size,
                      num_minibatches=cfg.num_minibatches, minibatch_rows=cfg.minibatch_rows, obs_shape=(OBS,),
                      obs_dtype=np.float32, atn_shape=(ACT,), atn_dtype=np.float32, cpu_offload=False, device=device,
                      lstm=None, lstm_total_agents=num_envs, use_amp_obs=False)


def collect(pe, policy, ex, obs, env_id):
    """core.py:130-183 until the experience is full. ``obs`` is the env's current observation
    tensor; returns the observation after the last step."""
    import torch
    while not ex.full:
        with torch.no_grad():
            action, logprob, _, value, _ = policy(obs)
        nobs, rew, term, trunc, _ = pe.step(action)
        ex.store(obs, None, value.flatten(), action, logprob, rew, term, trunc, env_id, mask=pe.masks)
        obs = nobs
    return obs


def train(policy, opt, ex, cfg: TrainConfig, sync_grads=None, epochs: Optional[int] = None,
          max_minibatches: Optional[int] = None, timers: Optional[Dict[str, float]] = None):
    """core.py:207-380 on the device experience; ``sync_grads(params)`` runs between
    ``loss.backward()`` and ``clip_grad_norm_``. Returns the mean losses. ``timers`` (a dict)
    accumulates 'gae_ms', 'update_ms' and 'allreduce_ms' of the phases (the clock is synchronised
    around each phase: for measurement only)."""
    import torch

    def tick():
        if timers is not None:
            torch.cuda.synchronize()
        return time.perf_counter()

    t0 = tick()
    ex.sort_training_data()
    ex.flatten_batch()
    ex.compute_advantages(cfg.gamma, cfg.gae_lambda)
    t1 = tick()
    if timers is not None:
        timers["gae_ms"] = timers.get("gae_ms", 0.0) + (t1 - t0) * 1e3
    params = [p for p in policy.parameters() if p.requires_grad]
    epochs = cfg.update_epochs if epochs is None else epochs
    stats = {"pg_loss": 0.0, "v_loss": 0.0, "bound_loss": 0.0, "minibatches": 0}
    for _ in range(epochs):
        for mb in range(ex.num_minibatches):
            if max_minibatches is not None and stats["minibatches"] >= max_minibatches:
                break
            ta = tick()
            obs = ex.b_obs[mb].reshape(-1, OBS)
            atn = ex.b_actions[mb].reshape(-1, ACT)
            _, newlogprob, entropy, newvalue, bound = policy(obs, atn)
            logratio = newlogprob - ex.b_logprobs[mb].reshape(-1)
            ratio = logratio.exp()
            adv = ex.b_advantages[mb].reshape(-1)
            if cfg.norm_adv:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            pg = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)).mean()
            newvalue = newvalue.view(-1)
            ret, val = ex.b_returns[mb], ex.b_values[mb]
            if cfg.clip_vloss:
                v_clipped = val + torch.clamp(newvalue - val, -cfg.vf_clip_coef, cfg.vf_clip_coef)
                v_loss = torch.max((newvalue - ret) ** 2, (v_clipped - ret) ** 2).mean()
            else:
                v_loss = ((newvalue - ret) ** 2).mean()
            loss = pg - cfg.ent_coef * entropy.mean() + v_loss * cfg.vf_coef + bound * cfg.bound_coef
            opt.zero_grad(set_to_none=False)  # in place: gradients may be all-reduce bucket views
            loss.backward()
            tb = tick()
            if sync_grads is not None:
                sync_grads(params)
            tc = tick()
            torch.nn.utils.clip_grad_norm_(params, cfg.max_grad_norm)
            opt.step()
            td = tick()
            if timers is not None:
                timers["update_ms"] = timers.get("update_ms", 0.0) + (td - ta) * 1e3
                timers["allreduce_ms"] = timers.get("allreduce_ms", 0.0) + (tc - tb) * 1e3
            stats["pg_loss"] += float(pg.detach())
            stats["v_loss"] += float(v_loss.detach())
            stats["bound_loss"] += float(bound.detach())
            stats["minibatches"] += 1
    k = max(stats["minibatches"], 1)
    for key in ("pg_loss", "v_loss", "bound_loss"):
        stats[key] /= k
    return stats
