"""The rollout -> learner loop on the GPU (SURVEY §8e and BASELINE configs[0] / configs[3]).

* configs[0]-style plumbing (phc_train.py:278-370 -> clean_pufferl/core.py:130-183, 207-443) at 16
  envs: PHCPufferEnv -> device Experience (store, sort, flatten) -> GAE -> one PPO minibatch step of a
  PHCPolicy-shaped MLP (934 -> ... -> 69 Gaussian actor + value head), all on cuda:0.
* configs[3] logic on one GPU (the driver runs the real 8-GPU node): two ranks spawned fresh (they
  touch the GPU only in their own process), both on cuda:0, gloo collectives (the
  HE_BENCH_SHARED_DEVICE rehearsal pattern). Each rank owns a disjoint env shard with its own
  engine and seed (config.py:173), collects its own rollout, keeps its obs normaliser in sync
  (synced_running_norm_update) and averages its gradients (allreduce_gradients, between
  core.py:366 and :373); after the update the policy parameters are bit-identical on both ranks.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N_ENVS = 16
BPTT = 8


def _clips(model, k=4, frames=90):
    from humanoid_amd import synthetic
    return {f"clip{i}": synthetic.make_clip(model, np.random.default_rng(100 + i), num_frames=frames) for i in range(k)}


class Policy(torch.nn.Module):
    """PHCPolicy-shaped (policy.py): obs 934 -> MLP actor mean 69 with a learned log-std, MLP critic 1
    (narrower hidden layers than the reference's, the same interface)."""

    def __init__(self, hidden=256):
        super().__init__()
        self.actor = torch.nn.Sequential(torch.nn.Linear(934, hidden), torch.nn.SiLU(), torch.nn.Linear(hidden, hidden),
                                         torch.nn.SiLU(), torch.nn.Linear(hidden, 69))
        self.critic = torch.nn.Sequential(torch.nn.Linear(934, hidden), torch.nn.SiLU(), torch.nn.Linear(hidden, 1))
        self.logstd = torch.nn.Parameter(torch.full((69,), -2.9))

    def dist(self, obs):
        return torch.distributions.Normal(self.actor(obs), self.logstd.exp())


class RunningNorm:
    """running_norm.py:22-34 state (mean, var, count)."""

    def __init__(self, device):
        self.running_mean = torch.zeros(1, 934, device=device)
        self.running_var = torch.ones(1, 934, device=device)
        self.count = torch.ones(1, device=device)

    def __call__(self, x):
        return (x - self.running_mean) / torch.sqrt(self.running_var + 1e-5)


def collect_and_update(pe, policy, norm, opt, steps=BPTT, sync_norm=None, sync_grads=None, seed=0):
    """One collection of `steps` policy steps (core.py:130-183) and one PPO minibatch step
    (core.py:303-380). Returns (loss, experience)."""
    from humanoid_amd.experience import Experience
    n = pe.num_agents
    dev = torch.device("cuda", 0)
    ex = Experience(batch_size=n * steps, bptt_horizon=steps, minibatch_size=n * steps // 2, num_minibatches=2,
                    minibatch_rows=n // 2, obs_shape=(934,), obs_dtype=np.float32, atn_shape=(69,),
                    atn_dtype=np.float32, cpu_offload=False, device=dev, lstm=None, lstm_total_agents=n,
                    use_amp_obs=False)
    g = torch.Generator(device=dev).manual_seed(seed)
    obs, _ = pe.reset()
    env_id = np.arange(n)
    for _ in range(steps):
        with torch.no_grad():
            d = policy.dist(norm(obs))
            action = d.mean + d.stddev * torch.randn(d.mean.shape, generator=g, device=dev)
            logprob = d.log_prob(action).sum(-1)
            value = policy.critic(norm(obs)).squeeze(-1)
        nobs, rew, term, trunc, _ = pe.step(action.contiguous())
        ex.store(obs, None, value, action, logprob, rew, term.float(), trunc.float(), env_id, mask=pe.masks)
        obs = nobs
    ex.sort_training_data()
    ex.flatten_batch()
    ex.compute_advantages(0.98, 0.2)  # config.py:202-203
    if sync_norm is not None:  # phc_train.py:331-332: the normaliser update, on global moments
        sync_norm(norm, ex.obs)
    # PPO clipped objective on minibatch 0 (core.py:303-380, clip 0.2, vf 0.5, ent 0)
    mb_obs = ex.b_obs[0].reshape(-1, 934)
    mb_act = ex.b_actions[0].reshape(-1, 69)
    old_lp = ex.b_logprobs[0].reshape(-1)
    adv = ex.b_advantages[0]
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    d = policy.dist(norm(mb_obs))
    ratio = (d.log_prob(mb_act).sum(-1) - old_lp).exp()
    pg = torch.max(-adv * ratio, -adv * ratio.clamp(0.8, 1.2)).mean()
    v = policy.critic(norm(mb_obs)).squeeze(-1)
    loss = pg + 0.5 * ((v - ex.b_returns[0]) ** 2).mean()
    opt.zero_grad()
    loss.backward()
    if sync_grads is not None:
        sync_grads(list(policy.parameters()))
    torch.nn.utils.clip_grad_norm_(policy.parameters(), 1.0)
    opt.step()
    return float(loss.detach()), ex


def _param_digest(policy):
    h = hashlib.sha256()
    for p in policy.parameters():
        h.update(p.detach().cpu().numpy().tobytes())
    return h.hexdigest()


def test_configs0_loop_16_envs(model):
    """configs[0] plumbing at 16 envs: env -> Experience -> GAE -> minibatch step, finite and
    consistent (every stored row is one env-step; the update moves the parameters)."""
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    pe = PHCPufferEnv(EnvConfig(num_envs=N_ENVS, motion_file=_clips(model), seed=1))
    torch.manual_seed(0)
    policy = Policy().cuda()
    opt = torch.optim.Adam(policy.parameters(), lr=2e-5)
    before = _param_digest(policy)
    loss, ex = collect_and_update(pe, policy, RunningNorm("cuda"), opt)
    assert np.isfinite(loss)
    assert ex.ptr == N_ENVS * BPTT
    assert torch.isfinite(ex.b_advantages).all() and torch.isfinite(ex.b_returns).all()
    # sorted rows: each env's BPTT steps are contiguous (structs.py:128-142)
    assert ex.b_obs.shape == (2, N_ENVS // 2, BPTT, 934)
    assert _param_digest(policy) != before
    pe.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        import torch.distributed as dist
        from humanoid_amd import dist as hd
        from humanoid_amd.env import EnvConfig, PHCPufferEnv
        from humanoid_amd.model import load_default_model
        r, w, _ = hd.init("gloo")  # every rank on cuda:0: the shared-device rehearsal (gloo)
        torch.cuda.set_device(0)
        model = load_default_model()
        pe = PHCPufferEnv(EnvConfig(num_envs=N_ENVS, motion_file=_clips(model), seed=hd.rank_seed(1, r)))
        torch.manual_seed(0)  # identical initial policy on every rank
        policy = Policy().cuda()
        opt = torch.optim.Adam(policy.parameters(), lr=2e-5)
        norm = RunningNorm("cuda")

        def sync_grads(params):
            # gloo reduces host tensors: the gradients make the round trip through the host
            for p in params:
                g = p.grad.detach().cpu()
                p.grad.data = g
            hd.allreduce_gradients(params)
            for p in params:
                p.grad.data = p.grad.data.cuda()

        def sync_norm(nm, x):
            c = RunningNorm("cpu")
            hd.synced_running_norm_update(c, x.detach().cpu())
            nm.running_mean.copy_(c.running_mean)
            nm.running_var.copy_(c.running_var)
            nm.count.copy_(c.count)

        loss, ex = collect_and_update(pe, policy, norm, opt, sync_norm=sync_norm, sync_grads=sync_grads, seed=r)
        obs_sum = float(ex.obs.double().sum())
        q.put((r, _param_digest(policy), list(hd.env_shard(r, N_ENVS)), obs_sum, loss,
               float(norm.running_mean.double().sum())))
        pe.close()
        dist.destroy_process_group()
    except Exception as exc:  # surface the failure to the parent
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_world2_ranks_rollout_and_synced_update():
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for r in res:
        assert r[1] != "error", r[2]
    (_, d0, s0, o0, l0, m0), (_, d1, s1, o1, l1, m1) = res
    assert d0 == d1, "policy parameters differ across ranks after the synced update"
    assert m0 == m1, "obs normalisers differ across ranks"
    assert not set(s0) & set(s1) and sorted(s0 + s1) == list(range(2 * N_ENVS))  # disjoint env shards
    assert o0 != o1, "ranks must collect different rollouts (seed 1 + rank)"


def _rccl_world1_worker(port, q):
    """configs[3] per-rank slice at the reference's sizes through a one-rank RCCL group."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        import torch.distributed as dist
        from humanoid_amd import dist as hd, learner as L
        from humanoid_amd.env import EnvConfig, PHCPufferEnv
        from humanoid_amd.model import load_default_model
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        model = load_default_model()
        n = 4096
        cfg = L.TrainConfig()
        pe = PHCPufferEnv(EnvConfig(num_envs=n, motion_file=_clips(model, k=8, frames=150), seed=1))
        torch.manual_seed(0)
        policy = L.make_policy(dev)
        nparams = L.num_trainable(policy)
        opt = torch.optim.Adam(policy.parameters(), lr=cfg.learning_rate, eps=1e-5)
        ex = L.make_experience(n, cfg, dev)
        obs, _ = pe.reset()
        L.collect(pe, policy, ex, obs, np.arange(n))
        rows = ex.ptr
        hd.synced_running_norm_update(policy.obs_norm, ex.obs)
        before = [p.detach().clone() for p in policy.parameters() if p.requires_grad]
        seen = {}

        def sync_grads(params):
            pre = torch.cat([p.grad.reshape(-1) for p in params]).clone()
            seen["calls"] = hd.allreduce_gradients(params, min_world=1)
            post = torch.cat([p.grad.reshape(-1) for p in params])
            seen["identical"] = bool(torch.equal(pre, post))  # sum over one rank / 1 = the gradient itself
            seen["grad_bytes"] = int(pre.numel() * 4)
            seen["finite"] = bool(torch.isfinite(pre).all())

        stats = L.train(policy, opt, ex, cfg, sync_grads=sync_grads, epochs=1, max_minibatches=1)
        # the bucket-view form: all-reduces launched from the backward hooks on the flat buckets
        gb = hd.GradBuckets(policy.parameters(), min_world=1)

        def sync_buckets(params):
            pre = torch.cat([p.grad.reshape(-1) for p in params]).clone()
            seen["bucket_calls"] = gb.finish()
            seen["bucket_identical"] = bool(torch.equal(pre, torch.cat([p.grad.reshape(-1) for p in params])))

        L.train(policy, opt, ex, cfg, sync_grads=sync_buckets, epochs=1, max_minibatches=1)
        seen["buckets"] = len(gb.buckets)
        moved = sum(int(not torch.equal(b, p.detach())) for b, p in
                    zip(before, [p for p in policy.parameters() if p.requires_grad]))
        adv_ok = bool(torch.isfinite(ex.b_advantages).all() and torch.isfinite(ex.b_returns).all())
        q.put(("ok", backend, nparams, rows, seen, stats, moved, adv_ok, tuple(ex.b_obs.shape)))
        pe.close()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put(("error", traceback.format_exc()))


def test_configs3_rank_slice_through_rccl_world1():
    """BASELINE configs[3] per rank on one GPU: 4096 envs x 32 steps into the device Experience with
    the reference-size policy (16,984,134 params, phc_policy.py:23-66) in the loop, GAE, one PPO
    minibatch step of 32768 rows, and the 67.9 MB gradient all-reduce on device tensors between
    backward and clip (core.py:366-373) through a one-rank RCCL ("nccl") group."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_world1_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert res[0] == "ok", res[1]
    _, backend, nparams, rows, seen, stats, moved, adv_ok, bshape = res
    assert backend == "nccl"
    assert nparams == 16_984_134
    assert rows == 131072 and bshape == (4, 4096, 8, 934)
    assert seen["calls"] == 2 and seen["grad_bytes"] == 67_936_536  # 2 buckets of <= 64 MB
    assert seen["identical"] and seen["finite"]
    assert seen["bucket_calls"] == seen["buckets"] >= 4 and seen["bucket_identical"]
    assert adv_ok and all(np.isfinite(v) for v in (stats["pg_loss"], stats["v_loss"], stats["bound_loss"]))
    assert moved > 0
