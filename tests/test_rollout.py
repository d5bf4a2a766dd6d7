"""Rollout -> trainer handoff: include/humanoid_rollout.h through
humanoid_amd.experience against the host restatement oracle.HostExperience / oracle.gae.

CPU tests pin the oracle: GAE closed forms (the reference module could not be built here, so GAE
parity vs the reference module is unpinned) and a float32 scalar loop; the sort
against Python's sorted. GPU tests compare bit for bit: copies, index order and the GAE values
(the windowed device recurrence reproduces the serial float32 one, he_rollout.hip)."""
import numpy as np
import pytest

from oracle import oracle as O

GAMMA, LAM = 0.98, 0.2  # config.py:202-203


def _loop_gae(d, v, r, gamma, lam):
    """c_gae.pyx:23-30 with NumPy float32 scalars (one rounding per operation)."""
    f = np.float32
    n = len(r)
    adv = np.zeros(n, np.float32)
    last = f(0)
    g, gl = f(gamma), f(gamma) * f(lam)
    for t in range(n - 1):
        c, nx = n - 2 - t, n - 1 - t
        nnt = f(1.0 - float(d[nx]))
        delta = (f(r[nx]) + (g * f(v[nx])) * nnt) - f(v[c])
        last = delta + (gl * nnt) * last
        adv[c] = last
    return adv


def test_oracle_gae_closed_forms():
    rng = np.random.default_rng(0)
    n = 50
    v = rng.integers(-8, 8, n).astype(np.float32)
    r = rng.integers(-8, 8, n).astype(np.float32)
    # gamma = lambda = 1, no dones: adv[t] = sum_{k>t} r[k] + v[n-1] - v[t]
    adv = O.gae(np.zeros(n), v, r, 1.0, 1.0)
    want = np.array([r[t + 1:].sum() + v[-1] - v[t] for t in range(n - 1)] + [0.0], np.float32)
    np.testing.assert_array_equal(adv, want)
    # lambda = 0: adv[t] = delta[t] = r[t+1] + gamma v[t+1] (1 - d[t+1]) - v[t]
    d = (rng.random(n) < 0.3).astype(np.float32)
    adv = O.gae(d, v, r, 0.5, 0.0)
    want = np.append(r[1:] + 0.5 * v[1:] * (1 - d[1:]) - v[:-1], 0).astype(np.float32)
    np.testing.assert_array_equal(adv, want)
    # a done at t+1 cuts the recurrence: adv[t] = r[t+1] - v[t]
    d = np.zeros(n, np.float32)
    d[10] = 1
    adv = O.gae(d, v, r, 0.9, 0.7)
    assert adv[9] == r[10] - v[9]
    assert O.gae([], [], [], GAMMA, LAM).size == 0
    np.testing.assert_array_equal(O.gae([1], [3], [2], GAMMA, LAM), [0])


def test_oracle_gae_matches_float32_loop():
    rng = np.random.default_rng(1)
    for n, pd, g, lam in [(300, 0.02, GAMMA, LAM), (257, 0.0, 0.99, 0.95), (64, 0.5, 1.0, 1.0)]:
        d = (rng.random(n) < pd).astype(np.float32)
        v = rng.standard_normal(n).astype(np.float32) * 3
        r = rng.standard_normal(n).astype(np.float32)
        np.testing.assert_array_equal(O.gae(d, v, r, g, lam), _loop_gae(d, v, r, g, lam))


def test_oracle_sort_matches_python_sorted():
    rng = np.random.default_rng(2)
    keys = [(int(e), int(s)) for s in range(6) for e in rng.permutation(40)[:30]]
    keys += [keys[3]]  # a duplicate key: stability decides
    want = np.asarray(sorted(range(len(keys)), key=keys.__getitem__))
    got = O.sort_keys([k[0] for k in keys], [k[1] for k in keys])
    np.testing.assert_array_equal(got, want)


def test_host_experience_layout():
    """The host checker's minibatch layout is the reference's reshape/transpose (structs.py:130-137)."""
    hx = O.HostExperience(32, 4, 2, 4, 3, 2)
    rng = np.random.default_rng(3)
    for _ in range(4):
        n = 8
        hx.store(rng.random((n, 3), np.float32), rng.random(n, np.float32), rng.random((n, 2), np.float32),
                 rng.random(n, np.float32), rng.random(n, np.float32), np.zeros(n, np.float32),
                 np.zeros(n, np.float32), list(range(n)), np.ones(n, bool))
    assert hx.full
    idxs = hx.sort_training_data()
    np.testing.assert_array_equal(idxs, np.arange(32).reshape(4, 8).T.reshape(-1))
    hx.flatten_batch()
    assert hx.b_obs.shape == (2, 4, 4, 3) and hx.b_values.shape == (2, 16)


def test_experience_has_no_cpu_path():
    torch = pytest.importorskip("torch")
    from humanoid_amd.engine import EngineError
    from humanoid_amd.experience import Experience
    with pytest.raises(EngineError):
        Experience(64, 8, 32, 2, 4, (934,), np.float32, (69,), np.float32, False, "cpu", None, 8, False)
    del torch


# ------------------------------------------------------------------------------------------ GPU

def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("n,pd,g,lam", [(0, 0, GAMMA, LAM), (1, 0, GAMMA, LAM), (2, 0.5, GAMMA, LAM),
                                        (3, 0, GAMMA, LAM), (1000, 0.01, GAMMA, LAM), (131072, 0.005, GAMMA, LAM),
                                        (131072, 0.0, GAMMA, LAM), (20000, 0.0, 0.99, 0.95),
                                        (5000, 0.001, 1.0, 1.0), (3000, 0.0, 0.999, 0.999), (777, 0.1, 0.5, 0.0)])
def test_gpu_gae_bit_exact(n, pd, g, lam):
    import torch
    from humanoid_amd.experience import compute_gae
    rng = np.random.default_rng(n + int(1000 * pd))
    d = (rng.random(n) < pd).astype(np.float32)
    v = (rng.standard_normal(n) * 5).astype(np.float32)
    r = rng.standard_normal(n).astype(np.float32)
    want = O.gae(d, v, r, g, lam)
    got = compute_gae(torch.from_numpy(d).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(r).cuda(), g, lam)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(got.cpu().numpy()), _bits(want))
    # the Cython signature: NumPy in, NumPy out
    np.testing.assert_array_equal(_bits(compute_gae(d, v, r, g, lam)), _bits(want))


def _rollout(dev_exp, host_exp, num_envs, obs_dim, atn_dim, rng, mask_p, torch):
    """Drive both buffers with the same per-step data until full (core.py:129-183's store calls)."""
    env_id = list(range(num_envs))
    steps = 0
    while not host_exp.full:
        obs = rng.standard_normal((num_envs, obs_dim)).astype(np.float32)
        val = rng.standard_normal(num_envs).astype(np.float32)
        act = rng.standard_normal((num_envs, atn_dim)).astype(np.float32)
        lp = rng.standard_normal(num_envs).astype(np.float32)
        rew = rng.standard_normal(num_envs).astype(np.float32)
        done = rng.random(num_envs) < 0.05
        trunc = rng.random(num_envs) < 0.05
        mask = rng.random(num_envs) >= mask_p
        host_exp.store(obs, val, act, lp, rew, done.astype(np.float32), trunc.astype(np.float32), env_id, mask)
        c = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        dev_exp.store(c(obs), None, c(val), c(act), c(lp), c(rew), c(done), c(trunc), env_id,
                      None if mask_p == 0 else c(mask))
        assert dev_exp.ptr == host_exp.ptr
        steps += 1
    assert dev_exp.full
    return steps


@pytest.mark.gpu
@pytest.mark.parametrize("mask_p", [0.0, 0.3])
def test_gpu_experience_matches_host(mask_p):
    import torch
    from humanoid_amd.experience import Experience
    num_envs, obs_dim, atn_dim = 96, 934, 69
    bptt, num_mb, rows = 8, 3, 40
    batch = num_mb * rows * bptt  # 960 rows: 10 dense steps, or more with masking (last one cut)
    dev = Experience(batch, bptt, rows * bptt, num_mb, rows, (obs_dim,), np.float32, (atn_dim,), np.float32,
                     False, "cuda:0", None, num_envs, False)
    hx = O.HostExperience(batch, bptt, num_mb, rows, obs_dim, atn_dim)
    rng = np.random.default_rng(11)
    _rollout(dev, hx, num_envs, obs_dim, atn_dim, rng, mask_p, torch)
    idxs = dev.sort_training_data()
    want_idxs = hx.sort_training_data()
    np.testing.assert_array_equal(idxs.cpu().numpy(), want_idxs)
    dev.flatten_batch()
    hx.flatten_batch()
    for name in ("b_obs", "b_actions", "b_logprobs", "b_dones", "b_truncated", "b_values"):
        a, b = getattr(dev, name).cpu().numpy(), getattr(hx, name)
        assert a.shape == b.shape, name
        np.testing.assert_array_equal(a, b, err_msg=name)
    extra = rng.standard_normal(batch).astype(np.float32)
    for ex in (None, extra):
        dev.compute_advantages(GAMMA, LAM, None if ex is None else torch.from_numpy(ex).cuda())
        hx.compute_advantages(want_idxs, GAMMA, LAM, ex)
        np.testing.assert_array_equal(_bits(dev.b_advantages.cpu().numpy()), _bits(hx.b_advantages))
        np.testing.assert_array_equal(_bits(dev.b_returns.cpu().numpy()), _bits(hx.b_returns))
        np.testing.assert_array_equal(_bits(dev.returns.cpu().numpy()), _bits(hx.returns))
    # a second collection reuses the cleared counters
    dev.reset_collection()
    hx2 = O.HostExperience(batch, bptt, num_mb, rows, obs_dim, atn_dim)
    _rollout(dev, hx2, num_envs, obs_dim, atn_dim, rng, mask_p, torch)
    np.testing.assert_array_equal(dev.sort_training_data().cpu().numpy(), hx2.sort_training_data())


@pytest.mark.gpu
def test_gpu_experience_rejects_bad_env_ids():
    import torch
    from humanoid_amd.engine import EngineError
    from humanoid_amd.experience import Experience
    n = 16
    for ids in ([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 14],  # duplicate within one store
                torch.tensor([0] * 15 + [99], dtype=torch.int32, device="cuda:0")):  # out of range
        e = Experience(32, 2, 32, 1, 16, (4,), np.float32, (2,), np.float32, False, "cuda:0", None, n, False)
        for _ in range(2):
            z = torch.zeros(n, device="cuda:0")
            e.store(torch.zeros(n, 4, device="cuda:0"), None, z, torch.zeros(n, 2, device="cuda:0"), z, z, z, z, ids)
        with pytest.raises(EngineError):
            e.sort_training_data()


@pytest.mark.gpu
def test_gpu_order_full_size_properties():
    """BASELINE size (config.py:190-192: 131072 rows = 4096 envs x 32 steps, bptt 8, 4 minibatches):
    idxs is a permutation sorted by (env, step), and the gather agrees with torch indexing."""
    import torch
    from humanoid_amd.experience import Experience
    envs, steps, bptt, num_mb = 4096, 32, 8, 4
    batch = envs * steps
    rows = batch // num_mb // bptt
    e = Experience(batch, bptt, batch // num_mb, num_mb, rows, (934,), np.float32, (69,), np.float32, False,
                   "cuda:0", None, envs, False)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    perm_ids = [torch.randperm(envs, device="cuda:0", generator=g).to(torch.int32) for _ in range(steps)]
    for s in range(steps):
        z = torch.full((envs,), float(s), device="cuda:0")
        obs = torch.randn(envs, 934, device="cuda:0", generator=g)
        e.store(obs, None, perm_ids[s].float(), torch.zeros(envs, 69, device="cuda:0"), z, z, z, z, perm_ids[s])
    idxs = e.sort_training_data()
    assert torch.equal(torch.sort(idxs).values, torch.arange(batch, device="cuda:0"))
    env_of = e.values[idxs].long()   # the env id was stored as the value
    step_of = e.logprobs[idxs].long()  # and the step as the log-prob
    key = env_of * steps + step_of
    assert torch.equal(key, torch.arange(batch, device="cuda:0"))
    e.flatten_batch()
    assert torch.equal(e.b_obs, e.obs[e.b_idxs_obs])
    assert torch.equal(e.b_values, e.values[e.b_idxs_flat])


@pytest.mark.gpu
def test_episode_step_kernel_edges():
    """he_episode_step (PHCPufferEnv.step bookkeeping, clean_pufferl/env.py:120-160) against the
    torch restatement on random flags, including the all-reset and no-reset steps."""
    import torch
    from humanoid_amd.engine import load_library
    lib = load_library()
    rng = np.random.default_rng(7)
    n = 3000
    dev = "cuda:0"
    for mode in ("random", "all", "none"):
        reset = rng.random(n) < 0.3 if mode == "random" else np.full(n, mode == "all")
        term = reset & (rng.random(n) < 0.5)
        rew = torch.as_tensor(rng.standard_normal(n).astype(np.float32), device=dev)
        raw = torch.as_tensor(rng.random((n, 5)).astype(np.float32), device=dev)
        r8 = torch.as_tensor(reset.astype(np.uint8), device=dev)
        t8 = torch.as_tensor(term.astype(np.uint8), device=dev)
        ret = torch.as_tensor(rng.standard_normal(n).astype(np.float32), device=dev)
        ln = torch.as_tensor(rng.integers(0, 300, n).astype(np.int32), device=dev)
        ret0, ln0 = ret.clone(), ln.clone()
        raw_acc = torch.zeros(5, device=dev)
        acc = torch.zeros(5, dtype=torch.float64, device=dev)
        rew_out = torch.empty_like(rew)
        t_out, terminals, truncs, masks = (torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(4))
        rc = lib.he_episode_step(n, rew.data_ptr(), raw.data_ptr(), r8.data_ptr(), t8.data_ptr(), rew_out.data_ptr(),
                                 t_out.data_ptr(), terminals.data_ptr(), truncs.data_ptr(), masks.data_ptr(),
                                 ret.data_ptr(), ln.data_ptr(), raw_acc.data_ptr(), acc.data_ptr(), None)
        assert rc == 0
        torch.cuda.synchronize()
        rb, tb = r8.bool(), t8.bool()
        assert torch.equal(rew_out, rew) and torch.equal(t_out, t8)
        assert torch.equal(terminals.bool(), tb & rb) and torch.equal(truncs.bool(), rb & ~tb)
        assert torch.equal(masks.bool(), ~(rb & ~tb))
        assert torch.equal(ret, torch.where(rb, torch.zeros_like(ret0), ret0 + rew))
        assert torch.equal(ln, torch.where(rb, torch.zeros_like(ln0), ln0 + 1))
        want = [(ret0.double() * rb).sum(), (ln0.double() * rb).sum(), rb.double().sum(),
                (rb & ~tb).double().sum(), (tb & rb).double().sum()]
        np.testing.assert_allclose(acc.cpu().numpy(), [float(w) for w in want], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(raw_acc.cpu().numpy(), raw.mean(0).cpu().numpy(), rtol=1e-6)
    assert lib.he_episode_step(0, *([None] * 13), None) == 0
    assert lib.he_episode_step(-1, *([None] * 13), None) != 0
