"""Multi-process (world_size 2, gloo, CPU) tests of the learner collectives and env sharding
(SURVEY §8e). The rollout data path itself has no collective: replicas are independent."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from humanoid_amd import dist as hd
    try:
        r, w, _ = hd.init("gloo")
        assert (r, w) == (rank, world)
        # gradients: rank-dependent values, averaged in 2 buckets
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.zeros(s)) for s in [(3, 5), (7,), (1000,), (2, 2)]]
        for i, p in enumerate(params):
            p.grad = torch.full_like(p, float(rank + 1)) * (i + 1)
        calls = hd.allreduce_gradients(params, bucket_bytes=2048)
        grads_ok = all(torch.allclose(p.grad, torch.full_like(p, 1.5 * (i + 1))) for i, p in enumerate(params))
        # running norm: synced update == single-process update on the concatenated batch
        g = torch.Generator().manual_seed(1)
        full = torch.randn(2 * 64, 934, generator=g) * 3 + 1
        mine = full[rank * 64:(rank + 1) * 64]

        class Norm:
            def __init__(self):
                self.running_mean = torch.zeros(1, 934)
                self.running_var = torch.ones(1, 934)
                self.count = torch.ones(1)
        a, b = Norm(), Norm()
        hd.synced_running_norm_update(a, mine)
        mean, var = full.mean(0, keepdim=True), full.var(0, unbiased=False, keepdim=True)
        b.running_mean = b.running_mean * 0 + mean
        b.running_var = b.running_var * 0 + var
        norm_ok = torch.allclose(a.running_mean, b.running_mean, atol=1e-5) and \
            torch.allclose(a.running_var, b.running_var, atol=1e-3)
        keys = hd.all_gather_failed_keys([f"clip{rank}", "shared"])
        shard = list(hd.env_shard(rank, 8))
        q.put((rank, calls, grads_ok, norm_ok, keys, shard, hd.rank_seed(1, rank)))
        dist.destroy_process_group()
    except Exception as exc:  # surface the failure to the parent
        q.put((rank, "error", repr(exc)))


def test_gloo_world2_collectives():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for r in res:
        assert r[1] != "error", r
    shards = []
    for rank, calls, grads_ok, norm_ok, keys, shard, seed in res:
        assert calls >= 2 and grads_ok and norm_ok
        assert keys == ["clip0", "clip1", "shared"]
        assert seed == 1 + rank
        shards += shard
    assert sorted(shards) == list(range(16))  # disjoint cover of the global env ids


def test_single_process_noops():
    from humanoid_amd import dist as hd
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.ones(3)
    assert hd.allreduce_gradients([p]) == 0
    assert hd.all_gather_failed_keys(["b", "a", "b"]) == ["a", "b"]
    m, v = hd.global_batch_moments(torch.tensor([[1.0], [3.0]]))
    assert np.allclose(m.numpy(), [[2.0]]) and np.allclose(v.numpy(), [[1.0]])
