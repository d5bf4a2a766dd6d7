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


def _bucket_worker(rank, world, port, q):
    """GradBuckets (overlapped bucket all-reduce during backward) against allreduce_gradients on
    the same model and per-rank batches: the averaged gradients are equal, and two steps in a row
    keep the views (zero_grad(set_to_none=False))."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from humanoid_amd import dist as hd
    try:
        hd.init("gloo")

        def model():
            torch.manual_seed(0)
            return torch.nn.Sequential(torch.nn.Linear(40, 64), torch.nn.SiLU(), torch.nn.Linear(64, 64),
                                       torch.nn.LayerNorm(64), torch.nn.Linear(64, 3))
        g = torch.Generator().manual_seed(10 + rank)
        xs = [torch.randn(32, 40, generator=g) for _ in range(2)]
        ref, mine = model(), model()
        ok = True
        opt_r = torch.optim.SGD(ref.parameters(), lr=0.1)
        opt_m = torch.optim.SGD(mine.parameters(), lr=0.1)
        gb = hd.GradBuckets(mine.parameters(), bucket_bytes=4096, overlap=True)
        calls = []
        for x in xs:
            opt_r.zero_grad()
            ref(x).square().mean().backward()
            hd.allreduce_gradients(list(ref.parameters()))
            opt_m.zero_grad(set_to_none=False)
            mine(x).square().mean().backward()
            calls.append(gb.finish())
            for a, b in zip(ref.parameters(), mine.parameters()):
                ok = ok and torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-7)
            opt_r.step()
            opt_m.step()
        # one backward() per finish(): a second backward before finish() raises instead of adding
        # into buffers whose all-reduce is in flight
        opt_m.zero_grad(set_to_none=False)
        mine(xs[0]).square().mean().backward()
        try:
            mine(xs[1]).square().mean().backward()
            refused = False
        except RuntimeError as exc:
            refused = "one backward() per finish()" in str(exc)
        gb.finish()
        # a parameter with no gradient on one rank (a branch rank 1 skips): the buckets still go out in
        # index order on both ranks (no hang), and the average matches allreduce_gradients
        torch.manual_seed(1)
        trunk, branch = torch.nn.Linear(40, 64), torch.nn.Linear(64, 64)
        head = torch.nn.Linear(64, 3)
        net = torch.nn.ModuleList([trunk, branch, head])
        ref2 = [p.detach().clone().requires_grad_(True) for p in net.parameters()]
        gb2 = hd.GradBuckets(net.parameters(), bucket_bytes=2048, overlap=True)
        h = trunk(xs[0])
        if rank == 0:
            h = branch(h)
        head(h).square().mean().backward()
        gb2.finish()
        pr = dict(zip(["tw", "tb", "bw", "bb", "hw", "hb"], ref2))
        h = xs[0] @ pr["tw"].T + pr["tb"]
        if rank == 0:
            h = h @ pr["bw"].T + pr["bb"]
        (h @ pr["hw"].T + pr["hb"]).square().mean().backward()
        for t in ref2:
            if t.grad is None:
                t.grad = torch.zeros_like(t)
        hd.allreduce_gradients(ref2)
        skip_ok = all(torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-7) for a, b in zip(ref2, net.parameters()))
        q.put((rank, ok and refused and skip_ok, calls, len(gb.buckets)))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_gloo_world2_overlapped_grad_buckets():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
        _, ok, calls, nb = r
        assert ok and nb >= 3 and calls == [nb, nb]


def test_grad_buckets_refuse_lost_views():
    from humanoid_amd import dist as hd
    m = torch.nn.Linear(4, 2)
    gb = hd.GradBuckets(m.parameters(), overlap=False)
    m(torch.ones(1, 4)).sum().backward()
    assert gb.finish() == 0  # no process group: nothing to reduce
    m.zero_grad(set_to_none=True)
    with pytest.raises(RuntimeError, match="bucket view"):
        gb.finish()


def test_single_process_noops():
    from humanoid_amd import dist as hd
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.ones(3)
    assert hd.allreduce_gradients([p]) == 0
    assert hd.all_gather_failed_keys(["b", "a", "b"]) == ["a", "b"]
    m, v = hd.global_batch_moments(torch.tensor([[1.0], [3.0]]))
    assert np.allclose(m.numpy(), [[2.0]]) and np.allclose(v.numpy(), [[1.0]])
