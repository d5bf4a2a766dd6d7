"""Rollout -> trainer handoff timing at the reference's PPO batch (config.py:190-203:
batch 131072 = 4096 envs x 32 steps, bptt 8, minibatch 32768 -> 4 minibatches, obs 934, actions 69).

Device path (humanoid_amd.experience.Experience): 32 stores of 4096 rows (obs/actions/values/...
already on the GPU, as the env and policy leave them), sort_training_data, flatten_batch,
compute_advantages; each phase timed with HIP events on the current stream.
Host path (the reference's data flow, restated by oracle.HostExperience): per store the five
`.cpu().numpy()` copies + the Python sort-key list (structs.py:108-126), then the Python `sorted`,
the host gathers (obs stays on the device in the reference, gathered there by torch indexing) and
the C restatement of the Cython GAE, plus the advantage H2D copy (core.py:249).

Usage: python tests/diag/handoff_bench.py [--out profiles/r01/handoff_bench.json] [--mask]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from humanoid_amd.experience import Experience  # noqa: E402
from oracle import oracle as O  # noqa: E402

ENVS, STEPS, BPTT, NUM_MB, OBS, ATN = 4096, 32, 8, 4, 934, 69
BATCH = ENVS * STEPS
ROWS = BATCH // NUM_MB // BPTT
GAMMA, LAM = 0.98, 0.2


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--mask", action="store_true", help="store with a (truncation) mask, as PHCPufferEnv does")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    step_data = []
    for s in range(STEPS):
        step_data.append(dict(obs=torch.randn(ENVS, OBS, device=dev, generator=g),
                              val=torch.randn(ENVS, device=dev, generator=g),
                              act=torch.randn(ENVS, ATN, device=dev, generator=g),
                              lp=torch.randn(ENVS, device=dev, generator=g),
                              rew=torch.randn(ENVS, device=dev, generator=g),
                              done=torch.rand(ENVS, device=dev, generator=g) < 0.01,
                              trunc=torch.zeros(ENVS, dtype=torch.bool, device=dev)))
    env_ids = torch.arange(ENVS, dtype=torch.int32, device=dev)
    mask = torch.ones(ENVS, dtype=torch.bool, device=dev) if a.mask else None
    e = Experience(BATCH, BPTT, BATCH // NUM_MB, NUM_MB, ROWS, (OBS,), np.float32, (ATN,), np.float32, False, dev,
                   None, ENVS, False)

    def collect():
        e.reset_collection()
        for d in step_data:
            e.store(d["obs"], None, d["val"], d["act"], d["lp"], d["rew"], d["done"], d["trunc"], env_ids, mask)

    store_ms = timed(collect, a.reps) / STEPS
    sort_ms = timed(e.sort_training_data, a.reps)  # includes the once-per-batch error check (sync)
    flat_ms = timed(e.flatten_batch, a.reps)
    gae_ms = timed(lambda: e.compute_advantages(GAMMA, LAM), a.reps)

    # algorithmic HBM bytes: store reads+writes every field once; the gather the same plus idxs
    row_bytes = 4 * (OBS + ATN + 5)
    store_bytes = ENVS * (2 * row_bytes + 4 + 8)
    gather_bytes = BATCH * (2 * 4 * (OBS + ATN + 4) + 8)
    res = {"config": dict(envs=ENVS, steps=STEPS, batch=BATCH, bptt=BPTT, num_minibatches=NUM_MB, obs=OBS, atn=ATN,
                          masked_store=bool(a.mask)),
           "device_ms": dict(store_per_step=round(store_ms, 4), sort=round(sort_ms, 4), flatten=round(flat_ms, 4),
                             gae_minibatch=round(gae_ms, 4),
                             per_batch_total=round(store_ms * STEPS + sort_ms + flat_ms + gae_ms, 3)),
           "store_GBps": round(store_bytes / store_ms / 1e6, 1), "flatten_GBps": round(gather_bytes / flat_ms / 1e6, 1)}

    # host path: the reference's flow over the same data
    hx = O.HostExperience(BATCH, BPTT, NUM_MB, ROWS, OBS, ATN)
    t0 = time.perf_counter()
    ones = np.ones(ENVS, bool)
    for d in step_data:
        torch.cuda.synchronize()
        vals = [d[k].float().cpu().numpy() for k in ("val", "lp", "rew", "done", "trunc")]
        act = d["act"].cpu().numpy()  # the action D2H (core.py:170)
        idx = np.where(ones)[0]
        p = hx.ptr
        hx.values[p:p + ENVS], hx.logprobs[p:p + ENVS], hx.rewards[p:p + ENVS] = vals[0][idx], vals[1][idx], vals[2][idx]
        hx.dones[p:p + ENVS], hx.truncateds[p:p + ENVS] = vals[3][idx], vals[4][idx]
        hx.actions[p:p + ENVS] = act[idx]
        hx.sort_keys.extend([(i, hx.step) for i in env_ids.tolist()])
        hx.ptr += ENVS
        hx.step += 1
    t1 = time.perf_counter()
    keys = hx.sort_keys
    idxs = np.asarray(sorted(range(len(keys)), key=keys.__getitem__))  # structs.py:129
    t2 = time.perf_counter()
    b = idxs.reshape(ROWS, NUM_MB, BPTT).transpose(1, 0, 2)
    bt = torch.as_tensor(b).to(dev).long()
    obs_dev = e.obs  # the reference keeps obs on the device and gathers it there
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    _ = obs_dev[bt]
    for arr in (hx.actions, hx.logprobs, hx.dones, hx.truncateds):
        torch.as_tensor(arr).to(dev)[bt]
    torch.as_tensor(hx.values).to(dev)[bt.reshape(NUM_MB, -1)]
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    adv = O.gae(hx.dones[idxs], hx.values[idxs], hx.rewards[idxs], GAMMA, LAM)
    torch.as_tensor(adv).to(dev)
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    ms = lambda x: round(1e3 * x, 3)  # noqa: E731
    res["host_path_ms"] = dict(store_per_step=ms((t1 - t0) / STEPS), sort=ms(t2 - t1), flatten=ms(t4 - t3),
                               gae=ms(t5 - t4), per_batch_total=ms((t1 - t0) + (t2 - t1) + (t4 - t3) + (t5 - t4)))
    res["speedup_per_batch"] = round(res["host_path_ms"]["per_batch_total"] / res["device_ms"]["per_batch_total"], 1)
    print(json.dumps(res))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
