"""Trace the fastest root of the random-action regime.

Protocol of tools/action_regimes.py: 4096 standing envs (cases.standing_state, numpy seed 8,
xy jitter 1 m), 60 policy steps of actions U(-amp, amp) x the PD scale, new every step. Pass 1
finds the env whose root gets fastest and the step where that happens. Pass 2 repeats the same
run, which is bit-reproducible. It records that env's state, PD targets and warm-start cache at
every step, together with what the solver held at each step's end: contacts by kind (terrain,
self, joint limit), the dropped contacts, and the largest joint angle. Replays then run the env
through the fp64 oracle from 6 steps before the peak with the same targets:
  (a) the engine's scheme (2 simulate() x 2 substeps of 1/120 s);
  (b) the same interval at dt/4 (8 substeps of 1/480 s per simulate).
Usage (GPU): python tests/diag/trace_runaway.py [amp ...] > gpurun_out/trace_runaway.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))

import cases  # noqa: E402


def com_speed(model, rb):
    v = cases.com_velocity(model, rb)
    return np.linalg.norm(v, axis=-1)


def run(hm, model, amp, n, steps, capture=None):
    import torch
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import pd_action_offset_scale
    off, sc = pd_action_offset_scale(model)
    rng = np.random.default_rng(8)
    eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params())
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
    eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
    speeds = np.zeros((steps, n), np.float32)
    trace = []
    for k in range(steps):
        a = rng.uniform(-amp, amp, (n, 69)).astype(np.float32)
        if capture is not None:
            e = capture
            trace.append(dict(root=eng.root_states[e].cpu().numpy().copy(),
                              dof=eng.dof_state.view(n, 69, 2)[e].cpu().numpy().copy(),
                              cache=eng.contact_cache[e].cpu().numpy().copy(),
                              targets=(off + sc * a[e]).astype(np.float32)))
        eng.dof_targets.copy_(torch.as_tensor(off + sc * a, device="cuda:0"))
        eng.simulate(2)
        speeds[k] = eng.root_states[:, 7:10].norm(dim=1).cpu().numpy()
        if capture is not None:
            e = capture
            trace[-1].update(root_after=eng.root_states[e].cpu().numpy().copy(),
                             rb_after=eng.rb_state.view(n, 24, 13)[e].cpu().numpy().copy(),
                             cache_after=eng.contact_cache[e].cpu().numpy().copy(),
                             dropped=int(eng.dropped_contacts[e].item()),
                             slots=int(eng.num_contacts[e].item()))
    torch.cuda.synchronize()
    del eng
    return speeds, trace


def contact_kinds(cache):
    from humanoid_amd import _abi
    cnt, keys, lam = _abi.cache_rows(cache[None])
    out = {"terrain": 0, "self": 0, "limit": 0, "limit_impulse": 0.0, "self_bodies": []}
    for r in range(int(cnt[0])):
        b0, b1, sub, kind = _abi.key_fields(keys[0, r])
        if kind != 0:
            continue
        if b1 == -1:
            out["terrain"] += 1
        elif b1 == -2:
            out["limit"] += 1
            out["limit_impulse"] = max(out["limit_impulse"], float(lam[0, r]))
        else:
            out["self"] += 1
            out["self_bodies"].append([int(b0), int(b1)])
    return out


def replay(hm, model, tr, k0, k1, substeps):
    from humanoid_amd import _abi
    from oracle import oracle as O
    sp = _abi.default_sim_params(substeps=substeps)
    root = tr[k0]["root"][None].copy()
    dof = tr[k0]["dof"][None].copy()
    cache = tr[k0]["cache"][None].copy() if substeps == _abi.default_sim_params().substeps else O.new_cache(1)
    out = []
    for k in range(k0, k1):
        o = O.physics_step(hm, sp, root, dof, tr[k]["targets"][None].copy(), 2, cache=cache)
        out.append({"step": k, "root_speed": float(np.linalg.norm(root[0, 7:10])),
                    "com_speed": float(com_speed(model, o["rb_state"])[0])})
    return out


def main():
    from humanoid_amd import _abi
    from humanoid_amd.body_sets import BODY_NAMES
    from humanoid_amd.model import load_default_model
    model = load_default_model()
    hm = _abi.make_model(model)
    amps = [float(a) for a in sys.argv[1:]] or [0.75]
    n, steps = 4096, 60
    res = {}
    for amp in amps:
        speeds, _ = run(hm, model, amp, n, steps)
        vmax = speeds.max(0)
        e = int(vmax.argmax())
        kpk = int(speeds[:, e].argmax())
        _, tr = run(hm, model, amp, n, steps, capture=e)
        assert abs(float(np.linalg.norm(tr[kpk]["root_after"][7:10])) - float(speeds[kpk, e])) < 1e-6, \
            "pass 2 must reproduce pass 1 bit for bit"
        per_step = []
        for k in range(max(0, kpk - 6), min(steps, kpk + 3)):
            t = tr[k]
            ck = contact_kinds(t["cache_after"])
            q = np.linalg.norm(t["dof"][:, 0].reshape(23, 3), axis=-1)
            per_step.append({"step": k, "root_speed": float(np.linalg.norm(t["root_after"][7:10])),
                             "com_speed": float(com_speed(model, t["rb_after"][None])[0]),
                             "root_height": float(t["root_after"][2]),
                             "lowest_body_z": float(t["rb_after"][:, 2].min()),
                             "contacts": ck, "dropped": t["dropped"], "slots": t["slots"],
                             "max_joint_angle": float(q.max()),
                             "max_joint": BODY_NAMES[1 + int(q.argmax())]})
        k0, k1 = max(0, kpk - 6), min(steps, kpk + 3)
        out_dir = os.environ.get("HE_RECORD_DIR")
        if out_dir:  # the traced env's states, targets and caches, for CPU replays of the oracle
            np.savez_compressed(os.path.join(out_dir, f"trace_runaway_{amp}.npz"), env=e, peak_step=kpk, k0=k0,
                                **{f"{f}": np.stack([tr[k][f] for k in range(k0, k1)])
                                   for f in ("root", "dof", "cache", "targets", "root_after", "rb_after")})
        res[str(amp)] = {"env": e, "peak_step": kpk, "peak_root_speed": float(speeds[kpk, e]),
                         "envs_over_10mps": int((vmax > 10).sum()), "envs_over_15mps": int((vmax > 15).sum()),
                         "engine": per_step,
                         "oracle_same_dt": replay(hm, model, tr, k0, k1, 2),
                         "oracle_dt_over_4": replay(hm, model, tr, k0, k1, 8)}
        print(amp, e, kpk, float(speeds[kpk, e]), file=sys.stderr, flush=True)
    res["definition"] = ("tools/action_regimes.py protocol; the fastest root's env traced (engine: per policy step "
                         "after the step; contacts = the normal / limit rows of the last solve by kind); oracle "
                         "replays from 6 steps before the peak with the engine's state, cache and targets, at the "
                         "engine's physics step (1/120 s) and at dt/4 (1/480 s, cold cache)")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
