"""One policy step from identical states, engine (fp32) vs oracle (fp64), against the oracle's own
spread under the sensitivity probes' modelled rounding (tests/cases.probe_physics_step): per
scenario the distribution of |gpu - oracle| / |probe - oracle| over the joint velocities and angles.
Calibrates the probes (diagnostic).

  python tests/diag/diag_onestep.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cases  # noqa: E402


def main():
    import torch
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model, pd_action_offset_scale
    from oracle import oracle as O
    model = load_default_model()
    hm = _abi.make_model(model)
    off, sc = pd_action_offset_scale(model)
    rng = np.random.default_rng(3)
    scen = {}
    r, d = cases.random_state(64, rng, height=(3.0, 4.0))
    scen["airborne"] = (r, d, rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32))
    r, d = cases.standing_state(model, 64, rng, xy_jitter=1.0)
    scen["standing_random"] = (r, d, (off + sc * rng.uniform(-0.3, 0.3, (64, 69))).astype(np.float32))
    r, d = cases.random_state(64, rng, height=(0.85, 1.0), ang=0.8, vel=0.5)
    scen["contact_rich"] = (r, d, rng.uniform(-0.5, 0.5, (64, 69)).astype(np.float32))
    sp = _abi.default_sim_params()
    res = {}
    for name, (root, dof, tg) in scen.items():
        n = root.shape[0]
        eng = Engine(hm, n, device=0, sim_params=sp)
        # settle 10 steps on the oracle first so the state is a trajectory state with a warm cache
        c = O.new_cache(n)
        for _ in range(10):
            O.physics_step(hm, sp, root, dof, tg, 2, cache=c)
        eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
        eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
        eng.dof_targets.copy_(torch.as_tensor(tg, device="cuda:0"))
        eng.contact_cache.copy_(torch.as_tensor(c, device="cuda:0"))
        r_o, d_o = root.copy(), dof.copy()
        O.physics_step(hm, sp, r_o, d_o, tg, 2, cache=c.copy())
        ps = []
        for k in range(4):
            r_s, d_s = root.copy(), dof.copy()
            cases.probe_physics_step(hm, sp, r_s, d_s, tg, 2, c.copy(), 7 + k)
            ps.append(d_s)
        eng.simulate(2)
        torch.cuda.synchronize()
        dg = eng.dof_state.view(n, 69, 2).cpu().numpy()
        out = {}
        for j, what in ((1, "vel"), (0, "pos")):
            eg = np.abs(dg[..., j] - d_o[..., j])
            ep = np.max([np.abs(p[..., j] - d_o[..., j]) for p in ps], axis=0)
            m = ep > 0
            ratio = eg[m] / ep[m]
            out[what] = {"gpu_err_median": float(np.median(eg)), "probe_spread_median": float(np.median(ep)),
                         "ratio_median": float(np.median(ratio)), "ratio_p90": float(np.percentile(ratio, 90)),
                         "ratio_p99": float(np.percentile(ratio, 99))}
        res[name] = out
        print(name, json.dumps(out), flush=True)
        del eng


if __name__ == "__main__":
    main()
