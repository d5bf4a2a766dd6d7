"""Solver convergence of the fp64 oracle: the complementarity residual after
k Gauss-Seidel sweeps, cold (impulses from 0) vs warm-started (the previous solve's impulses by
contact key), on settled lying bodies and on the PD stand-still. Each case first runs to a settled
state with the engine's defaults (8 sweeps, warm start); the residual is then measured for one
step from that state and its cache. Writes JSON to stdout (profiles/r02/pgs_residual.json)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import cases
    from humanoid_amd import _abi
    from humanoid_amd.model import load_default_model
    from oracle import oracle as O
    model = load_default_model()
    hm = _abi.make_model(model)
    rng = np.random.default_rng(3)
    out = {}
    for name, (root, dof), settle in (("lying_settled", cases.lying_state(32, rng), 150),
                                      ("standing", cases.standing_state(model, 32, rng, xy_jitter=1.0), 60)):
        n = root.shape[0]
        tgt = np.zeros((n, 69), np.float32)
        sp = _abi.default_sim_params()
        cache = O.new_cache(n)
        for _ in range(settle):
            O.physics_step(hm, sp, root, dof, tgt, 2, cache=cache)
        res = {}
        for warm in (0, 1):
            for k in (1, 2, 4, 8, 16, 32):
                r, d, c = root.copy(), dof.copy(), cache.copy()
                o = O.physics_step(hm, _abi.default_sim_params(solver_iterations=k, warm_start=warm), r, d, tgt, 2,
                                   cache=c)
                res[f"{'warm' if warm else 'cold'}_{k}"] = {"median": float(np.median(o["residual"])),
                                                           "max": float(o["residual"].max())}
        out[name] = {"settle_steps": settle, "mean_slots": float(o["num_contacts"].mean()), "residual_m_per_s": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
