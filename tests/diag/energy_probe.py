"""Energy-stability probe of physics schemes on the CPU oracle (the runaway regime).

Standing envs under random PD actions U(-amp, amp) of the PD scale, new every policy step, for
`steps` policy steps: per scheme the envs whose root ever exceeds 10 m/s, the worst root speed,
the median internal kinetic energy at the end and the largest link world angular velocity.
Airborne envs (no contact) under U(+-0.5): median internal kinetic energy after 3 s.

  python tests/diag/energy_probe.py [--n 256] [--steps 60]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cases  # noqa: E402
from humanoid_amd import _abi  # noqa: E402
from humanoid_amd.model import load_default_model, pd_action_offset_scale  # noqa: E402
from oracle import oracle as O  # noqa: E402


def internal_ke(hm, model, sp, root, dof):
    me = O.momentum_energy(hm, sp, root, dof)
    M = float(np.sum(model.mass))
    return me[:, 6] - 0.5 * (me[:, :3] ** 2).sum(1) / M


def run(hm, model, amp, n, steps, airborne=False, seed=8, **sim):
    off, sc = pd_action_offset_scale(model)
    rng = np.random.default_rng(seed)
    root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
    if airborne:
        root[:, 2] += 200.0
        sim.setdefault("self_collision", 0)
    sp = _abi.default_sim_params(**sim)
    cache = O.new_cache(n)
    vmax = np.zeros(n)
    cmax = np.zeros(n)
    M = float(np.sum(model.mass))
    wmax = 0.0
    for _ in range(steps):
        a = rng.uniform(-amp, amp, (n, 69)).astype(np.float32)
        out = O.physics_step(hm, sp, root, dof, (off + sc * a).astype(np.float32), 2, cache=cache)
        vmax = np.maximum(vmax, np.linalg.norm(root[:, 7:10], axis=1))
        cmax = np.maximum(cmax, np.linalg.norm(O.momentum_energy(hm, sp, root, dof)[:, :3], axis=1) / M)
        wmax = max(wmax, float(np.linalg.norm(out["rb_state"][..., 10:13], axis=-1).max()))
    ke = internal_ke(hm, model, sp, root, dof)
    return {"over10": int((vmax > 10).sum()), "vmax": round(float(vmax.max()), 2),
            "com_over5": int((cmax > 5).sum()), "com_vmax": round(float(cmax.max()), 2),
            "ke_med": round(float(np.median(ke)), 1), "ke_max": round(float(ke.max()), 1), "wmax": round(wmax, 1)}


# schemes as he_sim_params overrides (the engine default is "default")
SCHEMES = {
    "default": {},
    "explicit": dict(bias_midpoint=0),
    "r02": dict(bias_midpoint=0, substeps=1, solver_iterations=8),
    "r02_midpoint": dict(substeps=1, solver_iterations=8),
    "explicit_sub4": dict(bias_midpoint=0, substeps=4),
    "sub4": dict(substeps=4),
    "sweeps8": dict(solver_iterations=8),
    "no_world_clamp": dict(max_angular_velocity=1e9),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--schemes", default=",".join(SCHEMES))
    ap.add_argument("--amps", default="0.5,1.0")
    ap.add_argument("--airborne", action="store_true")
    args = ap.parse_args()
    model = load_default_model()
    hm = _abi.make_model(model)
    res = {}
    for name in args.schemes.split(","):
        name = name.strip()
        if name in SCHEMES:
            sim = SCHEMES[name]
        else:  # ad-hoc: "substeps=4;solver_iterations=8"
            sim = {}
            for kv in name.split(";"):
                k, v = kv.split("=")
                sim[k] = float(v) if "." in v or "e" in v else int(v)
        r = {}
        t0 = time.time()
        for amp in [float(x) for x in args.amps.split(",")]:
            r[f"U{amp}"] = run(hm, model, amp, args.n, args.steps, **sim)
        if args.airborne:
            r["air0.5"] = run(hm, model, 0.5, max(16, args.n // 4), 90, airborne=True, **sim)
        r["s"] = round(time.time() - t0, 1)
        res[name] = r
        print(name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
