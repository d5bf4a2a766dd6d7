"""Where random PD actions stop being physical: 4096 standing envs, 60 policy steps of
random actions U(-amp, amp) of the PD scale, per amplitude the envs whose root ever exceeds
10 / 15 / 50 m/s, the worst root and centre-of-mass speeds, the worst joint angle and the median
internal kinetic energy (about the centre of mass) at the end. Engine (GPU) run, under the default
physics scheme and, for comparison, round 2's step (one 1/60 s physics step per simulate, explicit
bias) under round 3's angular-velocity clamps.

  python tools/action_regimes.py > profiles/r03/action_regimes.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

import cases  # noqa: E402


def kinetic(model, rb):
    """Total and centre-of-mass kinetic energy of every env from the rigid-body rows [n, B, 13]
    (origin position, xyzw quaternion, origin velocity, angular velocity)."""
    import torch
    dev = rb.device
    m = torch.as_tensor(model.mass, dtype=torch.float32, device=dev)
    c = torch.as_tensor(model.com, dtype=torch.float32, device=dev)
    inertia = torch.as_tensor(model.inertia, dtype=torch.float32, device=dev)
    q = rb[..., 3:7]
    x, y, z, w = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                     2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                     2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1).view(*q.shape[:-1], 3, 3)
    om = rb[..., 10:13]
    vc = rb[..., 7:10] + torch.cross(om, (R @ c[..., None])[..., 0], dim=-1)  # velocity of the body COM
    wl = (R.transpose(-1, -2) @ om[..., None])[..., 0]
    rot = 0.5 * (wl * (inertia @ wl[..., None])[..., 0]).sum(-1)
    ke = (0.5 * m * (vc * vc).sum(-1) + rot).sum(-1)
    vcom = (m[:, None] * vc).sum(1) / m.sum()
    return ke, vcom, 0.5 * m.sum() * (vcom * vcom).sum(-1)


SCHEMES = {"default": {}, "r02": dict(substeps=1, bias_midpoint=0)}  # round 2's step with round 3's clamps


def main():
    import torch
    from humanoid_amd import _abi
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model, pd_action_offset_scale
    model = load_default_model()
    hm = _abi.make_model(model)
    off, sc = pd_action_offset_scale(model)
    n = 4096
    res = {}
    runs = [("default", a) for a in (0.1, 0.25, 0.5, 0.75, 1.0)] + [("r02", 0.5), ("r02", 1.0)]
    for scheme, amp in runs:
        rng = np.random.default_rng(8)
        eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params(**SCHEMES[scheme]))
        root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
        eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
        eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
        vmax = torch.zeros(n, device="cuda:0")
        cmax = torch.zeros(n, device="cuda:0")
        for _ in range(60):
            a = rng.uniform(-amp, amp, (n, 69)).astype(np.float32)
            eng.dof_targets.copy_(torch.as_tensor(off + sc * a, device="cuda:0"))
            eng.simulate(2)
            vmax = torch.maximum(vmax, eng.root_states[:, 7:10].norm(dim=1))
            cmax = torch.maximum(cmax, kinetic(model, eng.rb_state.view(n, -1, 13))[1].norm(dim=1))
        ke, _, kc = kinetic(model, eng.rb_state.view(n, -1, 13))
        q = eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3).norm(dim=-1)
        v = vmax.cpu().numpy()
        v[~np.isfinite(v)] = np.inf  # a blown-up env counts as over every bound
        c = cmax.cpu().numpy()
        c[~np.isfinite(c)] = np.inf
        key = str(amp) if scheme == "default" else f"{scheme}:{amp}"
        res[key] = {"envs_over_10mps": int((v > 10).sum()), "envs_over_15mps": int((v > 15).sum()),
                    "envs_over_50mps": int((v > 50).sum()),
                    "root_speed_max": float(v.max()), "root_speed_p99": float(np.percentile(v, 99)),
                    "com_speed_max": float(c.max()), "envs_com_over_5mps": int((c > 5).sum()),
                    "internal_ke_median_J": float((ke - kc).nan_to_num(nan=float("inf")).median()),
                    "joint_angle_max": float(q.max())}
        print(key, res[key], file=sys.stderr, flush=True)
        del eng
    res["definition"] = ("4096 standing envs (cases.standing_state), 60 policy steps (2 s) of actions U(-amp, amp) x the "
                         "PD scale, new each step; per env the largest root and centre-of-mass speeds over the run; internal kinetic "
                         "energy = total - centre-of-mass part, at the end; keys 'r02:amp' are round 2's scheme")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
