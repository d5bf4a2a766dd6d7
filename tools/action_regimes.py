"""Where random PD actions stop being physical: 4096 standing envs, 60 policy steps of
random actions U(-amp, amp) of the PD scale, per amplitude the envs whose root ever exceeds
10 m/s and the worst root speed and joint angle. Engine (GPU) run.

  python tools/action_regimes.py > profiles/r02/action_regimes.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

import cases  # noqa: E402


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
    for amp in (0.1, 0.25, 0.5, 0.75, 1.0):
        rng = np.random.default_rng(8)
        eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params())
        root, dof = cases.standing_state(model, n, rng, xy_jitter=1.0)
        eng.root_states.copy_(torch.as_tensor(root, device="cuda:0"))
        eng.dof_state.copy_(torch.as_tensor(dof.reshape(n * 69, 2), device="cuda:0"))
        vmax = torch.zeros(n, device="cuda:0")
        for _ in range(60):
            a = rng.uniform(-amp, amp, (n, 69)).astype(np.float32)
            eng.dof_targets.copy_(torch.as_tensor(off + sc * a, device="cuda:0"))
            eng.simulate(2)
            vmax = torch.maximum(vmax, eng.root_states[:, 7:10].norm(dim=1))
        q = eng.dof_state.view(n, 69, 2)[..., 0].reshape(n, 23, 3).norm(dim=-1)
        v = vmax.cpu().numpy()
        res[str(amp)] = {"envs_over_10mps": int((v > 10).sum()), "envs_over_50mps": int((v > 50).sum()),
                         "root_speed_max": float(v.max()), "root_speed_p99": float(np.percentile(v, 99)),
                         "joint_angle_max": float(q.max())}
        print(amp, res[str(amp)], file=sys.stderr)
        del eng
    res["definition"] = ("4096 standing envs (cases.standing_state), 60 policy steps (2 s) of actions U(-amp, amp) x the "
                         "PD scale, new each step; per env the largest root speed over the run")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
