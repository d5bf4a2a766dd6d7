"""Which bodies the contact rows' support reaches, per env, on the bench workloads (the physics
kernel's Zh-product classes): the union of the rows' bodies' ancestor chains, read
from the warm-start cache's row keys after some steps, classed by the smallest DFS prefix of bodies
that holds it (legs = bodies 0..8, the class the iterations run over 32 dofs; +spine/head = 0..13;
all). Prints one JSON object (configs[1] stand-still, configs[2] fixed action and tracking actions,
configs[4]).

  python tools/support_histogram.py [STEPS]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def support_class(model, cache):
    from humanoid_amd import _abi
    n, keys, _ = _abi.cache_rows(cache)
    par = np.asarray(model.parents)
    anc = []
    for b in range(len(par)):
        m, x = 0, b
        while x >= 0:
            m |= 1 << x
            x = int(par[x])
        anc.append(m)
    out = {"no rows": 0, "legs (bodies 0-8)": 0, "legs+spine+head (0-13)": 0, "all": 0}
    for e in range(keys.shape[0]):
        lb = 0
        for k in keys[e, :n[e]]:
            b0, b1, _, _ = _abi.key_fields(k)
            lb |= anc[b0] | (anc[b1] if b1 >= 0 else 0)
        if n[e] == 0:
            out["no rows"] += 1
        elif lb & ~0x1FF == 0:
            out["legs (bodies 0-8)"] += 1
        elif lb & ~0x3FFF == 0:
            out["legs+spine+head (0-13)"] += 1
        else:
            out["all"] += 1
    return out


def main():
    import torch
    import bench
    from humanoid_amd.model import load_default_model
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    model = load_default_model()
    res = {"steps": steps}
    for name, cfg, track in (("configs[1] standstill", "standstill", False), ("configs[2] fixed action", "imitation", False),
                             ("configs[2] tracking", "imitation", True), ("configs[4] dr", "dr", False)):
        args = argparse.Namespace(config=cfg, num_envs=4096, clips=128, seed=0, max_contacts=40)
        ro = bench.Rollout(args, model, 0, 0)
        for _ in range(steps):
            if track:
                ro.tracking_actions()
            ro.step()
        torch.cuda.synchronize()
        res[name] = support_class(model, ro.eng.contact_cache.cpu().numpy())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
