"""Bit-identity of two engine builds (e.g. a scheduler-flag variant): the bench rollout for 20 steps
with each library in its own process, states compared. Usage: python tools/lib_identity.py LIB_A LIB_B"""
import os
import subprocess
import sys

CODE = r"""
import argparse, sys, numpy as np, torch
sys.path.insert(0, '.')
import bench
from humanoid_amd.model import load_default_model
args = argparse.Namespace(config='imitation', num_envs=4096, clips=128, seed=0, max_contacts=40)
ro = bench.Rollout(args, load_default_model(), 0, 0)
for _ in range(20):
    ro.tracking_actions(); ro.step()
torch.cuda.synchronize()
np.savez(sys.argv[1], root=ro.eng.root_states.cpu().numpy(), dof=ro.eng.dof_state.cpu().numpy(), obs=ro.obs.cpu().numpy())
"""


def main():
    outs = []
    for k, lib in enumerate(sys.argv[1:3]):
        out = f"gpurun_out/ident_{k}.npz"
        env = dict(os.environ, HE_ENGINE_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, "-c", CODE, out], check=True, env=env, timeout=300)
        outs.append(out)
    import numpy as np
    a, b = np.load(outs[0]), np.load(outs[1])
    for key in a.files:
        same = np.array_equal(a[key], b[key])
        print(key, "identical" if same else f"differs (max {np.abs(a[key] - b[key]).max():.3g})")


if __name__ == "__main__":
    main()
