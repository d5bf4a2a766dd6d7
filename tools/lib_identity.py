"""Bit-identity of two engine builds (e.g. a scheduler-flag variant): the bench rollout for 20 steps
with each library in its own process, states compared. Usage: python tools/lib_identity.py LIB_A LIB_B [--lying | --fused]"""
import os
import subprocess
import sys

CODE = r"""
import argparse, sys, numpy as np, torch
sys.path.insert(0, '.')
import bench
from humanoid_amd.model import load_default_model
args = argparse.Namespace(config='imitation', num_envs=4096, clips=128, seed=0, max_contacts=40, fused=len(sys.argv) > 2)
ro = bench.Rollout(args, load_default_model(), 0, 0)
for _ in range(20):
    ro.tracking_actions(); ro.step()
torch.cuda.synchronize()
np.savez(sys.argv[1], root=ro.eng.root_states.cpu().numpy(), dof=ro.eng.dof_state.cpu().numpy(), obs=ro.obs.cpu().numpy())
"""


# --lying: 512 lying bodies lowered into the plane (25-40 contacts, most solves past 32 rows: the TGS
# wide class) under random targets, 10 policy steps
CODE_LYING = r"""
import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import cases
from humanoid_amd import _abi
from humanoid_amd.engine import Engine
from humanoid_amd.model import load_default_model
n = 512
hm = _abi.make_model(load_default_model())
rng = np.random.default_rng(5)
root, dof = cases.lying_state(n, rng)
root[:, 2] = 0.08 + rng.uniform(0, 0.04, n).astype(np.float32)
eng = Engine(hm, n, device=0, sim_params=_abi.default_sim_params())
cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
eng.root_states.copy_(cu(root))
eng.dof_state.copy_(cu(dof.reshape(n * 69, 2)))
caches = []
for _ in range(10):
    eng.dof_targets.copy_(cu(rng.uniform(-0.5, 0.5, (n, 69)).astype(np.float32)))
    eng.simulate(2)
    caches.append(eng.contact_cache.cpu().numpy().copy())
torch.cuda.synchronize()
np.savez(sys.argv[1], root=eng.root_states.cpu().numpy(), dof=eng.dof_state.cpu().numpy(),
         rb=eng.rb_state.cpu().numpy(), force=eng.dof_force.cpu().numpy(), cache=np.asarray(caches))
"""


def main():
    outs = []
    lying = "--lying" in sys.argv
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for k, lib in enumerate(libs[:2]):
        out = f"gpurun_out/ident_{k}.npz"
        env = dict(os.environ, HE_ENGINE_LIB=os.path.abspath(lib))
        extra = ["fused"] if "--fused" in sys.argv else []  # the rollout as the one-launch env step
        subprocess.run([sys.executable, "-c", CODE_LYING if lying else CODE, out] + extra, check=True, env=env, timeout=300)
        outs.append(out)
    import numpy as np
    a, b = np.load(outs[0]), np.load(outs[1])
    for key in a.files:
        same = np.array_equal(a[key], b[key])
        print(key, "identical" if same else f"differs (max {np.abs(a[key] - b[key]).max():.3g})")


if __name__ == "__main__":
    main()
