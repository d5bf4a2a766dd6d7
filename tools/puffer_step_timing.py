import sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch, argparse
import bench
from humanoid_amd.model import load_default_model
from humanoid_amd.env import EnvConfig, PHCPufferEnv
model = load_default_model()
args = argparse.Namespace(config="standstill", num_envs=4096, clips=128, seed=0, max_contacts=40, puffer_steps=200)
clips = bench.make_clips(args, model)
cfg = EnvConfig(num_envs=4096, motion_file={f"clip{i}": c for i, c in enumerate(clips)}, seed=0, max_contacts=40)
pe = PHCPufferEnv(cfg); pe.reset()
_, actions, _ = bench.build_workload(args, model, 0)
ad = torch.as_tensor(actions, device="cuda:0")
for name, a in (("numpy", actions), ("device", ad), ("numpy", actions)):
    for _ in range(10): pe.step(a)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(200): pe.step(a)
    t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(name, "host us/step %.1f" % ((t1 - t0) / 200 * 1e6), "wall us/step %.1f" % ((t2 - t0) / 200 * 1e6), "rate %.0f" % (4096 * 200 / (t2 - t0)))

if os.environ.get("PROFILE"):
    import cProfile, pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200): pe.step(ad)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
