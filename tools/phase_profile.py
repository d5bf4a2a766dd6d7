"""Per-phase cycle breakdown of the physics kernel (diagnostic twin library
libhumanoid_engine_phases.so, he_set_debug_stamps).

Runs the bench workload (default configs[1], 4096 envs) for a few steps with stamps enabled and
prints mean shader cycles per env per policy step for each phase.
Usage: python tools/phase_profile.py [--config standstill|imitation|dr] [--steps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the product library leaves the stamps out; this loads the diagnostic twin (humanoid_amd/build.py)
os.environ.setdefault("HE_ENGINE_LIB", os.path.join(ROOT, "humanoid_amd", "libhumanoid_engine_phases.so"))

PHASES = ["kinematics", "inertia+rnea", "subtree sums", "bias/IS/drives", "crba", "ltdl factor", "free solve",
          "contact gen", "Z rows + L^-T", "delassus A", "pgs", "du solve + forces", "integrate", "final fk+write",
          "contact: limit slots", "self: pair tests+slots", "terrain: rank+prefix", "terrain: slots",
          "terrain: geometry (to P0/P1)", "self: segment tests", "rows: J^T + bias", "rows: L^-T sweep",
          "pgs: set-up", "(unused)", "fused imitation",
          "mid: um sweep", "mid: velocities + rnea", "mid: subtree + dc", "mid: L^-T",
          "tgs: bias rnea", "tgs: rhs L^-T", "tgs: next sweep set-up"]  # slots 25-28: the midpoint bias; slots 14-19 are carved out of "contact gen", 20-21 out of "Z rows", 22 out of "pgs" (its set-up before the sweeps); 29-31 the TGS iterations (TGS: "pgs" = the sweeps, "du solve" = the velocity updates, "integrate" = drive force + integration, per iteration)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="standstill")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--max-contacts", type=int, default=40)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--scheme", choices=["default", "pgs", "r02", "tgs_small"], default="default")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from humanoid_amd.model import load_default_model
    bargs = argparse.Namespace(config=args.config, num_envs=args.num_envs, clips=128, seed=0,
                               max_contacts=args.max_contacts, fused=args.fused, scheme=args.scheme)
    model = load_default_model()
    ro = bench.Rollout(bargs, model, 0, 0)
    for _ in range(args.warmup):
        ro.step()
    buf = torch.zeros(args.num_envs, 32, dtype=torch.int64, device=ro.eng.device)
    ro.eng.set_debug_stamps(buf)
    nc = []
    for _ in range(args.steps):
        ro.step()
        nc.append(ro.eng.num_contacts.float().mean().item())
    torch.cuda.synchronize()
    ro.eng.set_debug_stamps(None)
    cyc = buf.cpu().numpy().astype(np.float64) / args.steps
    mean = cyc.mean(0)
    total = mean[:len(PHASES)].sum()
    rows = {PHASES[i]: {"cycles": round(float(mean[i])), "share": round(float(mean[i] / total), 4)}
            for i in range(len(PHASES))}
    # the launch waits for its slowest waves: the per-env distribution, and the phases of the slowest 2 %
    tot = cyc[:, :len(PHASES)].sum(1)
    slow = tot >= np.percentile(tot, 98)
    ms = cyc[slow].mean(0)
    slow_rows = {PHASES[i]: round(float(ms[i])) for i in range(len(PHASES)) if ms[i] > 0}
    dist = {"p50": round(float(np.percentile(tot, 50))), "p90": round(float(np.percentile(tot, 90))),
            "p98": round(float(np.percentile(tot, 98))), "max": round(float(tot.max())),
            "mean": round(float(tot.mean())), "slowest_2pct_phases": slow_rows}
    print(json.dumps({"config": args.config, "num_envs": args.num_envs, "mean_contacts": float(np.mean(nc)),
                      "scheme": args.scheme,
                      "cycles_per_env_step": round(float(total)), "phases": rows,
                      "per_env_cycles": dist}, indent=1))


if __name__ == "__main__":
    main()
