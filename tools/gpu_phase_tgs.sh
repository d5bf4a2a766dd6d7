#!/bin/bash
# Phase profiles of the TGS kernel (the default) on configs[1], [2] and [4], and of the PGS option on
# configs[1]. Usage: bash tools/gpu_phase_tgs.sh TAG. Each GPU step has its own limit; stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-a}
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_standstill_$TAG.json 2> gpurun_out/phases_$TAG.err &&
timeout -k 10 300 python tools/phase_profile.py --config imitation > gpurun_out/phases_imitation_$TAG.json 2>> gpurun_out/phases_$TAG.err &&
timeout -k 10 300 python tools/phase_profile.py --config dr > gpurun_out/phases_dr_$TAG.json 2>> gpurun_out/phases_$TAG.err &&
timeout -k 10 300 python tools/phase_profile.py --scheme pgs > gpurun_out/phases_pgs_$TAG.json 2>> gpurun_out/phases_$TAG.err
rc=$?
python3 - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
names = ["standstill", "imitation", "dr", "pgs"]
ds = {}
for n in names:
    try:
        ds[n] = json.load(open(f"gpurun_out/phases_{n}_{tag}.json"))
    except Exception:
        pass
print("cycles/env-step", {n: d["cycles_per_env_step"] for n, d in ds.items()}, "contacts", {n: round(d["mean_contacts"], 2) for n, d in ds.items()})
for k in next(iter(ds.values()))["phases"]:
    row = [ds[n]["phases"][k]["cycles"] for n in ds]
    if any(row):
        print(f"{k:30s}", " ".join(f"{v:8d}" for v in row))
for n, d in ds.items():
    e = d.get("per_env_cycles", {})
    print(n, {k: v for k, v in e.items() if k != "slowest_2pct_phases"})
    print("  slowest 2 %:", e.get("slowest_2pct_phases"))
PY
exit $rc
