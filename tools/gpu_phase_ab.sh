#!/bin/bash
# Phase profiles of stamp-build variants (tools/build_variant.py NAME -DHE_PHASE_STAMPS=1 ...),
# interleaved, 2 passes: per-wave cycles by phase, so a change inside one phase is resolved
# below the bench's box noise. Usage: bash tools/gpu_phase_ab.sh NAME... (humanoid_amd/_variants/NAME.so)
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for n in "$@"; do
    HE_ENGINE_LIB=$PWD/humanoid_amd/_variants/$n.so timeout -k 10 120 python tools/phase_profile.py > gpurun_out/phv_${n}_$pass.json || exit 1
  done
done
python3 - "$@" <<'PY'
import json, sys
names = sys.argv[1:]
keys = None
for n in names:
    d = [json.load(open(f"gpurun_out/phv_{n}_{p}.json")) for p in (1, 2)]
    tot = [x["cycles_per_env_step"] for x in d]
    ph = {k: round(sum(x["phases"][k]["cycles"] for x in d) / 2) for k in d[0]["phases"]}
    big = {k: v for k, v in ph.items() if v > 5000}
    print(n, tot, big)
PY
