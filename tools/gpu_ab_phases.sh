#!/bin/bash
# A/B of the main library against variant builds (tools/ab_bench.sh), then the phase profile of the
# main build. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 600 bash tools/ab_bench.sh "$@" > gpurun_out/ab_$TAG.txt 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_$TAG.json 2> gpurun_out/phases_$TAG.err
rc=$?
cat gpurun_out/ab_$TAG.txt
python3 -c "import json;d=json.load(open('gpurun_out/phases_$TAG.json'));print(d['cycles_per_env_step'], d['mean_contacts']);[print(f'{k:28s} {v[\"cycles\"]:8d} {v[\"share\"]:.3f}') for k,v in d['phases'].items()]"
exit $rc
