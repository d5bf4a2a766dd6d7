#!/bin/bash
# Round 5: the TGS kernel's parity tests, its phase profile beside the PGS kernel's, and its bench
# leg. Each GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-a}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tgs.py > gpurun_out/r05_tgs_tests_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py --scheme tgs > gpurun_out/phases_tgs_$TAG.json 2> gpurun_out/phases_tgs_$TAG.err &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_pgs_$TAG.json 2> gpurun_out/phases_pgs_$TAG.err &&
timeout -k 10 300 python -u bench.py --scheme tgs --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 > gpurun_out/r05_bench_tgs_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r05_tgs_tests_$TAG.log | tail -2
for f in gpurun_out/phases_tgs_$TAG.json gpurun_out/phases_pgs_$TAG.json; do python3 -c "
import json;d=json.load(open('$f'));print('$f', d['cycles_per_env_step'], d['mean_contacts']);[print(f'{k:28s} {v[\"cycles\"]:8d} {v[\"share\"]:.3f}') for k,v in d['phases'].items() if v['cycles']>0]"; done
tail -1 gpurun_out/r05_bench_tgs_$TAG.log | cut -c1-300
exit $rc
