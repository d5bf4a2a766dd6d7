#!/bin/bash
# One GPU session: parity tests, per-phase profile, bench, rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
# SKIP_TESTS=1: measure only (a candidate kernel whose parity is being investigated)
{ [ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; } &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_$TAG.json 2> gpurun_out/phases.err &&
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level > gpurun_out/bench_prof_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
python3 -c "import json;d=json.load(open('gpurun_out/phases_$TAG.json'));print(d['cycles_per_env_step'], d['mean_contacts']);[print(f'{k:22s} {v[\"cycles\"]:8d} {v[\"share\"]:.3f}') for k,v in d['phases'].items()]" 2>/dev/null
tail -2 gpurun_out/bench_$TAG.log
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; 2>/dev/null | cut -c1-200
exit $rc
