#!/bin/bash
# Round-3 GPU session: the GPU suite, a quick bench and the rocprofv3 kernel stats of the same bench
# command. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
BENCH="bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level --no-tracking"
{ [ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s ${TESTS:-} > gpurun_out/gpu_tests_$TAG.log 2>&1; }
rc=$?
grep -E "PASSED|FAILED|ERROR|mismatch|widened|envs over|median internal" gpurun_out/gpu_tests_$TAG.log | tail -80
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python $BENCH > gpurun_out/bench_$TAG.log 2>&1 &&
{ [ "${PHASES:-0}" = 0 ] || timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_$TAG.json 2> gpurun_out/phases_$TAG.err; } &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 $BENCH > gpurun_out/bench_prof_$TAG.log 2>&1
rc2=$?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-1500
[ "${PHASES:-0}" = 0 ] || python3 -c "import json;d=json.load(open('gpurun_out/phases_$TAG.json'));print(d['cycles_per_env_step'], d['mean_contacts']);[print(f'{k:28s} {v[\"cycles\"]:8d} {v[\"share\"]:.3f}') for k,v in d['phases'].items()]"
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; 2>/dev/null | cut -c1-200
exit $(( rc > rc2 ? rc : rc2 ))
