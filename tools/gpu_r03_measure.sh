#!/bin/bash
# Round-3 measurement session (no test suite): action regimes, contact histogram, the default bench
# (CPU baseline included), the phase profile and the rocprofv3 kernel stats of the bench command.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
BENCH="bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level --no-tracking"
timeout -k 10 300 python -u tools/action_regimes.py > gpurun_out/action_regimes_$TAG.json 2> gpurun_out/action_regimes_$TAG.err &&
timeout -k 10 200 python -u tools/contact_histogram.py > gpurun_out/contact_histogram_$TAG.json 2> gpurun_out/contact_histogram_$TAG.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_$TAG.json 2> gpurun_out/phases_$TAG.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 $BENCH > gpurun_out/bench_prof_$TAG.log 2>&1
rc=$?
cat gpurun_out/action_regimes_$TAG.err | tail -8
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-1200
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; 2>/dev/null | cut -c1-200
exit $rc
