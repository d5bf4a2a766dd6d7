#!/bin/bash
# Round 4: the whole GPU suite with -s (the parity counts and runaway sweep printed into the log,
# records under gpurun_out/), smoke(), and one default bench line. Each GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
TAG=${1:-r04a}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
grep -E "FAILED|U\(\+-" gpurun_out/gpu_tests_$TAG.log | tail -8
tail -2 gpurun_out/smoke_$TAG.log
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-400
exit $rc
