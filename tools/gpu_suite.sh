#!/bin/bash
# The whole GPU suite with -s (records into gpurun_out/), then smoke(). Each step its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
TAG=${1:-suite}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests_$TAG.log | grep -v PASSED | head -20
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
tail -3 gpurun_out/smoke_$TAG.log
exit $rc
