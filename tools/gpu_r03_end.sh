#!/bin/bash
# Round-end check of the shipped build: the GPU suite, smoke(), then the full measurement session
# (tools/gpu_r03_final.sh TAG). Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03end}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
bash tools/gpu_r03_final.sh $TAG
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
tail -3 gpurun_out/smoke_$TAG.log
exit $rc
