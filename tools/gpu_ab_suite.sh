#!/bin/bash
# The GPU suite on the product build, then an A/B of the product against variant libraries on
# configs[1], [2], [4] (tools/ab_bench.sh). Each step its own time limit; stops at the first failure.
# Usage: bash tools/gpu_ab_suite.sh TAG VARIANT.so ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests_$TAG.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1
for c in standstill imitation dr; do
  CONFIG=$c bash tools/ab_bench.sh "$@" > gpurun_out/ab_${TAG}_$c.txt 2>&1 || exit 1
  echo "== $c"; cat gpurun_out/ab_${TAG}_$c.txt
done
