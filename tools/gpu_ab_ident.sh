#!/bin/bash
# GPU suite on the main library, then an interleaved A/B of variant builds against it
# (tools/ab_bench.sh) and a bit-identity check of the first variant (tools/lib_identity.py).
# Usage: bash tools/gpu_ab_ident.sh humanoid_amd/_variants/NAME.so [...]  (SKIP_TESTS=1 skips the suite)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | grep -c PASSED
  grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -8
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python tools/lib_identity.py humanoid_amd/libhumanoid_engine.so "$1" > gpurun_out/ident.log 2>&1 || exit 1
cat gpurun_out/ident.log
bash tools/ab_bench.sh "$@" 2>&1 | tee gpurun_out/ab.txt
