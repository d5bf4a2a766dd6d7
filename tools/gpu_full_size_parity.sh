#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_full_size.py tests/test_gpu_invariants.py -k "${1:-30_steps or free_fall}" > gpurun_out/r05_fs.log 2>&1
rc=$?
grep -E "PASSED|FAILED|parity:|^E " gpurun_out/r05_fs.log | cut -c1-1500 | head -30
exit $rc
