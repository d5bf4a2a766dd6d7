#!/bin/bash
# Round 4: the measurement session (tools/gpu_r04_end.sh TAG), then the cold-solve tolerance probe.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r04_end.sh ${1:-r04b} || exit $?
timeout -k 10 300 python -u tests/diag/cold_tol.py > gpurun_out/cold_tol.log 2>&1
cat gpurun_out/cold_tol.log
