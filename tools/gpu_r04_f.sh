#!/bin/bash
# Round 4: first step's host time and the configs[2] kernel trace with the shipped warm-up.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/first_launch2.py plain > gpurun_out/first_launch4.json 2>gpurun_out/first_launch4.err || exit $?
cat gpurun_out/first_launch4.json
Q="bench.py --config imitation --steps 20 --warmup 5 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/flw_final -o run -- python3 $Q > gpurun_out/flw_final.log 2>&1
