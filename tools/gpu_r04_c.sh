#!/bin/bash
# Round 4: first-launch modes (tools/first_launch2.py), one fresh process each.
set -o pipefail
mkdir -p gpurun_out
for m in plain one_env warm_mem physics plain; do
  timeout -k 10 120 python tools/first_launch2.py $m >> gpurun_out/first_launch2.jsonl 2>> gpurun_out/first_launch2.err || exit $?
done
cat gpurun_out/first_launch2.jsonl
timeout -k 10 60 ./tools/ubench/pgs_row > gpurun_out/ubench_pgs_row2.json 2>&1 && cat gpurun_out/ubench_pgs_row2.json
