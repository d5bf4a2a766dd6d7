#!/bin/bash
# A/B timing of environment-variable settings of one build: each setting ("VAR=value ...", one
# argument each) benched on CONFIGS (default "standstill imitation dr"), AB_PASSES passes interleaved,
# each run under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
for pass in ${AB_PASSES:-1 2}; do
  for cfg in ${CONFIGS:-standstill imitation dr}; do
    for setting in "$@"; do
      v=$(env $setting timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['avg_launch_ms'])") || exit 1
      echo "$pass $cfg [$setting] $v"
    done
  done
done
