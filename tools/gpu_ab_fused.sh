#!/bin/bash
# A/B of the bench step as one fused launch (he_env_step, --fused) against the two launches, per
# config, 2 interleaved passes; each run under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for cfg in standstill tracking dr; do
    for form in two fused; do
      f=""; [ $form = fused ] && f="--fused"
      v=$(timeout -k 10 150 python bench.py --config $cfg $f --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])") || exit 1
      echo "$pass $cfg $form $v"
    done
  done
done
