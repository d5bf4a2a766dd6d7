#!/bin/bash
# Partner-wave cost on the shipped kernel: the physics launch at 1024 envs (one wave per SIMD),
# 2048 (two per SIMD, one round) and 4096 (two rounds), configs[1], 2 interleaved passes.
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  for n in 1024 2048 4096; do
    v=$(timeout -k 10 120 python bench.py --num-envs $n --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['avg_launch_ms'], d['kernel_timing']['first_launch_ms']['max'])") || exit 1
    echo "$pass $n $v"
  done
done > gpurun_out/partner_cost_r04.txt
rc=$?
cat gpurun_out/partner_cost_r04.txt
exit $rc
