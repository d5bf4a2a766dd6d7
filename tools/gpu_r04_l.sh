#!/bin/bash
# A/B: he_env_step as one fused launch (physics + imitation epilogue) against the two launches, at
# 4096 envs on configs[1] and configs[2], 3 interleaved passes; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
run() {  # config, extra flag
  timeout -k 10 120 python bench.py --config $1 $2 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for pass in 1 2 3; do
  for cfg in standstill imitation; do
    a=$(run $cfg "") || exit 1
    b=$(run $cfg --fused) || exit 1
    echo "$pass $cfg two-launch $a fused $b"
  done
done > gpurun_out/ab_fused_r04.txt
rc=$?
cat gpurun_out/ab_fused_r04.txt
exit $rc
