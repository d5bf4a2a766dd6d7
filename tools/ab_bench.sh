#!/bin/bash
# A/B timing of variant engine builds (tools/build_variant.py) on one GPU box: each library is
# benched twice, interleaved, each run under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
LIBS="humanoid_amd/libhumanoid_engine.so $*"
for pass in ${AB_PASSES:-1 2}; do
  for lib in $LIBS; do
    v=$(HE_ENGINE_LIB=$PWD/$lib timeout -k 10 120 python bench.py --config ${CONFIG:-standstill} --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());u=d.get('unfused_kernels',{});print(d['value'], d['roofline']['avg_launch_ms'], u.get('imitation_kernel',{}).get('avg_launch_ms'))") || exit 1
    echo "$pass $lib $v"
  done
done
