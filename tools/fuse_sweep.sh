#!/bin/bash
# One-launch (fused) against two-launch env step over env counts: each bench run under its own
# time limit, interleaved; the summary goes to gpurun_out/fuse_sweep.txt.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/fuse_sweep.txt
: > $out
for n in 16 256 1024 2048 3072 4096; do
  for f in "" "--fused"; do
    v=$(timeout -k 10 120 python bench.py --num-envs $n $f --steps 200 --warmup 20 --no-cpu-baseline --no-puffer-level --no-tracking 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])") || exit 1
    echo "$n ${f:-two-launch} $v" | tee -a $out
  done
done
