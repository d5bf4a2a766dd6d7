#!/bin/bash
# Round 4: the first-dispatch warm-up (he_create_envs) -- first full reset per warm mode (0 off, 1 one
# trivial kernel per TU, 2 every kernel once), then rocprofv3 kernel traces of the configs[2] bench under
# modes 2 and 1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/first_launch3.jsonl
for w in 0 1 2; do
  HE_WARM_MODE=$w timeout -k 10 120 python tools/first_launch2.py plain | sed "s/^{/{\"warm_mode\": $w, /" >> gpurun_out/first_launch3.jsonl || exit $?
done
cat gpurun_out/first_launch3.jsonl
Q="bench.py --config imitation --steps 20 --warmup 5 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner"
for w in 2 1; do
  HE_WARM_MODE=$w timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/flw_$w -o run -- python3 $Q > gpurun_out/flw_$w.log 2>&1 || exit $?
done
