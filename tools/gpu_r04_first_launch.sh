#!/bin/bash
# Round 4: per-dispatch kernel and memory-copy trace of the configs[2] bench (128 clips), three
# fresh processes, to locate the occasional slow first imitation launch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
Q="bench.py --config imitation --steps 20 --warmup 5 --no-cpu-baseline --no-puffer-level --no-tracking"
for i in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/fl_$i -o run -- python3 $Q > gpurun_out/fl_$i.log 2>&1 || exit $?
done
find gpurun_out/fl_1 -name "*.csv" | head
