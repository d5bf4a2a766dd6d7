#!/bin/bash
# Round 4: the PGS row microbenchmark, then the first-launch kernel traces (tools/gpu_r04_first_launch.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/pgs_row > gpurun_out/ubench_pgs_row.json 2>&1 &&
cat gpurun_out/ubench_pgs_row.json &&
bash tools/gpu_r04_first_launch.sh
