#!/bin/bash
# Round 4: desynchronised start of odd workgroups (HE_DESYNC x s_sleep 127 ~ 8k cycles each), interleaved A/B.
set -o pipefail
mkdir -p gpurun_out
V="humanoid_amd/_variants/ds1.so humanoid_amd/_variants/ds2.so humanoid_amd/_variants/ds4.so humanoid_amd/_variants/ds8.so"
AB_PASSES="1 2 3" bash tools/ab_bench.sh $V > gpurun_out/ab_desync.txt 2>&1 || exit $?
cat gpurun_out/ab_desync.txt
