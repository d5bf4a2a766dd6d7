#!/bin/bash
# Round 4: s_setprio placements over the serial phases, interleaved A/B (configs[1] x3, configs[2] x2).
set -o pipefail
mkdir -p gpurun_out
V="humanoid_amd/_variants/p_m.so humanoid_amd/_variants/p_md.so humanoid_amd/_variants/p_mds.so humanoid_amd/_variants/p_mdsx.so"
AB_PASSES="1 2 3" bash tools/ab_bench.sh $V > gpurun_out/ab_prio2_standstill.txt 2>&1 || exit $?
cat gpurun_out/ab_prio2_standstill.txt
CONFIG=imitation AB_PASSES="1 2" bash tools/ab_bench.sh $V > gpurun_out/ab_prio2_imit.txt 2>&1 || exit $?
cat gpurun_out/ab_prio2_imit.txt
