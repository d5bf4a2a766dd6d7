#!/bin/bash
# Round 4: s_setprio 3 over the midpoint's sweeps (priomid) and also the du sweep (priodu): interleaved A/B.
set -o pipefail
mkdir -p gpurun_out
AB_PASSES="1 2 3" bash tools/ab_bench.sh humanoid_amd/_variants/priomid.so humanoid_amd/_variants/priodu.so > gpurun_out/ab_prio_mid.txt 2>&1 || exit $?
cat gpurun_out/ab_prio_mid.txt
