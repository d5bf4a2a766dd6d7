#!/bin/bash
# Round 4: warm-up check (tools/gpu_r04_d.sh), then the deferred-writelane PGS variant: bit-identity
# against the shipped build and interleaved A/B on configs[1] and configs[2].
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r04_d.sh || exit $?
timeout -k 10 400 python tools/lib_identity.py humanoid_amd/libhumanoid_engine.so humanoid_amd/_variants/defer.so > gpurun_out/ident_defer.log 2>&1 || exit $?
cat gpurun_out/ident_defer.log
AB_PASSES="1 2 3" bash tools/ab_bench.sh humanoid_amd/_variants/defer.so > gpurun_out/ab_defer_standstill.txt 2>&1 || exit $?
cat gpurun_out/ab_defer_standstill.txt
CONFIG=imitation AB_PASSES="1 2" bash tools/ab_bench.sh humanoid_amd/_variants/defer.so > gpurun_out/ab_defer_imit.txt 2>&1 || exit $?
cat gpurun_out/ab_defer_imit.txt
