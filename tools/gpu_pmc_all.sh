#!/bin/bash
# Every PMC pass of the round's final profile: SQ issue / MFMA (standstill, imitation) and HBM
# traffic (FETCH_SIZE, WRITE_SIZE; standstill, imitation), each its own rocprofv3 run and limit.
set -o pipefail
TAG=${1:-r03}
bash tools/gpu_mfma.sh $TAG > gpurun_out/pmc_all_mfma_$TAG.out 2>&1 &&
CONFIG=imitation bash tools/gpu_mfma.sh ${TAG}_imit > gpurun_out/pmc_all_mfma_imit_$TAG.out 2>&1 &&
bash tools/gpu_pmc.sh $TAG > gpurun_out/pmc_all_traffic_$TAG.out 2>&1 &&
CONFIG=imitation bash tools/gpu_pmc.sh ${TAG}_imit > gpurun_out/pmc_all_traffic_imit_$TAG.out 2>&1
rc=$?
tail -n 2 gpurun_out/pmc_all_*_$TAG.out
exit $rc
