#!/bin/bash
# Every PMC pass of a round's final profile: SQ issue / MFMA and HBM traffic (FETCH_SIZE, WRITE_SIZE
# in separate passes) for configs[1] (standstill), configs[2] (imitation) and configs[4] (dr), each
# its own rocprofv3 run and limit. Usage: bash tools/gpu_pmc_all.sh TAG
set -o pipefail
TAG=${1:-run}
bash tools/gpu_mfma.sh $TAG > gpurun_out/pmc_all_mfma_$TAG.out 2>&1 &&
CONFIG=imitation bash tools/gpu_mfma.sh ${TAG}_imit > gpurun_out/pmc_all_mfma_imit_$TAG.out 2>&1 &&
CONFIG=dr bash tools/gpu_mfma.sh ${TAG}_dr > gpurun_out/pmc_all_mfma_dr_$TAG.out 2>&1 &&
bash tools/gpu_pmc.sh $TAG > gpurun_out/pmc_all_traffic_$TAG.out 2>&1 &&
CONFIG=imitation bash tools/gpu_pmc.sh ${TAG}_imit > gpurun_out/pmc_all_traffic_imit_$TAG.out 2>&1 &&
CONFIG=dr bash tools/gpu_pmc.sh ${TAG}_dr > gpurun_out/pmc_all_traffic_dr_$TAG.out 2>&1
rc=$?
tail -n 2 gpurun_out/pmc_all_*_$TAG.out
exit $rc
