#!/bin/bash
# Dynamic instruction mix of the bench kernels: one rocprofv3 PMC pass (8 SQ counters, kernel trace
# only) per config, summarised by tools/imix.py into gpurun_out/imix_<config>_TAG.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
for CONFIG in ${CONFIGS:-standstill tracking dr}; do
  rm -rf gpurun_out/imix_${CONFIG}_$TAG
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d gpurun_out/imix_${CONFIG}_$TAG -o run -- python3 bench.py --config $CONFIG --steps 10 --warmup 3 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/imix_${CONFIG}_$TAG.log 2>&1 &&
  python3 tools/imix.py gpurun_out/imix_${CONFIG}_$TAG --config $CONFIG > gpurun_out/imix_${CONFIG}_$TAG.json || exit 1
done
