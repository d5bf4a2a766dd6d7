#!/bin/bash
# Matrix-core and issue utilisation of the bench kernels: one rocprofv3 PMC pass (8 SQ counters +
# GRBM_GUI_ACTIVE, kernel trace only), summarised by tools/pmc_mfma.py into gpurun_out/pmc_mfma.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
CONFIG=${CONFIG:-standstill}
rm -rf gpurun_out/mfma_$TAG
[ -f profiles/pmc_mfma.json ] && [ ! -f gpurun_out/pmc_mfma.json ] && cp profiles/pmc_mfma.json gpurun_out/pmc_mfma.json
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/mfma_$TAG -o run -- python3 bench.py --config $CONFIG --steps 10 --warmup 3 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/mfma_$TAG.log 2>&1 &&
python3 tools/pmc_mfma.py gpurun_out/mfma_$TAG --config $CONFIG --out gpurun_out/pmc_mfma.json
rc=$?
tail -3 gpurun_out/mfma_$TAG.log
exit $rc
