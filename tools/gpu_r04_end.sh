#!/bin/bash
# Round-4 measurement session on the shipped build: GPU suite (-s, records), smoke, then the full
# measurement set of tools/gpu_r03_final.sh (bench configs[1]/[2]/[4], rocprofv3 stats, phases, action
# regimes, contact histograms, every PMC pass). Each GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
TAG=${1:-r04end}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
bash tools/gpu_r03_final.sh $TAG
rc=$?
# keep the summaries and the engine kernels' rows of the per-dispatch CSVs: gpurun copies back <= 64 MiB
python tools/trim_csv.py gpurun_out
du -sh gpurun_out
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
tail -2 gpurun_out/smoke_$TAG.log
exit $rc
