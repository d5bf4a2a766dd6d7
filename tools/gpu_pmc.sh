#!/bin/bash
# HBM traffic: two separate rocprofv3 PMC passes over the bench (FETCH_SIZE, WRITE_SIZE), then the
# summary into gpurun_out/pmc_traffic.json. CONFIG=standstill|imitation|dr selects the workload.
# Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
CONFIG=${CONFIG:-standstill}
B="bench.py --config $CONFIG --steps 10 --warmup 3 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner"
rm -rf gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG
[ -f profiles/pmc_traffic.json ] && [ ! -f gpurun_out/pmc_traffic.json ] && cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 $B > gpurun_out/pmc_fetch_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 $B > gpurun_out/pmc_write_$TAG.log 2>&1 &&
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG --config $CONFIG --out gpurun_out/pmc_traffic.json
rc=$?
tail -3 gpurun_out/pmc_fetch_$TAG.log
exit $rc
