#!/bin/bash
# Instruction-cache health of the bench kernels: one rocprofv3 PMC pass of 8 SQ-block counters
# (SQC instruction cache requests / hits / misses / duplicate misses, SIMD instruction fetches,
# wave cycles, issue stalls, busy cycles), kernel trace only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
N=${N:-4096}
rm -rf gpurun_out/icache_$TAG
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/icache_$TAG -o run -- python3 bench.py --num-envs $N --steps 10 --warmup 3 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/icache_$TAG.log 2>&1
rc=$?
python3 tools/trim_csv.py gpurun_out/icache_$TAG
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/icache_{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    gmax = collections.defaultdict(int)
    for r in rows:
        gmax[r["Kernel_Name"]] = max(gmax[r["Kernel_Name"]], int(r["Grid_Size"]))
    for r in rows:
        for k in ("physics_kernel", "imitation_kernel"):
            if k in r["Kernel_Name"] and int(r["Grid_Size"]) == gmax[r["Kernel_Name"]]:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
tail -2 gpurun_out/icache_$TAG.log
exit $rc
