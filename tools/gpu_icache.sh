#!/bin/bash
# Instruction-fetch counters for the physics kernel (one PMC pass each, kernel trace only).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
rm -rf gpurun_out/ic_$TAG
timeout -k 10 60 rocprofv3 -L > gpurun_out/ic_avail.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_[A-Z_]*CYCLES[A-Z_]*" gpurun_out/ic_avail.txt | sort -u > gpurun_out/ic_names.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/ic_$TAG/a -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-puffer-level > gpurun_out/ic_$TAG.log 2>&1
rc=$?
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/ic_$TAG/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "physics_kernel" in row["Kernel_Name"]:
            acc["physics"][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: sum(v) / len(v) for c, v in sorted(d.items())})
PY
tail -3 gpurun_out/ic_$TAG.log
exit $rc
