#!/bin/bash
# SQ instruction-mix / stall counters for the physics kernel (one PMC pass, kernel trace only).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
rm -rf gpurun_out/sq_$TAG
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/sq_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sq_$TAG.log 2>&1
rc=$?
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/sq_$TAG/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = "physics" if "physics_kernel" in row["Kernel_Name"] else ("imitation" if "imitation_kernel" in row["Kernel_Name"] else None)
        if k: acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: sum(v) / len(v) for c, v in sorted(d.items())})
PY
tail -3 gpurun_out/sq_$TAG.log
exit $rc
