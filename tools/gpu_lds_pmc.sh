#!/bin/bash
# LDS health of the bench kernels: one rocprofv3 PMC pass (bank-conflict and unaligned-stall cycles,
# LDS-array cycles, LDS instructions and LDS issue stalls, against the waves' cycles), kernel trace only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
rm -rf gpurun_out/lds_$TAG
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/lds_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/lds_$TAG.log 2>&1
rc=$?
python3 tools/trim_csv.py gpurun_out/lds_$TAG
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/lds_{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k in ("physics_kernel", "imitation_kernel"):
            if k in r["Kernel_Name"] and int(r["Grid_Size"]) >= 131072:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
tail -2 gpurun_out/lds_$TAG.log
exit $rc
