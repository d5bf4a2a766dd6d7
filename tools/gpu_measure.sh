set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 &&
bash tools/gpu_mfma.sh s1 &&
CONFIG=imitation bash tools/gpu_mfma.sh i1 &&
bash tools/gpu_pmc.sh s1 &&
CONFIG=imitation bash tools/gpu_pmc.sh i1
rc=$?
tail -1 gpurun_out/bench_full.log
exit $rc
