set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|mismatch|widened" gpurun_out/gpu_tests.log | tail -60
[ $rc -le 1 ] && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level > gpurun_out/bench_quick.log 2>&1; tail -1 gpurun_out/bench_quick.log | cut -c1-400
exit $rc
