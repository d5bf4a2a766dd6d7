set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -s -k "bias_predictor or airborne or standing or limit" > gpurun_out/pred_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|median|mismatch|widened" gpurun_out/pred_tests.log | tail -40
[ $rc -eq 0 ] && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level > gpurun_out/bench_pred.log 2>&1; tail -1 gpurun_out/bench_pred.log | cut -c1-300
exit $rc
