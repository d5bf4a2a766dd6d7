set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner_ranks.py tests/test_facade_env.py "tests/test_gpu_parity.py::test_state_init_matches_reference_golden" -m gpu -v --timeout 320 --timeout-method thread -s > gpurun_out/r04_learner.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-puffer-level > gpurun_out/r04_bench1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04_learner.log | tail -20
tail -1 gpurun_out/r04_bench1.log | cut -c1-3000
exit $rc
