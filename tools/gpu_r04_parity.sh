# round 4: configs[4] / configs[2] 30-step parity records and the runaway trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_size.py -m gpu -v --timeout 500 --timeout-method thread -s -k "30_steps" > gpurun_out/r04_parity.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|events|one-step|tracking parity" gpurun_out/r04_parity.log | tail -20
[ $rc -le 1 ] && timeout -k 10 400 python -u tests/diag/trace_runaway.py 0.5 0.75 1.0 > gpurun_out/trace_runaway.json 2> gpurun_out/trace_runaway.err
rc2=$?
tail -5 gpurun_out/trace_runaway.err
exit $(( rc > rc2 ? rc : rc2 ))
