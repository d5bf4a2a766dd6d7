set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
timeout -k 10 400 python -u tests/diag/trace_runaway.py 0.75 1.0 > gpurun_out/trace_runaway.json 2> gpurun_out/trace_runaway.err
rc=$?
tail -3 gpurun_out/trace_runaway.err
exit $rc
