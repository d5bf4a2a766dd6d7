set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tests/diag/diag_physics.py > gpurun_out/diag.log 2>&1
cat gpurun_out/diag.log | tail -12
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases.json 2> gpurun_out/phases.err &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
cat gpurun_out/phases.json | head -60; tail -3 gpurun_out/phases.err; tail -3 gpurun_out/bench.log
exit $rc
