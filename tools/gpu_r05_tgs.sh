#!/bin/bash
# Round 5: the TGS kernel (solver_type 1) against the oracle, the PGS physics tests on the same build,
# then an interleaved A/B of the PGS kernel against the pre-TGS build (humanoid_amd/_variants/r04head.so)
# and the TGS scheme's bench leg. Each GPU step has its own limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_tgs.py > gpurun_out/r05_tgs_tests.log 2>&1 &&
timeout -k 10 600 $T tests/test_gpu_parity.py -k "physics or knee or tgs or overflow or fused" > gpurun_out/r05_pgs_tests.log 2>&1 &&
AB_PASSES="1 2" timeout -k 10 600 bash tools/ab_bench.sh humanoid_amd/_variants/r04head.so > gpurun_out/r05_ab_pgs.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --scheme tgs --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/r05_bench_tgs.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/r05_tgs_tests.log | tail -5
grep -E "passed|failed" gpurun_out/r05_pgs_tests.log | tail -2
cat gpurun_out/r05_ab_pgs.txt
tail -1 gpurun_out/r05_bench_tgs.log | cut -c1-400
exit $rc
