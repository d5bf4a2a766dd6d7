#!/bin/bash
# Round-end measurement session on the shipped build: the GPU suite (-s, records into gpurun_out/),
# smoke(), the bench lines of configs[1] (CPU baseline, PHCPufferEnv level, tracking, other schemes,
# learner), configs[2] and configs[4], rocprofv3 kernel stats of the quick bench command, the phase
# profile, action regimes, contact histograms and every PMC pass (tools/gpu_pmc_all.sh).
# Usage: bash tools/gpu_end.sh TAG. Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_RECORD_DIR=gpurun_out
TAG=${1:-end}
Q="bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full_$TAG.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config imitation --no-cpu-baseline --no-puffer-level --no-learner > gpurun_out/bench_imit_$TAG.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config dr --no-cpu-baseline --no-puffer-level --no-tracking --no-learner > gpurun_out/bench_dr_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 $Q > gpurun_out/bench_prof_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_$TAG.json 2> gpurun_out/phases_$TAG.err &&
timeout -k 10 300 python -u tools/action_regimes.py > gpurun_out/action_regimes_$TAG.json 2> gpurun_out/action_regimes_$TAG.err &&
timeout -k 10 200 python -u tools/contact_histogram.py > gpurun_out/contact_histogram_$TAG.json 2> gpurun_out/contact_histogram_$TAG.err &&
timeout -k 10 300 python -u tools/support_histogram.py 30 > gpurun_out/support_classes_$TAG.json 2> gpurun_out/support_classes_$TAG.err &&
bash tools/gpu_pmc_all.sh $TAG
rc=$?
# keep the summaries and the engine kernels' rows of the per-dispatch CSVs: gpurun copies back <= 64 MiB
python tools/trim_csv.py gpurun_out
du -sh gpurun_out
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
tail -2 gpurun_out/smoke_$TAG.log
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-600
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; 2>/dev/null | head -3 | cut -c1-150
exit $rc
