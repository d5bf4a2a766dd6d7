set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_run.py -m gpu -v --timeout 300 --timeout-method thread -s -k "cold_solve or saturated_actions_dr or overflow" > gpurun_out/gpu_tests_r03p2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|mismatch|widened" gpurun_out/gpu_tests_r03p2.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phases_r03p2.json 2> gpurun_out/phases_r03p2.err &&
timeout -k 10 200 python -u tools/contact_histogram.py > gpurun_out/contact_histogram_r03p2.json 2> gpurun_out/contact_histogram_r03p2.err &&
timeout -k 10 300 python -u tools/action_regimes.py > gpurun_out/action_regimes_r03p2.json 2> gpurun_out/action_regimes_r03p2.err
rc2=$?
python3 -c "import json;d=json.load(open('gpurun_out/phases_r03p2.json'));print(d['cycles_per_env_step'], d['mean_contacts']);[print(f'{k:28s} {v[\"cycles\"]:8d} {v[\"share\"]:.3f}') for k,v in d['phases'].items()]"
tail -8 gpurun_out/action_regimes_r03p2.err
exit $(( rc > rc2 ? rc : rc2 ))
