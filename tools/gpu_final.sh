set -o pipefail
bash tools/gpu_tests.sh > gpurun_out/final_tests.out 2>&1 && SKIP_TESTS=1 bash tools/gpu_round.sh r02final > gpurun_out/final_round.out 2>&1 && bash tools/gpu_mfma.sh r02final > gpurun_out/final_mfma.out 2>&1 && bash tools/gpu_pmc.sh r02final > gpurun_out/final_pmc.out 2>&1 && CONFIG=imitation bash tools/gpu_pmc.sh r02final_imit > gpurun_out/final_pmc_imit.out 2>&1
