set -o pipefail
mkdir -p gpurun_out
HE_ENGINE_LIB=$PWD/humanoid_amd/_variants/w2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -s -k "bias_predictor" > gpurun_out/w2_pred_tests.log 2>&1 || { tail -20 gpurun_out/w2_pred_tests.log; exit 1; }
tail -2 gpurun_out/w2_pred_tests.log
bash tools/gpu_ab_pred.sh humanoid_amd/_variants/w2.so humanoid_amd/_variants/w2c16.so > gpurun_out/ab_pred4.txt 2>&1; cat gpurun_out/ab_pred4.txt
