# phase profile of the physics kernel with the bias predictor off and on (diagnostic twin library)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_profile.py > gpurun_out/phases_pred_off.json 2>gpurun_out/phases_pred_off.err && \
timeout -k 10 120 python tools/phase_profile.py --bias-predictor > gpurun_out/phases_pred_on.json 2>gpurun_out/phases_pred_on.err
