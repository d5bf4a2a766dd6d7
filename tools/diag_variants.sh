set -o pipefail
CASE=${CASE:-traj30}
STEPS=${STEPS:-3}
for v in ${VARIANTS:-'{}' '{"bias_midpoint":0}' '{"substeps":1}' '{"solver_iterations":8}'}; do
  echo "== $v" >> gpurun_out/diag_variants.log
  timeout -k 10 120 python tests/diag/diag_traj.py $CASE "$v" $STEPS >> gpurun_out/diag_variants.log 2>&1 || exit 1
done
