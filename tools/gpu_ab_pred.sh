# A/B of the bias predictor's cost: the product build (predictor off / on), the build with the
# predictor compiled out (humanoid_amd/_variants/nopred.so) and any extra variant libraries given
# as arguments (off / on), interleaved, each run time-limited; stops at the first failure
set -o pipefail
mkdir -p gpurun_out
V=("humanoid_amd/libhumanoid_engine.so" "humanoid_amd/libhumanoid_engine.so --bias-predictor" "humanoid_amd/_variants/nopred.so")
for x in "$@"; do V+=("$x" "$x --bias-predictor"); done
for pass in 1 2 3; do
  for v in "${V[@]}"; do
    set -- $v
    r=$(HE_ENGINE_LIB=$PWD/$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-puffer-level --no-tracking --steps 200 --warmup 20 $2 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['avg_launch_ms'])") || exit 1
    echo "$pass $v $r"
  done
done
