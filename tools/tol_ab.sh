set -o pipefail
for pass in 1 2; do for t in 0 1e-5 3e-5 1e-4; do
  v=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-puffer-level --no-tracking --steps 200 --warmup 20 --solver-tolerance $t 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['avg_launch_ms'])") || exit 1
  echo "$pass standstill tol=$t $v"
  v=$(timeout -k 10 120 python bench.py --config imitation --no-cpu-baseline --no-puffer-level --no-tracking --steps 200 --warmup 20 --solver-tolerance $t 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['avg_launch_ms'])") || exit 1
  echo "$pass imitation tol=$t $v"
done; done
