#!/bin/bash
# One physics wave alone on its CU (81,920 B of extra LDS per wave: one workgroup per CU) against
# the shipped occupancy: the phase profile (stamp builds) and the launch time at 256 envs, then the
# shipped stamp build at 256 / 1024 / 2048 envs. Each step its own limit.
set -o pipefail
mkdir -p gpurun_out
V=humanoid_amd/_variants
HE_ENGINE_LIB=$PWD/$V/alone.so timeout -k 10 120 python tools/phase_profile.py --num-envs 256 > gpurun_out/phases_alone256.json &&
timeout -k 10 120 python tools/phase_profile.py --num-envs 256 > gpurun_out/phases_256.json &&
for lib in $V/alone_prod.so humanoid_amd/libhumanoid_engine.so; do
  HE_ENGINE_LIB=$PWD/$lib timeout -k 10 120 python bench.py --num-envs 256 --no-cpu-baseline --no-puffer-level --no-tracking --no-learner --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib', d['value'], d['roofline']['avg_launch_ms'])" || exit 1
done > gpurun_out/alone_launch.txt
rc=$?
cat gpurun_out/alone_launch.txt
exit $rc
