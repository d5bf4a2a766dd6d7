#!/bin/bash
# A/B of backend scheduler options (tools/build_variant.py -mllvm ...): the physics TU on configs[1]
# and the imitation TU on configs[2], 3 interleaved passes each; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
V=humanoid_amd/_variants
AB_PASSES="1 2 3" bash tools/ab_bench.sh $V/trk.so $V/relaxocc.so $V/memclause.so $V/memtrk.so > gpurun_out/ab_sched_phys.txt 2>&1 &&
AB_PASSES="1 2 3" CONFIG=imitation bash tools/ab_bench.sh $V/im_ilp.so $V/im_mem.so $V/im_trk.so > gpurun_out/ab_sched_imit.txt 2>&1
rc=$?
cat gpurun_out/ab_sched_phys.txt gpurun_out/ab_sched_imit.txt
exit $rc
