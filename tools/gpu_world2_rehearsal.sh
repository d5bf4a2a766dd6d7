#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: torchrun with 2 ranks sharing cuda:0
# (HE_BENCH_SHARED_DEVICE=1: gloo collectives, since RCCL needs one GPU per rank), learner leg
# included, so the barrier / max-over-ranks timing and the learner's collectives run at world 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HE_BENCH_SHARED_DEVICE=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_world2.log 2>&1
rc=$?
grep "^{" gpurun_out/bench_world2.log | cut -c1-1500
exit $rc
