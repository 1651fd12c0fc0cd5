#!/bin/bash
# Rehearsal of the driver's multi-rank bench path on one GPU: 2 ranks (oversubscribed), gloo
# (RCCL refuses two ranks on one GPU), sharded + all-reduce variants.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/dp2; mkdir -p $d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --batch 4096 > $d/sharded.log 2>&1 || exit $?
tail -1 $d/sharded.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --batch 4096 --no-shard > $d/allreduce.log 2>&1 || exit $?
tail -1 $d/allreduce.log
