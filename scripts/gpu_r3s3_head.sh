#!/bin/bash
# classifier-head micro bench (GAP + FC GEMM variants) + pool / layer tests + ResNet-18 b64 step A/B (FC split-K)
set -o pipefail
O=gpurun_out/r3s3h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py tests/test_layers_gpu.py -m gpu > $O/test_pool.txt 2>&1 || { tail -40 $O/test_pool.txt; exit 1; }
tail -2 $O/test_pool.txt
timeout -k 10 120 python -u scripts/bench_fc_head.py --batch 64 > $O/fc64.jsonl 2>&1 || { tail -20 $O/fc64.jsonl; exit 1; }
timeout -k 10 120 python -u scripts/bench_fc_head.py --batch 256 > $O/fc256.jsonl 2>&1 || { tail -20 $O/fc256.jsonl; exit 1; }
cat $O/fc64.jsonl $O/fc256.jsonl
for i in 1 2; do
for sk in 1 0; do
echo "LDNN_FC_SPLITK=$sk" >> $O/rn64.txt
LDNN_FC_SPLITK=$sk timeout -k 10 200 python -u scripts/bench_cnn.py --model resnet18 --batch 64 --graph --no-stock --steps 50 --warmup 10 >> $O/rn64.txt 2>&1 || { tail -20 $O/rn64.txt; exit 1; }
done
done
cat $O/rn64.txt | cut -c1-300
