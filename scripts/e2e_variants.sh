#!/bin/bash
# The reference's six experiment variants (BAR / BR / BDR / DAR / DR / DDR) end
# to end through train.py on one MI355X: 2 ranks sharing the GPU over gloo (RCCL needs one
# GPU per rank), EnhancedCNNModel, synthetic CIFAR-10-shaped data, hipGraph-replayed steps.
# Summary -> gpurun_out/e2e/summary.txt
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/e2e
: > gpurun_out/e2e/summary.txt
port=29611
for spec in "BAR allreduce balanced" "BR ring balanced" "BDR double_ring balanced" \
            "DAR allreduce skewed" "DR ring skewed" "DDR double_ring skewed"; do
  set -- $spec
  name=$1; topo=$2; part=$3
  extra=""; [ "$part" = skewed ] && extra="--fixed_ratio 0.5"
  t0=$(date +%s.%N)
  timeout -k 10 240 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    train.py --backend gloo --model enhanced_cnn --dataset cifar10 --n_train 4096 --n_test 512 \
    --epochs_global 2 --epochs_local 2 --batch_size 64 --topology $topo --partition $part $extra --graphs \
    --plots "" --out_dir gpurun_out/e2e/$name > gpurun_out/e2e/$name.log 2>&1
  rc=$?
  t1=$(date +%s.%N)
  echo "$name topology=$topo partition=$part rc=$rc wall_s=$(python3 -c "print(round($t1-$t0,1))")" >> gpurun_out/e2e/summary.txt
  grep -E "^\[global epoch|Test Loss|macro:" gpurun_out/e2e/$name.log >> gpurun_out/e2e/summary.txt
  [ $rc -eq 0 ] || exit $rc
  port=$((port + 1))
done
