#!/bin/bash
# The reference's 2 x 3 experiment matrix ({IID, class-skewed} x {all-reduce, ring,
# double ring}: BAR / BR / BDR / DAR / DR / DDR) end to end through train.py
# with the reference's full schedule: 5 workers, 20 global x 5 local epochs, batch 64,
# Adam 1e-3, StepLR(25), AutoAugment(CIFAR10) on the training shard, EnhancedCNNModel.
# Data: the non-saturating synthetic CIFAR-10-shaped set (cifar10-hard: 15 % label noise,
# overlapping low-contrast prototypes, shifts) -- no dataset download exists here.
# --aggregation_by weights (model averaging / gossip of the weights every global epoch):
# with the reference's default (gradients) the exchange is a no-op and the
# six variants would differ only by noise.
# 5 ranks share the one GPU over gloo (RCCL needs a GPU per rank).
# AGG=gradients (the reference's default: SURVEY Q1 no-op) | weights (default here); SYNC=step runs
# per-step data parallelism instead of the reference's once-per-global-epoch exchange.
#   bash scripts/experiment_matrix.sh     -> gpurun_out/matrix${TAG}/<variant>/
cd "${GRAFT_REPO_ROOT:-.}"
AGG=${AGG:-weights}
SYNC=${SYNC:-global_epoch}
M=gpurun_out/matrix${TAG}
mkdir -p $M
N=${N:-5}
port=29711
specs=("BAR allreduce balanced" "BR ring balanced" "BDR double_ring balanced"
       "DAR allreduce skewed" "DR ring skewed" "DDR double_ring skewed")
for spec in "${specs[@]}"; do
  set -- $spec
  name=$1; topo=$2; part=$3
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then continue; fi
  out=$M/$name
  rm -rf $out && mkdir -p $out
  t0=$(date +%s.%N)
  timeout -k 10 ${LIMIT:-420} python -m torch.distributed.run --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $port train.py --backend gloo --model enhanced_cnn --dataset cifar10-hard --n_train ${NTRAIN:-10000} \
    --n_test 2000 --epochs_global ${EG:-20} --epochs_local ${EL:-5} --batch_size 64 --lr 1e-3 --topology $topo \
    --partition $part --aggregation_by $AGG --sync_every $SYNC --augment autoaugment --graphs --quiet --time_limit 0 \
    --plots $out/Graphs --out_dir $out > $out/train.log 2>&1
  rc=$?
  t1=$(date +%s.%N)
  echo "$name topology=$topo partition=$part rc=$rc wall_s=$(python3 -c "print(round($t1-$t0,1))")" | tee -a $M/summary.txt
  [ $rc -eq 0 ] || exit $rc
  port=$((port + 1))
done
