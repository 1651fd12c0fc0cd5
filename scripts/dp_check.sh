cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/check_static_dp.py --backend gloo --graphs 1 --shard 1 > gpurun_out/dp_shard.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 scripts/check_static_dp.py --backend gloo --graphs 1 --shard 1 --hidden 520 > gpurun_out/dp_shard3.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 scripts/check_static_dp.py --backend gloo --graphs 1 --shard 0 > gpurun_out/dp_noshard.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1
