timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
echo "gpu tests rc=$rc" >> gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > gpurun_out/bench4.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --backend gloo --steps 5 --warmup 3 > gpurun_out/bench_gloo2.log 2>&1 || exit $?
for m in "enhanced_cnn 64" "resnet18 64"; do set -- $m
  timeout -k 10 200 python -u scripts/bench_cnn.py --model $1 --batch $2 --graph --no-stock >> gpurun_out/cnn_bnmask.jsonl 2>&1
  LDNN_BN_RELU_MASK=0 timeout -k 10 200 python -u scripts/bench_cnn.py --model $1 --batch $2 --graph --no-stock >> gpurun_out/cnn_bnmask.jsonl 2>&1
done
