set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5adam3; mkdir -p $O
timeout -k 10 300 python -u scripts/bench_cfg.py lenet5:256:50:sgd resnet18:64:20:sgd resnet18:256:8:sgd enhanced_cnn:64:30:adam > $O/cfg.jsonl 2> $O/cfg.err || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 4
LDNN_CONV_PAIR=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_pair0.json 2> $O/bench_pair0.err || exit 5
echo done
