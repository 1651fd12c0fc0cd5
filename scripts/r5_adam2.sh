set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5adam2; mkdir -p $O
timeout -k 10 300 python -u scripts/bench_cfg.py enhanced_cnn:64:30:adam enhanced_cnn:64:30:sgd enhanced_cnn:64:30:adam > $O/cfg1.jsonl 2> $O/cfg1.err || exit 3
timeout -k 10 300 python -u scripts/bench_cfg.py resnet18:256:8:sgd enhanced_cnn:64:30:adam > $O/cfg2.jsonl 2> $O/cfg2.err || exit 4
echo done
