set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5pair2; mkdir -p $O
timeout -k 10 300 python -u scripts/pair_probe.py --model enhanced_cnn --iters 40 > $O/pair.jsonl 2> $O/pair.err || exit 4
timeout -k 10 300 python -u scripts/pair_probe.py --model resnet18 --iters 40 >> $O/pair.jsonl 2>> $O/pair.err || exit 5
echo done
