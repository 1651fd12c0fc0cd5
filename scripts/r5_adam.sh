set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5adam; mkdir -p $O
for e in X=0 LDNN_CONV_PAIR=0 LDNN_CONV_BN_BWD=0 LDNN_NHWC_INPUT=0; do
  echo "{\"env\": \"$e\"}" >> $O/adam.jsonl
  env $e timeout -k 10 200 python -u scripts/bench_cnn.py --model enhanced_cnn --batch 64 --graph --no-stock --optimizer adam >> $O/adam.jsonl 2>> $O/adam.err || exit 3
done
(cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_adam -o prof_adam -- python -u scripts/bench_cnn.py --model enhanced_cnn --batch 64 --graph --no-stock --optimizer adam --steps 20 --warmup 5 > $O/prof_adam.txt 2>&1) || exit 4
echo done
