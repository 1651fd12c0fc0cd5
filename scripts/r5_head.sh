set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5head; mkdir -p $O
for w in 768 256 512 1024 1536 2048; do
  LDNN_HEAD_BWD_WGS=$w timeout -k 10 120 python -u scripts/bench_head.py >> $O/head.jsonl 2>> $O/head.err || exit 3
done
