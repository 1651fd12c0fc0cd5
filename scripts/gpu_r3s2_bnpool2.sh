#!/bin/bash
# fused BN + pool with XCD-placed rows: tests, reduce-grid knob A/B (LDNN_BNPOOL_BLOCKS 2048 / 8192), kernel traces
set -o pipefail
O=gpurun_out/r3s2bnpool2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 resnet18:256" "LDNN_BNPOOL_BLOCKS=2048" "LDNN_BNPOOL_BLOCKS=8192" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for blk in 2048 8192; do
p=$O/resnet18_b64_$blk; mkdir -p $p
LDNN_BNPOOL_BLOCKS=$blk timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model resnet18 --batch 64 --steps 20 --warmup 3 --no-stock --graph > $p/bench.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $p 23 > $p/summary.txt
echo "== blocks $blk"; grep "maxpool" $p/summary.txt
done
