#!/bin/bash
# patch (C = 8 stem) conv with 3 k-steps of B fragments in flight: conv tests, step A/B (LDNN_CONV_PATCH_PF 1 / 3), kernel trace
set -o pipefail
O=gpurun_out/r3s2patchpf
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 resnet18:256 enhanced_cnn:64" "LDNN_CONV_PATCH_PF=1" "LDNN_CONV_PATCH_PF=3" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for pf in 1 3; do
p=$O/resnet18_b64_pf$pf; mkdir -p $p
LDNN_CONV_PATCH_PF=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model resnet18 --batch 64 --steps 20 --warmup 3 --no-stock --graph > $p/bench.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $p 23 > $p/summary.txt
echo "== pf $pf"; grep "patch" $p/summary.txt
done
