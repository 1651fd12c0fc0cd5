#!/bin/bash
# Same-box A/B of the slab + BN-statistics fusion on EnhancedCNN b64, then its step timeline.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "enhanced_cnn:64" "LDNN_SLAB_BN=0" "LDNN_SLAB_BN=1" || exit $?
bash scripts/ab_cnn.sh "enhanced_cnn:64" "LDNN_SLAB_BN=0" "LDNN_SLAB_BN=1" || exit $?
p=gpurun_out/prof_ecnn_slabbn; mkdir -p $p
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model enhanced_cnn --batch 64 --steps 20 --warmup 5 --no-stock --graph > $p/bench.log 2>&1 || exit $?
python3 scripts/step_timeline.py $p > $p/timeline.txt
tail -1 $p/timeline.txt
