#!/bin/bash
# Optimizer tests, then same-box A/B of nontemporal optimizer streams (LDNN_OPT_NT) on EnhancedCNN (SGD, Adam) and the headline bench.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/optnt; mkdir -p $d; rm -f gpurun_out/ab_cnn.jsonl $d/bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "sgd or adam" -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -1 $d/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for e in LDNN_OPT_NT=0 LDNN_OPT_NT=1; do
    r=$(env $e timeout -k 10 200 python -u scripts/bench_cnn.py --model enhanced_cnn --batch 64 --graph --no-stock --optimizer adam 2>&1 | tail -1) || exit 1
    echo "{\"rep\": $rep, \"env\": \"$e\", \"adam\": 1, \"line\": $r}" | tee -a gpurun_out/ab_cnn.jsonl
    r=$(env $e timeout -k 10 200 python -u bench.py 2>&1 | tail -1) || exit 1
    echo "{\"rep\": $rep, \"env\": \"$e\", \"bench_ms\": $(echo $r | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a $d/bench.jsonl
  done
done
bash scripts/ab_cnn.sh "enhanced_cnn:64" "LDNN_OPT_NT=0" "LDNN_OPT_NT=1"
