#!/bin/bash
# Static-engine tests, then same-box A/B of nontemporal fp32 wgrad stores (gemm_q) on the headline bench.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/wgradnt; mkdir -p $d; rm -f $d/bench.jsonl
timeout -k 10 400 python -u -m pytest tests/test_static_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -1 $d/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for e in LDNN_WGRAD_NT=0 LDNN_WGRAD_NT=1; do
    r=$(env $e timeout -k 10 200 python -u bench.py 2>&1 | tail -1) || exit 1
    echo "{\"rep\": $rep, \"env\": \"$e\", \"bench_ms\": $(echo $r | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a $d/bench.jsonl
  done
done
