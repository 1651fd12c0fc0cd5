set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5headp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_head_fused_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
MLP_AB_ENVS="X=0 LDNN_HEAD_BWD_WGS=768 LDNN_HEAD_BWD_WGS=256" bash scripts/gpu_run.sh r5headp mlpab profmlp || exit 4
echo done
