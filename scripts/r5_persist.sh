set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5per; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_q_gpu.py -k persistent > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
MLP_AB_ENVS="X=0 LDNN_GEMM_PERSIST=0" bash scripts/gpu_run.sh r5per mlpab profmlp || exit 4
echo done
