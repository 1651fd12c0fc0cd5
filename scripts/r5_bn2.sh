set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5bn2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py \
  tests/test_head_fused_gpu.py tests/test_gemm_q_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_run.sh r5bn2 profmlp || exit 3
AB_ENVS="X=0 LDNN_BN_SMALL_ROWS=0 LDNN_BN_SMALL_ROWS=8192" bash scripts/gpu_run.sh r5bn2 ab:enhanced_cnn:64,resnet18:64 || exit 4
echo done
