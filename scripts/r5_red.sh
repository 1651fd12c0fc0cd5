set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5red2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
AB_ENVS="LDNN_CONV_BN_BWD=3 X=0" bash scripts/gpu_run.sh r5red2 ab:enhanced_cnn:64,resnet18:64,resnet18:256 prof:enhanced_cnn@64 || exit 4
echo done
