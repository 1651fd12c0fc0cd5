set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5knobs4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
AB_ENVS="X=0 LDNN_CONV_SLAB_TILES=64 LDNN_CONV_SLAB_TILES=32 LDNN_CONV_SLAB_MIN_KT=6" bash scripts/gpu_run.sh r5knobs4 ab:enhanced_cnn:64,resnet18:64 || exit 4
echo done
