set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5flat; mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py tests/test_layers_gpu.py tests/test_graphed_dp_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_run.sh r5flat cnn:lenet5@256 cnn:lenet5@256 prof:lenet5@256 || exit 4
echo done
