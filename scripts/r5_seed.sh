set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5seed; mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_layers_gpu.py tests/test_graphed_dp_gpu.py tests/test_gap_head_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_run.sh r5seed cnn:enhanced_cnn@64 cnn:enhanced_cnn@64 cnn:resnet18@64 prof:enhanced_cnn@64 || exit 4
echo done
