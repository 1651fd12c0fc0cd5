set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5comb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_run.sh r5comb phase:enhanced_cnn || exit 5
AB_ENVS="X=0 LDNN_CONV_COMBINE_LAST=0" bash scripts/gpu_run.sh r5comb ab:enhanced_cnn:64,resnet18:64 || exit 4
echo done
