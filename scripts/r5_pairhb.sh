set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5pairhb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "paired or downsample" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
AB_ENVS="X=0 LDNN_CONV_PAIR=3" bash scripts/gpu_run.sh r5pairhb ab:resnet18:64,resnet18:256 || exit 4
echo done
