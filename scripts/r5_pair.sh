set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5pair; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pair_probe.py --model enhanced_cnn > $O/pair.jsonl 2> $O/pair.err || exit 4
timeout -k 10 300 python -u scripts/pair_probe.py --model resnet18 >> $O/pair.jsonl 2>> $O/pair.err || exit 5
AB_ENVS="LDNN_CONV_BN_BWD=0 X=0" bash scripts/gpu_run.sh r5pair ab:enhanced_cnn:64,resnet18:64 || exit 6
echo done
