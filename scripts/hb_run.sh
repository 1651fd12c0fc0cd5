set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5hb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "big_tile or halo_conv_matches or fwd_dgrad_wgrad" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in 64 256; do for e in LDNN_CONV_HB=0 LDNN_CONV_HB=1 LDNN_CONV_HB=0 LDNN_CONV_HB=1; do
  echo "{\"env\": \"$e\", \"batch\": $b}" >> $O/micro.jsonl
  env $e timeout -k 10 200 python -u scripts/conv_micro.py --model resnet18 --batch $b --no-stock >> $O/micro.jsonl 2>> $O/micro.err || exit 3
done; done
for e in LDNN_CONV_HB=0 LDNN_CONV_HB=1 LDNN_CONV_HB=0 LDNN_CONV_HB=1; do
  echo "{\"env\": \"$e\", \"model\": \"ecnn\"}" >> $O/micro.jsonl
  env $e timeout -k 10 200 python -u scripts/conv_micro.py --model enhanced_cnn --batch 64 --no-stock >> $O/micro.jsonl 2>> $O/micro.err || exit 3
done
echo done
