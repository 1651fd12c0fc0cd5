timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py tests/test_conv_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/l_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 256; do timeout -k 10 200 python -u scripts/bench_cnn.py --model enhanced_cnn --batch $b --graph --no-stock >> gpurun_out/cnn64.log 2>&1 || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/prof_ecnn64; rm -rf $d && mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/bench_cnn.py --model enhanced_cnn --batch 64 --steps 20 --warmup 5 --no-stock --graph > $d/bench.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $d 25 > $d/summary.txt
