timeout -k 10 400 python -u -m pytest tests/test_static_mlp_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/mlp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mlp_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py > gpurun_out/bench_lib.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-library-gemms > gpurun_out/bench_nolib.log 2>&1 || exit $?
bash scripts/prof_bench.sh
