cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/r2e; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gputests.log 2>&1
rc=$?; tail -3 $d/gputests.log; exit $rc
