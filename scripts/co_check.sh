cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coalesce.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/co_tests.log 2>&1; rc=$?; tail -5 gpurun_out/co_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/bench_coalesce.py > gpurun_out/co_bench.log 2>&1; rc=$?; tail -30 gpurun_out/co_bench.log; exit $rc
