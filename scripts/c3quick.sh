#!/bin/bash
# Compact-code GPU tests, then the config-3 bench (compact) with parity check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_config3.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c3q_tests.log 2>&1 || { tail -30 gpurun_out/c3q_tests.log; exit 1; }
tail -3 gpurun_out/c3q_tests.log
timeout -k 10 400 python bench.py --config 3 --check > gpurun_out/c3c.log 2>&1 || exit $?
tail -c 600 gpurun_out/c3c.log
