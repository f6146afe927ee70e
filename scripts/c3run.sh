#!/bin/bash
# GPU tests of the config-3 / multi-stream paths, then config-3 bench runs
# (small with the CPU sort-join parity check, then the default size).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_config3.py tests/test_gpu_streams.py -v \
  --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 3 --c3-writes 1000000 --steps 10 --check \
  > gpurun_out/c3s.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 3 --steps 10 > gpurun_out/c3.log 2>&1
