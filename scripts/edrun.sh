#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -v --timeout 200 --timeout-method thread > gpurun_out/ted.log 2>&1 || exit $?
timeout -k 10 400 python scripts/bench_edges.py > gpurun_out/bed.log 2>&1
