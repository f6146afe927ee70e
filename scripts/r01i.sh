#!/bin/bash
# Full GPU check: smoke, pytest -m gpu, default bench, config-4 benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=smoke,pytest,bench bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py --config 4 > gpurun_out/c4.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 4 --history-txns 16700000 --steps 3 --warmup 1 > gpurun_out/c4big.log 2>&1 || exit $?
