#!/bin/bash
# Config-3 bench: compact codes (default) and plain wide.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config 3 --check > gpurun_out/c3c.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 3 --wide > gpurun_out/c3w.log 2>&1 || exit $?
