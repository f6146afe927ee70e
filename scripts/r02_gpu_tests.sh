#!/bin/bash
# GPU test suite (one process), then the default bench (no kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit $rc; }
[ -n "$NO_BENCH" ] && exit 0
NO_KT=1 bash scripts/r02_bench.sh
