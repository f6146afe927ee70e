#!/bin/bash
# Coalesce: GPU parity tests, then the coalesce bench (GPU vs one CPU core).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02co}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coalesce.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 scripts/bench_coalesce.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
cat gpurun_out/${TAG}_bench.log
