#!/bin/bash
# New-ingest check: the build sort tests and the one-rank RCCL test first,
# then the r03_ab.sh suite + A/B benches (HSC_BUILD_TRACE=1: per-stage build
# times on the bench's stderr).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_rccl.py tests/test_gpu_incremental.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${TAG}_ingest_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_ingest_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_ingest_tests.log | head -30; exit $rc; }
export HSC_BUILD_TRACE=1
exec_ab() { bash scripts/r03_ab.sh; }
exec_ab
