#!/bin/bash
# GPU tests of the small-batch path and ingest, then the default bench
# (API leg and build time).  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03c}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_small.py tests/test_collector.py tests/test_gpu_ingest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 500 python3 bench.py --no-cpu --no-pmc > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_bench.log
echo r03c done
