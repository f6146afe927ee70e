#!/bin/bash
# Collector / lone-call latency (scripts/latency.py, then its empty-kernel
# floor), the collector GPU tests, and a default bench without the CPU leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03e}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_collector.py tests/test_gpu_small.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python3 -u scripts/latency.py > gpurun_out/${T}_latency.log 2>&1 || { tail -20 gpurun_out/${T}_latency.log; exit 1; }
cat gpurun_out/${T}_latency.log
HSC_SMALL_EMPTY=1 LAT_COMMITS=100000 timeout -k 10 300 python3 -u scripts/latency.py > gpurun_out/${T}_latency_empty.log 2>&1 || { tail -20 gpurun_out/${T}_latency_empty.log; exit 1; }
grep lone gpurun_out/${T}_latency_empty.log
timeout -k 10 500 python3 bench.py --no-cpu --no-pmc > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_bench.log
echo r03e done
