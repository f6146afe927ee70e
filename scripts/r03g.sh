#!/bin/bash
# Window-build tests (fused sort-dedupe), small-batch / collector tests, the
# compact-tile tests, then config-3 A/B against comdb2_amd/lib/abx/*.so and a
# default bench without the CPU leg.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03g}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_incremental.py tests/test_gpu_small.py tests/test_collector.py tests/test_gpu_ctiles.py tests/test_gpu_config3.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 500 python3 bench.py --no-cpu --no-pmc > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_bench.log
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1]); print(d['ingest'])"
NO_TESTS=1 TAG=${T}_c3 bash scripts/r03f.sh || exit $?
echo r03g done
