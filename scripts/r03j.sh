#!/bin/bash
# Narrow join walks: the narrow GPU tests, then config-2 A/B of the in-tree
# library against comdb2_amd/lib/abx/*.so on one and two streams, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03j}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_full_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
NO_TESTS=1 TAG=$T bash scripts/r03d.sh > /dev/null 2>&1 || exit 1
for f in gpurun_out/${T}_ab_*.log; do python3 scripts/benchsum.py $f; done
echo r03j done
