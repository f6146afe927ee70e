#!/bin/bash
# Compact tiles: GPU tests, then config-3 A/B of the in-tree library against
# comdb2_amd/lib/abx/*.so (no CPU leg, no PMC), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03f}
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
  tail -1 gpurun_out/${T}_pytest.log
fi
for r in 1 2; do
  for lib in cur comdb2_amd/lib/abx/*.so; do
    name=$(basename "$lib" .so)
    if [ "$lib" = cur ]; then env=""; else env="HSC_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 300 python3 bench.py --config 3 --no-cpu --no-pmc --no-api > gpurun_out/${T}_${name}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_${name}_$r.log; exit 1; }
    python3 scripts/benchsum.py gpurun_out/${T}_${name}_$r.log
  done
done
echo r03f done
