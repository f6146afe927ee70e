#!/bin/bash
# Compact-tile GPU tests, then config-3 A/B of the 512-thread join
# (HSC_CJOIN2=1, default) against the 1024-thread one, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03h}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for r in 1 2; do
  for kv in HSC_CJOIN2=1 HSC_CJOIN2=0; do
    env $kv timeout -k 10 300 python3 bench.py --config 3 --no-cpu --no-pmc --no-api > gpurun_out/${T}_${kv}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_${kv}_$r.log; exit 1; }
    python3 scripts/benchsum.py gpurun_out/${T}_${kv}_$r.log
  done
done
echo r03h done
