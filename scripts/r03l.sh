#!/bin/bash
# Snapshot-rank pre-pass: the narrow / parity / small GPU tests (forced tile
# layouts now skip the small-batch path), then config-5 A/B of
# HSC_SNAP_PREPASS (default on) twice, and a config-2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03l}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_streams.py tests/test_gpu_full_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for r in 1 2; do
  for kv in HSC_SNAP_PREPASS=1 HSC_SNAP_PREPASS=0; do
    env $kv timeout -k 10 400 python3 bench.py --config 5 --no-cpu --no-pmc --no-api > gpurun_out/${T}_${kv}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_${kv}_$r.log; exit 1; }
    python3 scripts/benchsum.py gpurun_out/${T}_${kv}_$r.log
  done
done
timeout -k 10 400 python3 bench.py --no-cpu --no-pmc --no-api > gpurun_out/${T}_c2.log 2>&1 || exit 1
python3 scripts/benchsum.py gpurun_out/${T}_c2.log
echo r03l done
