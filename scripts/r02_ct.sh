#!/bin/bash
# Compact tiles: GPU tests, then config 3 with and without them (bench clock,
# per-kernel events).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ct}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py tests/test_gpu_compact.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
for mode in ct wide; do
  extra=""; [ $mode = wide ] && extra="--compact-wide"
  timeout -k 10 400 python3 bench.py --config 3 --no-cpu --no-pmc --no-api $extra ${BENCH_ARGS:-} > gpurun_out/${TAG}_c3_$mode.log 2>&1 || { tail -20 gpurun_out/${TAG}_c3_$mode.log; exit 1; }
  tail -1 gpurun_out/${TAG}_c3_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$mode', 'value', round(d['value']/1e6), 'ms', round(d['ms_per_step']*1e3,1), 'serial', round(d['config']['serial_ms_per_step']*1e3,1), 'frac', round(r['frac'],3), round(r['frac_1stream'],3), 'l3', round(r['l3_resident']['frac'],3), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()}, d['config']['window_layout'])"
done
