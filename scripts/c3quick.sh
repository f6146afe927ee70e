#!/bin/bash
# Compact/wide GPU tests, then the config-3 bench (compact) with parity check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_config3.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c3q_tests.log 2>&1 || { tail -30 gpurun_out/c3q_tests.log; exit 1; }
tail -3 gpurun_out/c3q_tests.log
timeout -k 10 400 python bench.py --config 3 --check > gpurun_out/c3c.log 2>&1 || exit $?
tail -1 gpurun_out/c3c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['probe_phase']; print(round(d['value']/1e6), round(d['ms_per_step']*1e3,1), d['config'].get('serial_ms_per_step'), d['parity'], {k: round(x['event_ms']*1e3,1) for k,x in p['kernels'].items()})"
