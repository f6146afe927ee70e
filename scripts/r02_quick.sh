#!/bin/bash
# Quick loop: selected GPU tests, bench ring (no CPU / PMC / API legs), stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1 || { tail -30 gpurun_out/quick_pytest.log; exit 1; }
  tail -2 gpurun_out/quick_pytest.log
fi
timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-api ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1 || { tail -20 gpurun_out/quick_bench.log; exit 1; }
tail -1 gpurun_out/quick_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']/1e6), 'ms', round(d['ms_per_step']*1e3,1), 'serial', round(d['config']['serial_ms_per_step']*1e3,1), 'frac', round(r['frac'],3), round(r['frac_1stream'],3), 'l3', round(r['l3_resident']['frac'],3), round(r['l3_resident']['frac_1stream'],3), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()}, 'ingest_ms', round(d['ingest_ms'],2))"
if [ -f comdb2_amd/lib/ab/stamps.so ] && [ -z "$NO_STAMPS" ]; then
  HSC_STAMPS=1 HSC_LIB=$PWD/comdb2_amd/lib/ab/stamps.so timeout -k 10 200 python3 bench.py --pmc-child > gpurun_out/quick_stamps.log 2>&1 || { tail -5 gpurun_out/quick_stamps.log; exit 1; }
  grep stamps gpurun_out/quick_stamps.log | tail -2
fi
