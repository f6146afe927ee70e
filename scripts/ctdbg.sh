#!/bin/bash
# Compact-tile join diagnostics: full join vs searches skipped vs gathers skipped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 0 1 2; do
  HSC_CT_DBG=$d timeout -k 10 300 python3 bench.py --config 3 --no-cpu --no-pmc --no-api --ring-gb 0 --streams 1 > gpurun_out/ctdbg_$d.log 2>&1 || { tail -20 gpurun_out/ctdbg_$d.log; exit 1; }
  tail -1 gpurun_out/ctdbg_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dbg $d', round(d['ms_per_step']*1e3,1), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()})"
done
