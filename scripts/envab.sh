#!/bin/bash
# bench.py (no CPU leg) under several values of one environment variable:
#   VAR=HSC_JOIN_WG_PER_CU VALUES="4 2 0" bash scripts/envab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/envab_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/envab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['probe_phase']; print('$VAR=$v', round(d['value']/1e6), round(d['ms_per_step']*1e3,1), {k: round(x['event_ms']*1e3,1) for k,x in p['kernels'].items()})"
done
