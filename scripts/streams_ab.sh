#!/bin/bash
# bench under several stream counts (no CPU / PMC / API legs): CONFIG, STREAMS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-3}; do for s in ${STREAMS:-2 3 4}; do
  timeout -k 10 400 python3 bench.py --config $c --streams $s --no-cpu --no-pmc --no-api > gpurun_out/sab_${c}_$s.log 2>&1 || { tail -20 gpurun_out/sab_${c}_$s.log; exit 1; }
  tail -1 gpurun_out/sab_${c}_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('config $c streams $s', 'value', round(d['value']/1e6), 'ms', round(d['ms_per_step']*1e3,1), 'serial', round(d['config']['serial_ms_per_step']*1e3,1), 'frac', round(r['frac'],3), round(r['frac_1stream'],3), 'l3', round(r['l3_resident']['frac'],3), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()})"
done; done
