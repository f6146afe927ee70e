cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in def all; do
  if [ $v = all ]; then export HSC_JOIN_ALL_WORDS=1; fi
  timeout -k 10 300 python3 bench.py --config 3 --no-cpu --no-pmc --no-api > gpurun_out/c3ab_$v.log 2>&1 || { tail -20 gpurun_out/c3ab_$v.log; exit 1; }
  tail -1 gpurun_out/c3ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', 'value', round(d['value']/1e6), 'ms', round(d['ms_per_step']*1e3,1), 'serial', round(d['config']['serial_ms_per_step']*1e3,1), 'frac', round(r['frac'],3), round(r['frac_1stream'],3), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()})"
done
