#!/bin/bash
# Default bench (no CPU / PMC / API legs) under the main library and A/B
# variants in comdb2_amd/lib/ab (LIBS="name ..."); narrow GPU tests on each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for l in main ${LIBS:-}; do
  if [ $l = main ]; then unset HSC_LIB; else export HSC_LIB=$PWD/comdb2_amd/lib/ab/$l.so; fi
  if [ $l != main ]; then
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_streams.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/libab_${l}_pytest.log 2>&1 || { tail -20 gpurun_out/libab_${l}_pytest.log; exit 1; }
    echo "$l: $(tail -1 gpurun_out/libab_${l}_pytest.log)"
  fi
  for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-api ${BENCH_ARGS:-} > gpurun_out/libab_${l}_$rep.log 2>&1 || { tail -20 gpurun_out/libab_${l}_$rep.log; exit 1; }
  tail -1 gpurun_out/libab_${l}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$l', 'value', round(d['value']/1e6), 'ms', round(d['ms_per_step']*1e3,1), 'serial', round(d['config']['serial_ms_per_step']*1e3,1), 'frac', round(r['frac'],3), round(r['frac_1stream'],3), 'l3', round(r['l3_resident']['frac'],3), round(r['l3_resident']['frac_1stream'],3), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()})"
  done
done
