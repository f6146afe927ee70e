#!/bin/bash
# A/B of library builds on one GPU box: bench.py (no CPU leg) alternating
# between the in-tree libhsc.so and each $AB_DIR/*.so (default
# comdb2_amd/lib/ab), ROUNDS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${AB_ARGS:---steps 20 --warmup 3 --no-cpu}
ROUNDS=${ROUNDS:-2}
AB_DIR=${AB_DIR:-comdb2_amd/lib/ab}
for r in $(seq 1 $ROUNDS); do
  for lib in cur $AB_DIR/*.so; do
    name=$(basename "$lib" .so)
    if [ "$lib" = cur ]; then env=""; else env="HSC_LIB=$PWD/$lib"; fi
    echo "== $name round $r"
    env $env timeout -k 10 300 python bench.py $ARGS > "gpurun_out/ab_${name}_$r.log" 2>&1
    rc=$?
    tail -1 "gpurun_out/ab_${name}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['value']/1e6), round(d['ms_per_step']*1e3,1), d['config'].get('serial_ms_per_step'), {k: round(x['event_ms']*1e3,1) for k,x in d['probe_phase']['kernels'].items()})" || tail -5 "gpurun_out/ab_${name}_$r.log"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
