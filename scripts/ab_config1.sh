#!/bin/bash
# A/B of the commit stream (config 1) between the in-tree library and another
# build (argument: path of its libhsc.so), alternating, each leg its own run.
other=$1; out=gpurun_out; mkdir -p $out
for i in 1 2; do
  for v in new other; do
    if [ $v = new ]; then lib=""; else lib=$other; fi
    HSC_LIB=$lib timeout -k 10 200 python -u bench.py --config 1 --no-cpu > $out/abc1_${v}_$i.json 2> $out/abc1_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $out/abc1_${v}_$i.err; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open('$out/abc1_${v}_$i.json') if l.startswith('{')][-1]); print('$v', round(d['value']), d['check_us']['mean'], d['small_path']['wait_us'], d['small_path']['launch_us'])"
  done
done
