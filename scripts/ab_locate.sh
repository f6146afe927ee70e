#!/bin/bash
# A/B of locate chunk shapes on config 2 (one and two streams), bench legs only.
out=gpurun_out; mkdir -p $out
for v in base l512 tp2; do
  if [ $v = base ]; then lib=""; else lib=comdb2_amd/lib/abx/libhsc_$v.so; fi
  HSC_LIB=$lib timeout -k 10 300 python -u bench.py --no-api --no-cpu --no-pmc --steps 20 > $out/ab_$v.json 2> $out/ab_$v.err
  rc=$?; echo "$v rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $out/ab_$v.err; exit $rc; fi
done
