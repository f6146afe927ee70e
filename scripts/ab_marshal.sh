#!/bin/bash
# A/B of the host marshal (scripts/marshal_bench.py, CPU only) between the
# in-tree library and another build, alternating.
other=$1
for i in 1 2; do
  for v in new other; do
    if [ $v = new ]; then lib=""; else lib=$other; fi
    echo "== $v $i"
    HSC_LIB=$lib timeout -k 10 120 python -u scripts/marshal_bench.py 2>&1 | grep -v "^flat"
  done
done
