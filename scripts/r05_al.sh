#!/bin/bash
# Round-5: 1024-thread k_plan_s (ab7/plan1024.so) vs 512 on config 2 (one and
# two streams).
tag=${1:-r05al}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-api --steps 50 > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do
  run p512_$r X=1
  run p1024_$r HSC_LIB=$PWD/comdb2_amd/lib/ab7/plan1024.so
done
