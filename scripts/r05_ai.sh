#!/bin/bash
# Round-5: config 5 overflow join blocks 2048 (default on skewed windows) vs 4096.
tag=${1:-r05ai}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config 5 --no-cpu --no-pmc --steps 30 > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do
  run x2048_$r X=1
  run x4096_$r HSC_JOIN_EXTRA=4096
done
