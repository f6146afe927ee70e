#!/bin/bash
# Round-5: price of the per-batch lane event on the config-2 bench loop.
tag=${1:-r05ab}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-api --steps 50 > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2 3; do
  run ev_$r X=1
  run noev_$r HSC_DIAG_NO_LANE_EVENT=1
done
