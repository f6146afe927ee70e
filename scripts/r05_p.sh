#!/bin/bash
# Round-5: batches in flight (HIP streams the ring rotates over) on configs 2/3/5.
tag=${1:-r05p}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
for c in 2 5 3; do
  for s in 2 3 4; do
    step c${c}_s$s 300 python -u bench.py --config $c --streams $s --steps 30 --no-cpu --no-pmc --no-api
  done
done
