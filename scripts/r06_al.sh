#!/bin/bash
# Round-6: config-1 steady state with / without the one-sweep passes (the
# background fold's build) -- check max past the first 1000
tag=${1:-r06al}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step c1a 400 python -u bench.py --config 1
step c1c 400 python -u bench.py --config 1
step c1b 400 python -u bench.py --config 1
step c1d 400 python -u bench.py --config 1
