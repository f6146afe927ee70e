#!/bin/bash
# Round-6 closing lines of the committed tree (after the level-1 tile maxima):
# configs 3, 5, 1 and the 2-member in-process rehearsal.
tag=${1:-r06bf}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step c3 500 python -u bench.py --config 3
step c5 500 python -u bench.py --config 5
step c1 500 python -u bench.py --config 1
step inproc2 500 python -u bench.py --inproc 2 --steps 30
