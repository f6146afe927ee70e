#!/bin/bash
# Round-5: config 1 (the drop-in entry now through the context's collector)
# and the in-process 2-member api legs with the in-flight sweep.
tag=${1:-r05z}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step c1 600 python -u bench.py --config 1
step inproc2 400 python -u bench.py --inproc 2 --steps 30
