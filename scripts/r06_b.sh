#!/bin/bash
# Round-6: GPU suite after the replica-slice fix, then config 4 and config 1.
tag=${1:-r06b}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
  return $rc
}
step pytest 900 python -u -m pytest tests/ -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread
rc=$?; tail -12 $out/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
step c4 600 python -u bench.py --config 4
step c1 600 python -u bench.py --config 1
