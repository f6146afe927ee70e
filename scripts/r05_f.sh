#!/bin/bash
# compressed narrow codes: the full GPU suite, then config 1 (folds now stay narrow)
tag=${1:-r05f}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread
tail -4 $out/${tag}_pytest.log
step c1 600 python -u bench.py --config 1 --no-cpu
