#!/bin/bash
# Round-5: verdict bitmap built by the plan + join (no pack pass): full GPU
# suite, configs 2 / 5 / 3 bench (bitmaps compared with --check).
tag=${1:-r05q}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c2 300 python -u bench.py --steps 30 --no-cpu --no-pmc --no-api --check
step c5 300 python -u bench.py --config 5 --steps 30 --no-cpu --no-pmc --no-api --check
step c3 300 python -u bench.py --config 3 --steps 30 --no-cpu --no-pmc --no-api --check
