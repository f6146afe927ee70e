#!/bin/bash
# Round-6 last check of the committed tree after the fused narrow level pass: the whole GPU suite, smoke, the default line, configs 4, 3, 5, 1.
tag=${1:-r06last3}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 900 python -u -m pytest tests/ -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step default 600 python -u bench.py
step c4 500 python -u bench.py --config 4
step c3 500 python -u bench.py --config 3
step c5 500 python -u bench.py --config 5
step c1 500 python -u bench.py --config 1
