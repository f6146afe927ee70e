#!/bin/bash
# Round-6 first GPU run of HEAD: full GPU suite, smoke, the default bench line,
# the 2-member in-process rehearsal (replicated + pieces drop-in legs).
tag=${1:-r06a}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 900 python -u -m pytest tests/ -m gpu -q --maxfail 15 --timeout 300 --timeout-method thread
tail -15 $out/${tag}_pytest.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step default 600 python -u bench.py
step inproc2 500 python -u bench.py --inproc 2 --steps 30
