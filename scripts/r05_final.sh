#!/bin/bash
# Round-5 closing run: full GPU suite, smoke, the default bench line (as the
# driver runs it) with its kernel trace, configs 3 / 5, the multi rehearsal.
tag=${1:-r05fin}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 800 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step default 600 python -u bench.py
step trace_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c2 -o k -- python3 bench.py --no-cpu --no-pmc --no-api
step c3 500 python -u bench.py --config 3
step c5 500 python -u bench.py --config 5
step inproc2 400 python -u bench.py --inproc 2 --steps 30
