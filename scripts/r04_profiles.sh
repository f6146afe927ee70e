#!/bin/bash
# Round-4 evidence run: GPU suite, bench lines (default = config 2 with its
# PMC passes, configs 1, 3, 5), and a kernel trace of the default bench.
# Each step under its own time limit; stops at the first fault / abort /
# timeout (exit codes other than 0 and 1).
tag=${1:-r04p}
out=gpurun_out; mkdir -p $out
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step bench 600 python -u bench.py
step config1 300 python -u bench.py --config 1
step config3 400 python -u bench.py --config 3
step config5 500 python -u bench.py --config 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace -o k -- python3 bench.py --steps 10 --no-cpu --no-pmc --no-api
