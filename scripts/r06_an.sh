#!/bin/bash
# Round-6: ingest cases for the LSN-in-key and one-sweep paths; config 1
# steady state x3 (small sorts back on the count + scan passes); config 2.
tag=${1:-r06an}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_gpu_ingest.py -m gpu -q -x --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c1a 400 python -u bench.py --config 1
step c1b 400 python -u bench.py --config 1
step c1c 400 python -u bench.py --config 1
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
