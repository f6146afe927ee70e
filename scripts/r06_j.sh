#!/bin/bash
# Round-6: full GPU suite after the stream-ordering fixes (graph cut copies,
# multi graph step, splitters, adopt), the txn-ordered writer sort, the
# contiguous writer gather and the ingest changes; config 4 / config 2 lines.
tag=${1:-r06j}
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
tail -3 $out/${tag}_pytest.log
step c4 500 python -u bench.py --config 4
step c4trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
step c2 400 python -u bench.py --no-cpu --no-api --no-pmc
