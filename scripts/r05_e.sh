#!/bin/bash
# config 4 (raw rows only, one-pass cut) + config 1 legs with slow-check detail
tag=${1:-r05e}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c4 500 python -u bench.py --config 4 --no-cpu
step c1 600 python -u bench.py --config 1 --no-cpu
