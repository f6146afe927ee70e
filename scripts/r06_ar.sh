#!/bin/bash
# Round-6: the unpack places distinct rows by a look-back (no bcount pass /
# scan) -- ingest, window, graph suites; config 2 and 4.
tag=${1:-r06ar}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest1 300 python -u -m pytest tests/test_gpu_ingest.py -m gpu -q -x --timeout 120 --timeout-method thread
step pytest 800 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_incremental.py tests/test_gpu_full_configs.py tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c4b 400 python -u bench.py --config 4 --no-cpu --no-pmc
