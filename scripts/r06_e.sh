#!/bin/bash
# Round-6: config-3 point index A/B (2-bucket index vs join records), the
# small-cut SCC kernel and config-4 line, the fold-stall diagnosis.
tag=${1:-r06e}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_ctiles.py tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -3 $out/${tag}_pytest.log
step c3pts 400 python -u bench.py --config 3 --no-cpu --no-api
step c3rec 400 python -u bench.py --config 3 --no-cpu --no-api --paths 64
step c3pts2 400 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
step folddiag 200 python -u scripts/fold_diag.py 1000 10000
step folddiag32k 300 python -u scripts/fold_diag.py 32768 100000
