#!/bin/bash
# Round-6: config-4 bucket lines (one line per read) -- graph tests, the
# config-4 line with PMC traffic, A/B against the directory search, trace.
tag=${1:-r06m}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c4 500 python -u bench.py --config 4
HSC_GRAPH_PT=0 step c4dir 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c4trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
