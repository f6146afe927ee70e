#!/bin/bash
# Round-6: ww rows from the sort's keys-only unpack (A/B HSC_GRAPH_NO_WW_FUSE=1)

tag=${1:-r06at}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
HSC_GRAPH_NO_WW_FUSE=1 step c4old 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c4b 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c4k 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_k -o k -- python3 bench.py --config 4 --no-cpu --no-pmc --steps 3 --warmup 1
