#!/bin/bash
# Round-6: config-3 one-stream kernel trace with the point index, config-2
# kernel trace (ingest kernels included), fold diagnosis with the host-noise
# baseline.
tag=${1:-r06h}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step c3s1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c3s1 -o k -- python3 bench.py --config 3 --no-cpu --no-pmc --no-api --streams 1
step c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c2 -o k -- python3 bench.py --no-cpu --no-pmc --no-api
step folddiag32k 300 python -u scripts/fold_diag.py 32768 100000
step pytestg 400 python -u -m pytest tests/test_graph.py tests/test_graph_shard.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytestg.log
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c4trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
