#!/bin/bash
# Round-6: tests touched by the vary-mask / append-path changes, config-4
# kernel traces (partitioned read search on / off), config 1 and config 2.
tag=${1:-r06c}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -5 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_incremental.py tests/test_gpu_pending.py tests/test_gpu_parity.py tests/test_graph.py tests/test_graph_shard.py tests/test_gpu_protocol.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -3 $out/${tag}_pytest.log
step c4trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4rp1 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
export HSC_GRAPH_RP=0
step c4trace0 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4rp0 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
unset HSC_GRAPH_RP
step c1 400 python -u bench.py --config 1 --no-cpu
step c2 400 python -u bench.py --no-cpu --no-api --no-pmc
