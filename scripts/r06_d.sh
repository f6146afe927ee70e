#!/bin/bash
# Round-6: the compact tiles' point index (config 3) and the config-4 writer
# gather: their GPU tests, the config-3 and config-4 bench lines, traces.
tag=${1:-r06d}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py tests/test_gpu_full_configs.py tests/test_graph.py tests/test_graph_shard.py tests/test_gpu_multi.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -3 $out/${tag}_pytest.log
step c3 500 python -u bench.py --config 3 --check
step c3trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c3s1 -o k -- python3 bench.py --config 3 --no-cpu --no-pmc --no-api --streams 1
step c4 500 python -u bench.py --config 4
step c4trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c4 -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc
step c1 400 python -u bench.py --config 1 --no-cpu
