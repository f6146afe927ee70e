#!/bin/bash
# Round-5 run: compact-tile locate chunks sized to one workgroup per CU,
# points mapped once per wave, in-process multi merge over verdict bytes.
# Each step under its own limit; stops at the first fault / abort / timeout.
tag=${1:-r05k}
part=${2:-all}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py tests/test_gpu_multi.py tests/test_gpu_narrow.py tests/test_gpu_full_configs.py tests/test_graph_shard.py -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step config3 400 python -u bench.py --config 3 --steps 20 --check
[ $part = c3 ] && exit 0
step inproc2 400 python -u bench.py --inproc 2 --steps 30
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 step rank1 300 python -u bench.py --rank-path --steps 50
step trace_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c3 -o k -- python3 bench.py --config 3 --steps 20 --no-pmc
step trace_inproc2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_inproc2 -o k -- python3 bench.py --inproc 2 --steps 20
