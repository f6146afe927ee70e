#!/bin/bash
# Round-5 multi-GPU run on the one-GPU box: the multi GPU tests, the world-1
# per-rank bench (one piece: no routing), 2 in-process members sharing the
# GPU (routed at marshal = the headline step; device-routed beside it), the
# loopback transport, and kernel traces of the two bench legs.  Each step
# under its own limit; stops at the first fault / abort / timeout.
tag=${1:-r05a}
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
if [ $part = full ]; then
step pytest 700 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
elif [ $part != b ]; then
step pytest_multi 500 python -u -m pytest tests/test_gpu_multi.py tests/test_graph_shard.py -m gpu -k "multi or Multi or adopt or routed or lone or rccl or loopback" -v --timeout 120 --timeout-method thread
tail -3 $out/${tag}_pytest_multi.log
fi
[ $part = a ] && exit 0
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 step rank1 300 python -u bench.py --rank-path --steps 50
step inproc2 400 python -u bench.py --inproc 2 --steps 30
[ $part = ab ] || [ $part = full ] && exit 0
step inproc2_loop 400 python -u bench.py --inproc 2 --steps 30 --loopback
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29532 step trace_rank1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_rank1 -o k -- python3 bench.py --rank-path --steps 20
step trace_inproc2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_inproc2 -o k -- python3 bench.py --inproc 2 --steps 20
