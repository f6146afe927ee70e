#!/bin/bash
# Round-5: multi steps with prepared call arguments (one foreign call per
# step): world-1 per-rank, 2 in-process members (direct and loopback), traces.
tag=${1:-r05t}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 step rank1 300 python -u bench.py --rank-path --steps 50
step inproc2 400 python -u bench.py --inproc 2 --steps 30
step inproc2_loop 400 python -u bench.py --inproc 2 --steps 30 --loopback --no-api
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29532 step trace_rank1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_rank1 -o k -- python3 bench.py --rank-path --steps 20
step trace_inproc2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_inproc2 -o k -- python3 bench.py --inproc 2 --steps 20 --no-api
