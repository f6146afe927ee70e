#!/bin/bash
# Round-5: multi benches with 8 hardware queues forced by bench.py.
tag=${1:-r05ah}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step inproc2 400 python -u bench.py --inproc 2 --steps 30
step inproc2_loop 400 python -u bench.py --inproc 2 --steps 30 --loopback --no-api
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29543 step rank1 300 python -u bench.py --rank-path --steps 50 --no-api
step pytest_multi 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -q -x --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest_multi.log
