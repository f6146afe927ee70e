#!/bin/bash
# Round-5: lane fences recorded when the context leaves a stream (not per
# batch): full GPU suite, config 2 / 5 / 3 benches, the per-rank step.
tag=${1:-r05ac}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c2a 300 python -u bench.py --no-cpu --no-pmc --no-api --steps 50
step c2b 300 python -u bench.py --no-cpu --no-pmc --no-api --steps 50
step c5 300 python -u bench.py --config 5 --no-cpu --no-pmc --steps 30 --check
step c3 300 python -u bench.py --config 3 --no-cpu --no-pmc --steps 30 --check
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29539 step rank1 300 python -u bench.py --rank-path --steps 50 --no-api
step inproc2 400 python -u bench.py --inproc 2 --steps 30 --no-api
