#!/bin/bash
# Round-5: full GPU suite on the current build; world-1 per-rank step.
tag=${1:-r05x}
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
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 step rank1 300 python -u bench.py --rank-path --steps 50 --no-api
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29536 step rank1b 300 python -u bench.py --rank-path --steps 50 --no-api
python3 -c "import __graft_entry__ as g; g.smoke()" > $out/${tag}_smoke.log 2>&1; echo smoke rc=$?
