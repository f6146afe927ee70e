#!/bin/bash
# Round-5: 4 in-process members on the one GPU (direct and loopback), config 2
# and config 5 pieces; per-member imbalance and routings compared.
tag=${1:-r05ak}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step inproc4 500 python -u bench.py --inproc 4 --steps 20 --no-api
step inproc4_loop 500 python -u bench.py --inproc 4 --steps 20 --loopback --no-api
step inproc2_c5 500 python -u bench.py --inproc 2 --config 5 --steps 20 --no-api
