#!/bin/bash
# Round-5: members' launches from pool threads on one GPU
# (HSC_MULTI_PAR_LAUNCH) with 8 hardware queues, 2 and 4 members.
tag=${1:-r05am}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step i2 400 python -u bench.py --inproc 2 --steps 30 --no-api
HSC_MULTI_PAR_LAUNCH=1 step i2_par 400 python -u bench.py --inproc 2 --steps 30 --no-api
step i4 500 python -u bench.py --inproc 4 --steps 20 --no-api
HSC_MULTI_PAR_LAUNCH=1 step i4_par 500 python -u bench.py --inproc 4 --steps 20 --no-api
