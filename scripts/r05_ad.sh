#!/bin/bash
# Round-5: no stream made at context creation (hardware queues); config 3 on
# three streams, config 1's first check, config 2.
tag=${1:-r05ad}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step c3 300 python -u bench.py --config 3 --no-cpu --no-pmc --steps 30
step c2 300 python -u bench.py --no-cpu --no-pmc --no-api --steps 50
step c1 600 python -u bench.py --config 1
