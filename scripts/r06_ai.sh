#!/bin/bash
# Round-6: LSN-packed sort A/B in swapped order (probe throughput check)
tag=${1:-r06ai}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
HSC_NO_LSN_PACK=1 step c2old 400 python -u bench.py --no-cpu --no-pmc --no-api
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_NO_LSN_PACK=1 step c2old2 400 python -u bench.py --no-cpu --no-pmc --no-api
step c2b 400 python -u bench.py --no-cpu --no-pmc --no-api
