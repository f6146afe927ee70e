#!/bin/bash
# Round-5: config 4 next-writer directory size A/B (HSC_GRAPH_DIR =
# "writers per bucket,max directory bits"; default 32,20).
tag=${1:-r05o}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step base 400 python -u bench.py --config 4 --steps 10 --no-cpu
HSC_GRAPH_DIR=4,24 step d4_24 400 python -u bench.py --config 4 --steps 10 --no-cpu
HSC_GRAPH_DIR=2,25 step d2_25 400 python -u bench.py --config 4 --steps 10 --no-cpu
HSC_GRAPH_DIR=8,23 step d8_23 400 python -u bench.py --config 4 --steps 10 --no-cpu
step base2 400 python -u bench.py --config 4 --steps 10 --no-cpu
