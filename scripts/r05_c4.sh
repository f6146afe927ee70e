#!/bin/bash
# Config 4 (dependency graph + SCC): the bench line through the C sharded step
# and a kernel trace of hsc_graph.hip at 100M ops.
tag=${1:-r05c4}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step bench 500 python -u bench.py --config 4 --no-cpu
step trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace -o k -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu
[ "$2" = c1 ] && step config1 600 python -u bench.py --config 1
exit 0
