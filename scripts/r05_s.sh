#!/bin/bash
# Round-5 record run: the default bench line (config 2, CPU baseline, PMC
# passes, api legs), its kernel trace, and configs 3 / 5 lines with traces.
tag=${1:-r05s}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step c5_x2048 300 python -u bench.py --config 5 --no-cpu --no-pmc
HSC_JOIN_EXTRA=512 step c5_x512 300 python -u bench.py --config 5 --no-cpu --no-pmc
step default 500 python -u bench.py
step trace_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c2 -o k -- python3 bench.py --no-cpu --no-pmc --no-api
step c3 400 python -u bench.py --config 3
step trace_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c3 -o k -- python3 bench.py --config 3 --no-cpu --no-pmc
step c5 400 python -u bench.py --config 5
step c4 500 python -u bench.py --config 4
step trace_c4 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c4 -o k -- python3 bench.py --config 4 --no-cpu --steps 10
