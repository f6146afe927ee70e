#!/bin/bash
# Round-6: PMC FETCH_SIZE / WRITE_SIZE per window-build kernel (config 2,
# bench.py --pmc-child: one window build + the probe ring), one pass each.
tag=${1:-r06bg}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T --output-format csv -d $out/${tag}_$ctr -o run -- python3 bench.py --pmc-child --config 2 > $out/${tag}_$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/${tag}_$ctr.log; exit $rc; fi
done
