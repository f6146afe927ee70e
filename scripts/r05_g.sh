#!/bin/bash
# the default bench line (config 2: PMC passes, api legs with the collector,
# CPU baseline), configs 3 and 5, and the two tests fixed after r05f
tag=${1:-r05g}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_narrow.py tests/test_collector.py -m gpu -q --timeout 200 --timeout-method thread
tail -3 $out/${tag}_pytest.log
step bench 600 python -u bench.py
step config3 400 python -u bench.py --config 3
step config5 500 python -u bench.py --config 5
