#!/bin/bash
# Round-6: compact join staged key words A/B (3 / 2 / 1 words in LDS) on
# config 3, parity of the 1-word form; config 2 re-check.
tag=${1:-r06k}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
HSC_CJOIN_WL=1 step pytest1 400 python -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest1.log
step wl3 300 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
HSC_CJOIN_WL=2 step wl2 300 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
HSC_CJOIN_WL=1 step wl1 300 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
step wl3b 300 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
step c2 300 python -u bench.py --no-cpu --no-api --no-pmc
