#!/bin/bash
# Round-5 A/B on config 3 (bound block size, bound tables in place, join
# staging two key words) plus the multi / single collector in-flight sweeps.
tag=${1:-r05l}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_collector.py tests/test_gpu_ctiles.py -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c3_base 300 python -u bench.py --config 3 --steps 20 --no-pmc
HSC_BOUND_NT=1024 step c3_nt1024 300 python -u bench.py --config 3 --steps 20 --no-pmc
HSC_BOUND_GLOBAL=1 step c3_glob 300 python -u bench.py --config 3 --steps 20 --no-pmc
HSC_CJOIN_WL=2 step c3_wl2 300 python -u bench.py --config 3 --steps 20 --no-pmc --check
step c3_base2 300 python -u bench.py --config 3 --steps 20 --no-pmc
step inproc2 400 python -u bench.py --inproc 2 --steps 30
step default 400 python -u bench.py --no-pmc
