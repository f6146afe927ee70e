#!/bin/bash
# Round-5: small-path staging warmed at context creation (config 1's first
# check), collector / incremental tests.
tag=${1:-r05aa}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_collector.py tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_multi.py -m gpu -q -x --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c1 600 python -u bench.py --config 1
