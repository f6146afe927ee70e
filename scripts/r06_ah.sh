#!/bin/bash
# Round-6: the LSN packed into the sort key's low bits (no gather by row
# index in the unpack) -- ingest / window / incremental / config GPU suites,
# the default line's ingest and an A/B (HSC_NO_LSN_PACK=1), unpack traces.
tag=${1:-r06ah}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_narrow.py tests/test_gpu_incremental.py tests/test_gpu_full_configs.py tests/test_gpu_ctiles.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_NO_LSN_PACK=1 step c2old 400 python -u bench.py --no-cpu --no-pmc --no-api
step c2k 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_k -o k -- python3 bench.py --no-cpu --no-pmc --no-api --steps 2
