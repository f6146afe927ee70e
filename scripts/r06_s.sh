#!/bin/bash
# Round-6: epoch-tagged point index (no clearing pass on rebuilds): compact
# tile tests, config-3 line (ingest), config 4 (short-circuit cut back).
tag=${1:-r06s}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_gpu_ctiles.py tests/test_gpu_config3.py tests/test_gpu_full_configs.py tests/test_gpu_multi.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c3 300 python -u bench.py --config 3 --no-cpu --no-api --no-pmc
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
