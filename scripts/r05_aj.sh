#!/bin/bash
# Round-5: stream tests (lane fences at stream switches, a rebuild between
# streams), then config 5 overflow join blocks 2048 vs 4096.
tag=${1:-r05aj}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_incremental.py -m gpu -q -x --timeout 200 --timeout-method thread > $out/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config 5 --no-cpu --no-pmc --steps 30 > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do
  run x2048_$r X=1
  run x4096_$r HSC_JOIN_EXTRA=4096
done
