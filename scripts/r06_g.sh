#!/bin/bash
# Round-6: appends after the huge-page fix (config 1, fold diagnosis), the
# 4-member one-GPU rehearsal with the box's 4 hardware queues and with 8.
tag=${1:-r06g}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_pending.py tests/test_gpu_recon.py -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step c1 400 python -u bench.py --config 1 --no-cpu
step folddiag32k 300 python -u scripts/fold_diag.py 32768 100000
step inproc4q4 500 python -u bench.py --inproc 4 --steps 30 --no-cpu --no-pmc --no-api --hw-queues 4
step inproc4 500 python -u bench.py --inproc 4 --steps 30 --no-cpu --no-pmc --no-api
