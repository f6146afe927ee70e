#!/bin/bash
# Round-5: full GPU suite; the in-process 2-member routed step with the
# members' launches from one thread vs the pool, and its HIP API trace.
tag=${1:-r05m}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
step pytest 700 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step inproc2 400 python -u bench.py --inproc 2 --steps 30 --no-api
HSC_MULTI_PAR_LAUNCH=1 step inproc2_par 400 python -u bench.py --inproc 2 --steps 30 --no-api
step hip_inproc2 400 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $out/${tag}_hip_inproc2 -o k -- python3 bench.py --inproc 2 --steps 20 --no-api
