#!/bin/bash
# Round-5: hardware queues per process (GPU_MAX_HW_QUEUES 4, the box default,
# vs 8) for the in-process 2-member step and configs 3 / 2.
tag=${1:-r05ae}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name cmd...
  local name=$1; shift
  timeout -k 10 400 "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
run inproc2_q4 python -u bench.py --inproc 2 --steps 30 --no-api
GPU_MAX_HW_QUEUES=8 run inproc2_q8 python -u bench.py --inproc 2 --steps 30 --no-api
run c3_q4 python -u bench.py --config 3 --no-cpu --no-pmc --steps 30
GPU_MAX_HW_QUEUES=8 run c3_q8 python -u bench.py --config 3 --no-cpu --no-pmc --steps 30
GPU_MAX_HW_QUEUES=8 run c3_q8_s4 python -u bench.py --config 3 --no-cpu --no-pmc --steps 30 --streams 4
GPU_MAX_HW_QUEUES=8 run c2_q8 python -u bench.py --no-cpu --no-pmc --no-api --steps 50
GPU_MAX_HW_QUEUES=8 run c2_q8_s3 python -u bench.py --no-cpu --no-pmc --no-api --steps 50 --streams 3
