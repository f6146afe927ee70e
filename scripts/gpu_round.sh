#!/bin/bash
# One GPU call: the GPU test suite, then bench lines.  Stops at the first
# step that faults, aborts or times out (exit codes other than 0 / 1).
# usage: scripts/gpu_round.sh TAG "bench args" ["bench args" ...]
tag=$1; shift
out=gpurun_out
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $out/${tag}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $out/${tag}_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 500 python -u bench.py $args > $out/${tag}_bench$i.json 2> $out/${tag}_bench$i.err
  rc=$?
  echo "bench $i ($args) rc=$rc"; tail -c 600 $out/${tag}_bench$i.json
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_bench$i.err; exit $rc; fi
done
