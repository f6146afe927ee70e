#!/bin/bash
# Round-6: config-2 A/B of the device-buffer headroom (1/2 vs the r05 1/8),
# alternating, to tell a regression from box variance.
tag=${1:-r06l}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-api --no-pmc > $out/${tag}_half$i.log 2> $out/${tag}_half$i.err || exit $?
  echo "half$i ok"
  HSC_DBUF_SLACK=8 timeout -k 10 300 python -u bench.py --no-cpu --no-api --no-pmc > $out/${tag}_eighth$i.log 2> $out/${tag}_eighth$i.err || exit $?
  echo "eighth$i ok"
done
