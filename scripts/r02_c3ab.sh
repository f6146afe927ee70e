#!/bin/bash
# Config 3 kernel traces, probes in group order vs read-set order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in group read; do
  HSC_PROBE_ORDER=$o timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/c3ab_$o -o run -- python3 bench.py --config 3 --no-pmc --steps 10 --ring-gb 0 > gpurun_out/c3ab_$o.log 2>&1 || { tail -5 gpurun_out/c3ab_$o.log; exit 1; }
  echo "== $o"; head -9 gpurun_out/c3ab_$o/run_kernel_stats.csv | cut -d, -f1-4
done
