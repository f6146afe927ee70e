#!/bin/bash
# Single-stream kernel traces (rocprofv3 --kernel-trace --stats) of the
# default config-2 workload for each environment setting in AB, with the
# overlap/gap summary of the timed probe loop (scripts/overlap.py) and the
# per-kernel stats; then the same for a build only (HSC_BUILD_TRACE stamps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03p}
mkdir -p gpurun_out
for kv in ${AB:-NONE=1}; do
  name=${TAG}_${kv//=/_}
  env $kv timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$name -o run -- python3 bench.py --no-cpu --no-pmc --no-api --streams ${STREAMS:-1} --steps 20 ${BENCH_ARGS:-} > gpurun_out/$name.log 2>&1 || { tail -20 gpurun_out/$name.log; exit 1; }
  python3 scripts/overlap.py $name
  head -25 gpurun_out/$name/run_kernel_stats.csv | cut -d, -f1-4
done
