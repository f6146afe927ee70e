#!/bin/bash
# Kernel trace of the large-set coalesce case (level-parallel sort + merge).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_co -o run -- python3 scripts/bench_coalesce.py level-parallel > gpurun_out/prof_co.log 2>&1 || exit $?
tail -12 gpurun_out/prof_co.log
cat gpurun_out/prof_co/run_kernel_stats.csv | cut -d, -f1-8
