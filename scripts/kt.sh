#!/bin/bash
# Kernel trace (+ optional PMC passes) of a short bench run; prints per-kernel
# average durations and counters.  PMC="SQ_A SQ_B ..." adds one counter pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-kt}
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$T -o run -- \
  python3 bench.py --no-cpu --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/$T.log 2>&1 || exit $?
if [ -n "$PMC" ]; then
  timeout -k 10 180 rocprofv3 --pmc $PMC -T --output-format csv -d gpurun_out/${T}_pmc -o run -- \
    python3 bench.py --no-cpu --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/${T}_pmc.log 2>&1 || exit $?
fi
exit 0
