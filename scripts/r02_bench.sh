#!/bin/bash
# Default bench (ring + PMC passes + CPU baseline), then a kernel trace of the
# same workload for profiles/.  TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.log; echo
[ -n "$NO_KT" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_kt -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt.log; exit 1; }
tail -c 300 gpurun_out/${TAG}_kt.log; echo
