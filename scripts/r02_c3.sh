#!/bin/bash
# Config 3: bench (ring + PMC traffic), then a kernel trace of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02c3}
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py --config 3 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench.log; echo
[ -n "$NO_KT" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_kt -o run -- python3 bench.py --config 3 --no-pmc ${BENCH_ARGS:-} > gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt.log; exit 1; }
echo kt-ok
