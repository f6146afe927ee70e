#!/bin/bash
# Single-stream kernel trace of the default workload (ring), for gap analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02s1}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --no-cpu --no-pmc --no-api --streams 1 --steps 20 ${BENCH_ARGS:-} > gpurun_out/$TAG.log 2>&1 || { tail -20 gpurun_out/$TAG.log; exit 1; }
python3 scripts/overlap.py $TAG
