#!/bin/bash
# Round-end evidence: rocprofv3 passes (kernel trace, FETCH_SIZE, WRITE_SIZE)
# over the default bench, then the default bench with its CPU baseline, then
# configs 3 and 5 (1 GPU, with their CPU sort-join parity checks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01i} PASSES=kt,fetch,write bash scripts/profile.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/re_bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/re_bench.log
timeout -k 10 400 python bench.py --config 3 --check --no-cpu > gpurun_out/re_c3.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --config 5 --check --no-cpu > gpurun_out/re_c5.log 2>&1 || exit $?
echo done
