#!/bin/bash
# Graph stress: GPU graph tests (stress histories vs Tarjan, rw pairs -> graph),
# then the config-4 bench on a high-concurrency history.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02g}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_graph.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
grep -E "stress|passed|failed" gpurun_out/${TAG}_pytest.log | tail -6
timeout -k 10 400 python3 bench.py --config 4 --history-txns ${TXNS:-2000000} --c4-concurrent 0.5 --c4-max-lag 512 --c4-keys ${KEYS:-200000} --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_c4stress.log 2> gpurun_out/${TAG}_c4stress.err || { tail -20 gpurun_out/${TAG}_c4stress.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_c4stress.log; echo
