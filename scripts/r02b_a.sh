#!/bin/bash
# Round-2 record, part A: GPU suite, default bench (ring + PMC + CPU baseline +
# C-ABI legs), its kernel trace (and timed-loop overlap).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r02b}
mkdir -p gpurun_out
step() { echo "[rec] $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
step bench
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.log; echo
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_kt -o run -- python3 bench.py --no-cpu --no-pmc --no-api > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
python3 scripts/overlap.py ${T}_kt > gpurun_out/${T}_kt_overlap.txt 2>&1 || true
step done
