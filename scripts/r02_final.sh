#!/bin/bash
# Round-2 record: GPU suite, default bench (ring + PMC + CPU baseline + C-ABI
# legs), its kernel trace, configs 1 / 3 / 5 and the 2-rank rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r02z}
mkdir -p gpurun_out
step() { echo "[final] $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
step bench
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_kt -o run -- python3 bench.py --no-cpu --no-pmc --no-api > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
python3 scripts/overlap.py ${T}_kt > gpurun_out/${T}_kt_overlap.txt 2>&1 || true
step config1
timeout -k 10 300 python3 bench.py --config 1 --no-pmc > gpurun_out/${T}_c1.log 2> gpurun_out/${T}_c1.err || { tail -20 gpurun_out/${T}_c1.err; exit 1; }
step config3
timeout -k 10 600 python3 bench.py --config 3 > gpurun_out/${T}_c3.log 2> gpurun_out/${T}_c3.err || { tail -20 gpurun_out/${T}_c3.err; exit 1; }
step config5
timeout -k 10 600 python3 bench.py --config 5 --check > gpurun_out/${T}_c5.log 2> gpurun_out/${T}_c5.err || { tail -20 gpurun_out/${T}_c5.err; exit 1; }
step rehearsal
for cfg in 2 5; do
  HSC_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2953$cfg bench.py --gpus 2 --config $cfg --no-cpu --no-pmc \
    > gpurun_out/${T}_c${cfg}_gloo2.log 2> gpurun_out/${T}_c${cfg}_gloo2.err || { tail -20 gpurun_out/${T}_c${cfg}_gloo2.err; exit 1; }
done
step done
