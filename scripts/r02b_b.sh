#!/bin/bash
# Round-2 record, part B: config 3 (bench with PMC traffic + kernel trace),
# configs 1 and 5, the 2-rank gloo rehearsals of configs 2 and 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r02b}
mkdir -p gpurun_out
step() { echo "[rec] $1 $(date +%T)"; }
step config3
timeout -k 10 600 python3 bench.py --config 3 --check > gpurun_out/${T}_c3.log 2> gpurun_out/${T}_c3.err || { tail -20 gpurun_out/${T}_c3.err; exit 1; }
step config3-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_c3kt -o run -- python3 bench.py --config 3 --no-pmc --no-api > gpurun_out/${T}_c3kt.log 2>&1 || { tail -20 gpurun_out/${T}_c3kt.log; exit 1; }
step config1
timeout -k 10 300 python3 bench.py --config 1 --no-pmc > gpurun_out/${T}_c1.log 2> gpurun_out/${T}_c1.err || { tail -20 gpurun_out/${T}_c1.err; exit 1; }
step config5
timeout -k 10 600 python3 bench.py --config 5 --check > gpurun_out/${T}_c5.log 2> gpurun_out/${T}_c5.err || { tail -20 gpurun_out/${T}_c5.err; exit 1; }
step rehearsal
for cfg in 2 3; do
  HSC_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2953$cfg bench.py --gpus 2 --config $cfg --no-cpu --no-pmc \
    > gpurun_out/${T}_c${cfg}_gloo2.log 2> gpurun_out/${T}_c${cfg}_gloo2.err || { tail -20 gpurun_out/${T}_c${cfg}_gloo2.err; exit 1; }
done
step done
