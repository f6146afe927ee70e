#!/bin/bash
# Config 4 sharded SCC: GPU tests, 1-GPU bench, 2-rank gloo rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_shard.py tests/test_graph.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/tgs.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/c4.log 2>&1 || exit $?
HSC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --config 4 --gpus 2 --steps 3 --warmup 1 > gpurun_out/c4g2.log 2>&1 || exit $?
