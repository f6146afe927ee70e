#!/bin/bash
# Config 5 (global Zipf(1.2) over 2^32 keys): 1-GPU bench with the oracle
# sort-join parity check, then the N=2 path rehearsed with both ranks on the
# one GPU over gloo (sampled splitters, row exchange, imbalance report).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02c5}
KEYS=${KEYS:-125000000}
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --config 5 --c5-keys $KEYS --no-cpu --no-pmc --check \
  > gpurun_out/${TAG}_n1.log 2> gpurun_out/${TAG}_n1.err || { tail -20 gpurun_out/${TAG}_n1.err; exit 1; }
tail -c 900 gpurun_out/${TAG}_n1.log; echo
[ -n "$NO_REHEARSAL" ] && exit 0
HSC_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 5 --c5-keys $KEYS \
  --no-cpu --no-pmc > gpurun_out/${TAG}_gloo2.log 2> gpurun_out/${TAG}_gloo2.err || { tail -20 gpurun_out/${TAG}_gloo2.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_gloo2.log; echo
