#!/bin/bash
# N > 1 paths rehearsed on the one GPU over gloo (both ranks on cuda:0):
# config 2 (bitmap all-gather merge) and config 5 (sampled splitters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02m}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_merge.py -m gpu -q --timeout 100 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for cfg in 2 5; do
  HSC_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2952$cfg bench.py --gpus 2 --config $cfg --no-cpu --no-pmc \
    > gpurun_out/${TAG}_c${cfg}_gloo2.log 2> gpurun_out/${TAG}_c${cfg}_gloo2.err || { tail -20 gpurun_out/${TAG}_c${cfg}_gloo2.err; exit 1; }
  tail -c 700 gpurun_out/${TAG}_c${cfg}_gloo2.log; echo
done
