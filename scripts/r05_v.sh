#!/bin/bash
# Round-5: HIP API trace of the world-1 per-rank routed step (host gaps).
tag=${1:-r05v}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $out/${tag}_hip_rank1 -o k -- python3 bench.py --rank-path --steps 20 > $out/${tag}_hip_rank1.log 2> $out/${tag}_hip_rank1.err
echo rc=$?
