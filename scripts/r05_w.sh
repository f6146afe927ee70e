#!/bin/bash
# Round-5: world-1 per-rank step, bitmap variants: plan + join atomics
# (default), a guarded atomic (ab6/guard.so), the pack pass (HSC_PACK_PASS).
tag=${1:-r05w}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name env...
  local name=$1; shift
  env "$@" RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534 timeout -k 10 300 python -u bench.py --rank-path --steps 50 --no-api > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do
  run atomic_$r X=1
  run guard_$r HSC_LIB=$PWD/comdb2_amd/lib/ab6/guard.so
  run pack_$r HSC_PACK_PASS=1
done
