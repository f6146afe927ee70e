#!/bin/bash
# rocprofv3 passes over the 1-GPU bench (run on the GPU box):
#   kt   : --kernel-trace --stats  (per-kernel durations)
#   fetch: --pmc FETCH_SIZE        (own pass; TCC slots)
#   write: --pmc WRITE_SIZE
# Outputs under gpurun_out/prof_<tag>_*; stops at the first fatal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:---steps 20 --warmup 3 --no-cpu --batches 2}
PASSES=${PASSES:-kt,fetch,write}
mkdir -p gpurun_out
run() {
  local name=$1; shift
  echo "== $name"
  timeout -k 10 300 "$@" > "gpurun_out/prof_${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/prof_${TAG}_${name}.log"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
[[ $PASSES == *kt* ]] && run kt rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_kt -o run -- python3 bench.py $ARGS
[[ $PASSES == *fetch* ]] && run fetch rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_${TAG}_fetch -o run -- python3 bench.py $ARGS
[[ $PASSES == *write* ]] && run write rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof_${TAG}_write -o run -- python3 bench.py $ARGS
[[ $PASSES == *sq* ]] && run sq rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES -T --output-format csv -d gpurun_out/prof_${TAG}_sq -o run -- python3 bench.py $ARGS
exit 0
