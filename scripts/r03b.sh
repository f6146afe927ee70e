#!/bin/bash
# Round-3 check: GPU suite, default bench (API leg: small-batch phases and the
# in-flight collector), config 1 (fold legs), config-5 A/B of the plan-free
# join, SQ counters of the one-stream probe kernels.  Every GPU step has its
# own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03b}
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2> "gpurun_out/${T}_$name.err"
  local rc=$?
  tail -c 600 "gpurun_out/${T}_$name.log"; echo; echo "== $name rc=$rc"
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/${T}_$name.err"; exit $rc; }
  return 0
}
if [ -z "$NO_TESTS" ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 500 python3 bench.py
run config1 400 python3 bench.py --config 1 --no-cpu
NO_TESTS=1 TAG=${T}_c5 CONFIG=5 AB="HSC_NT_FUSED=0 HSC_NT_FUSED=1" bash scripts/r03_ab.sh || exit $?
TAG=${T} PASSES=sq PROF_ARGS="--steps 20 --warmup 3 --no-cpu --no-api --no-pmc --streams 1" bash scripts/profile.sh || exit $?
echo r03b done
