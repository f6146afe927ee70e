#!/bin/bash
# pytest -m gpu, then bench (no CPU leg) narrow and wide.  Stops at the first
# fatal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} || exit $?
step bench_narrow 300 python bench.py --no-cpu ${BENCH_ARGS:-} || exit $?
[ -n "$NO_WIDE" ] || step bench_wide 300 python bench.py --no-cpu --wide ${BENCH_ARGS:-} || exit $?
exit 0
