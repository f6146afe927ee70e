#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench.  Each step has its own
# time limit; after a fault/abort/segfault/timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-smoke,pytest,bench}
[[ $STEPS == *smoke* ]] && { run smoke 420 python -c "import __graft_entry__ as g; g.smoke()" || exit $?; }
[[ $STEPS == *pytest* ]] && run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $STEPS == *bench* ]] && run bench 420 python bench.py ${BENCH_ARGS:-}
exit 0
