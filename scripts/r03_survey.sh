#!/bin/bash
# Round-3 survey on one box: config-2 A/B of the plan-free narrow join
# (HSC_NT_FUSED) with build-stage times, a one-stream kernel trace of the
# default path, then configs 3 and 5 with the compact plan-free join A/B.
# Every GPU step has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03s}
mkdir -p gpurun_out
HSC_BUILD_TRACE=1 NO_TESTS=1 TAG=${T}_c2 AB="HSC_NT_FUSED=0 HSC_NT_FUSED=1" bash scripts/r03_ab.sh || exit $?
grep -h "build us" gpurun_out/${T}_c2_*.err | head -4
TAG=${T}_kt STREAMS=1 bash scripts/r03_prof.sh || exit $?
NO_TESTS=1 TAG=${T}_c3 CONFIG=3 AB="HSC_CT_FUSED=0 HSC_CT_FUSED=1" bash scripts/r03_ab.sh || exit $?
NO_TESTS=1 TAG=${T}_c5 CONFIG=5 bash scripts/r03_ab.sh || exit $?
echo survey done
