#!/bin/bash
# GPU suite + smoke, then quick bench A/B runs of build knobs (no PMC, no CPU
# baseline, no API leg).  AB="HSC_NT_FUSED=0 HSC_NT_FUSED=1" names the
# environment settings; TAG names the outputs; CONFIG the bench config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
for kv in ${AB:-NONE=1}; do
  name=${kv//=/_}
  env $kv timeout -k 10 400 python3 bench.py --config ${CONFIG:-2} --no-cpu --no-api --no-pmc ${BENCH_ARGS:-} > gpurun_out/${TAG}_${name}.log 2> gpurun_out/${TAG}_${name}.err || { tail -20 gpurun_out/${TAG}_${name}.err; exit 1; }
  python3 scripts/benchsum.py gpurun_out/${TAG}_${name}.log
done
