#!/bin/bash
# GPU suite; a kernel trace of a short default bench (build timeline); then
# A/B of the in-tree library against comdb2_amd/lib/abx/*.so on one and two
# streams.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03d}
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${T}_pytest_gpu.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_kt -o run -- python3 bench.py --no-cpu --no-pmc --no-api --steps 20 > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_kt.log
for r in 1 2; do
  for lib in cur comdb2_amd/lib/abx/*.so; do
    name=$(basename "$lib" .so)
    if [ "$lib" = cur ]; then env=""; else env="HSC_LIB=$PWD/$lib"; fi
    for st in 1 2; do
      env $env timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-api --streams $st > gpurun_out/${T}_ab_${name}_s${st}_$r.log 2>&1 || { tail -5 gpurun_out/${T}_ab_${name}_s${st}_$r.log; exit 1; }
      python3 scripts/benchsum.py gpurun_out/${T}_ab_${name}_s${st}_$r.log
    done
  done
done
echo r03d done
