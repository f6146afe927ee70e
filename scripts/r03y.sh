#!/bin/bash
# Locate changes: narrow / full-config parity tests, locate phase stamps
# (configs 2 and 5, one stream), config 5 and config 2 benches.  Needs the
# diagnostic build first (here, on the CPU):
#   make -C comdb2_amd/csrc OUT=../lib/diag/stamps.so BUILD=build_stamps EXTRA=-DHSC_STAMPS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03y}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_full_configs.py tests/test_gpu_parity.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for c in 2 5; do
  HSC_STAMPS=1 HSC_LIB=$PWD/comdb2_amd/lib/diag/stamps.so timeout -k 10 300 python3 bench.py --config $c --pmc-child --streams 1 > gpurun_out/${T}_stamps_c$c.log 2>&1 || { tail gpurun_out/${T}_stamps_c$c.log; exit 1; }
  grep stamps gpurun_out/${T}_stamps_c$c.log | tail -2
done
timeout -k 10 600 python3 bench.py --config 5 --no-cpu --no-pmc --check > gpurun_out/${T}_c5.log 2> gpurun_out/${T}_c5.err || { tail gpurun_out/${T}_c5.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_c5.log
timeout -k 10 400 python3 bench.py --no-cpu --no-pmc --no-api > gpurun_out/${T}_c2.log 2> gpurun_out/${T}_c2.err || { tail gpurun_out/${T}_c2.err; exit 1; }
python3 scripts/benchsum.py gpurun_out/${T}_c2.log
echo r03y done
