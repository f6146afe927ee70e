#!/bin/bash
# Config-5 diagnosis: a one-stream kernel trace of the default config-5 bench
# and the narrow locate / join phase stamps (diagnostic build), then the same
# stamps for config 2 for comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03k}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_c5kt -o run -- python3 bench.py --config 5 --no-cpu --no-pmc --no-api --steps 20 --streams 1 > gpurun_out/${T}_c5kt.log 2>&1 || { tail -20 gpurun_out/${T}_c5kt.log; exit 1; }
head -12 gpurun_out/${T}_c5kt/run_kernel_stats.csv | cut -d, -f1-4
for c in 5 2; do
  HSC_STAMPS=1 HSC_LIB=$PWD/comdb2_amd/lib/abx/stamps.so timeout -k 10 300 python3 bench.py --config $c --pmc-child > gpurun_out/${T}_stamps_c$c.log 2>&1 || { tail -5 gpurun_out/${T}_stamps_c$c.log; exit 1; }
  grep stamps gpurun_out/${T}_stamps_c$c.log | tail -4
done
echo r03k done
