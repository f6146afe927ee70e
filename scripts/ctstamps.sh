#!/bin/bash
# Compact-tile join phase stamps (diagnostic build lib/ab/stamps.so), config 3, one stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HSC_STAMPS=1 HSC_LIB=$PWD/comdb2_amd/lib/ab/stamps.so timeout -k 10 200 python3 bench.py --pmc-child --config 3 > gpurun_out/ctstamps.log 2>&1 || { tail -5 gpurun_out/ctstamps.log; exit 1; }
grep stamps gpurun_out/ctstamps.log | tail -4
