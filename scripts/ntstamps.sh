#!/bin/bash
# Narrow-tile locate / join phase stamps (diagnostic build lib/ab/stamps.so), config 2, one stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HSC_STAMPS=1 HSC_LIB=$PWD/comdb2_amd/lib/ab/stamps.so timeout -k 10 200 python3 bench.py --pmc-child > gpurun_out/ntstamps.log 2>&1 || { tail -5 gpurun_out/ntstamps.log; exit 1; }
grep stamps gpurun_out/ntstamps.log | tail -4
