#!/bin/bash
# collector A/B: default, without the pre-lock assembly, without stream priorities
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/collector_ab.py > $out/r05h_default.log 2>&1 || exit $?
HSC_NO_PRE_ASSEMBLE=1 timeout -k 10 200 python -u scripts/collector_ab.py > $out/r05h_noasm.log 2>&1 || exit $?
HSC_NO_STREAM_PRIO=1 timeout -k 10 200 python -u scripts/collector_ab.py > $out/r05h_noprio.log 2>&1 || exit $?
HSC_NO_PRE_ASSEMBLE=1 HSC_NO_STREAM_PRIO=1 timeout -k 10 200 python -u scripts/collector_ab.py > $out/r05h_neither.log 2>&1 || exit $?
