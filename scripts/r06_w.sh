#!/bin/bash
# diagnostic: the config-2 window build with and without the unpack's LSN
# gather (timing only), kernel traces of both
tag=${1:-r06w}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_g -o k -- python3 bench.py --no-cpu --no-pmc --no-api --steps 2 > $out/${tag}_g.log 2>&1 || exit $?
HSC_DIAG_NO_LSN_GATHER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_ng -o k -- python3 bench.py --no-cpu --no-pmc --no-api --steps 2 > $out/${tag}_ng.log 2>&1 || exit $?
echo ok
