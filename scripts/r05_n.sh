#!/bin/bash
# Round-5: multi tests after the wait trims; config-3 compact locate shapes
# (threads x probes per thread) A/B against the in-tree build.
tag=${1:-r05n}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/${tag}_pytest.log 2>&1 || { tail -20 $out/${tag}_pytest.log; exit 1; }
tail -2 $out/${tag}_pytest.log
timeout -k 10 300 python -u bench.py --inproc 2 --steps 30 --no-api > $out/${tag}_inproc2.log 2> $out/${tag}_inproc2.err || exit 1
AB_DIR=comdb2_amd/lib/ab5 AB_ARGS="--config 3 --steps 20 --warmup 3 --no-cpu --no-pmc" ROUNDS=2 bash scripts/ab.sh
