#!/bin/bash
# Round-6: graph build-path tests (txn-unsorted ops, bucket-line overflow,
# the fused id check) and the graph / graph_shard suites.
tag=${1:-r06v}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_graph.py tests/test_graph_shard.py -m gpu -q --timeout 300 --timeout-method thread > $out/${tag}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $out/${tag}_pytest.log
