#!/bin/bash
# Round-6: the graph_shard failure with and without the writer sort's txn
# skip; config-2 ingest trace (vary mask / unpack changes).
tag=${1:-r06i}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="tests/test_graph_shard.py::test_gpu_multi_graph_scc_matches_oracle"
HSC_GRAPH_NO_TXN_SKIP=1 timeout -k 10 200 python -u -m pytest "$T" -m gpu -q --timeout 120 --timeout-method thread > $out/${tag}_noskip.log 2>&1; echo "noskip rc=$?"; tail -3 $out/${tag}_noskip.log
timeout -k 10 200 python -u -m pytest "$T" -m gpu -q --timeout 120 --timeout-method thread > $out/${tag}_skip.log 2>&1; echo "skip rc=$?"; tail -3 $out/${tag}_skip.log
timeout -k 10 200 python -u -m pytest tests/test_graph.py -m gpu -q --timeout 120 --timeout-method thread > $out/${tag}_graph.log 2>&1; echo "graph rc=$?"; tail -3 $out/${tag}_graph.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c2 -o k -- python3 bench.py --no-cpu --no-pmc --no-api > $out/${tag}_c2.log 2>&1; echo "c2 rc=$?"
