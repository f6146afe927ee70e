#!/bin/bash
# Round-6: the pack as 512 resident workgroups striding over the tiles, one
# histogram flush each (A/B HSC_PACK_GRID=0: one workgroup per tile; 256),
# ingest + graph GPU tests, config 2 ingest, config 4, trace.
tag=${1:-r06bc}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest1 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_graph.py tests/test_graph_shard.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread
tail -2 $out/${tag}_pytest1.log
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_PACK_GRID=0 step c2old 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_PACK_GRID=256 step c2g256 400 python -u bench.py --no-cpu --no-pmc --no-api
step c2b 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_PACK_GRID=0 step c2oldb 400 python -u bench.py --no-cpu --no-pmc --no-api
step c4 400 python -u bench.py --config 4 --no-cpu --no-pmc
HSC_PACK_GRID=0 step c4old 400 python -u bench.py --config 4 --no-cpu --no-pmc
step c2k 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_k -o k -- python3 bench.py --no-cpu --no-pmc --no-api --steps 2
for f in c2 c2old c2g256 c2b c2oldb c4 c4old; do echo "$f $(python3 -c "
import json,sys
l=[x for x in open('$out/${tag}_$f.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d.get('ms_per_step'), d.get('ingest',{}).get('ms'), d.get('ingest',{}).get('GBps'))")"; done
