#!/bin/bash
# Round-6: the narrow index built before the summaries, the window's tile
# maxima from its level-1 LSN maxima (A/B HSC_NTMAX_REBUILD=1: from the LSNs),
# the whole GPU suite, smoke, config 2 A/B, config 4, trace.
tag=${1:-r06be}
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/${tag}_$name.err; tail -25 $out/${tag}_$name.log; exit $rc; fi
}
step pytest 900 python -u -m pytest tests/ -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step c2 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_NTMAX_REBUILD=1 step c2reb 400 python -u bench.py --no-cpu --no-pmc --no-api
step c2b 400 python -u bench.py --no-cpu --no-pmc --no-api
HSC_NTMAX_REBUILD=1 step c2rebb 400 python -u bench.py --no-cpu --no-pmc --no-api
step default 600 python -u bench.py
step c4 500 python -u bench.py --config 4
step c2k 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_k -o k -- python3 bench.py --no-cpu --no-pmc --no-api --steps 2
for f in c2 c2reb c2b c2rebb default; do echo "$f $(python3 -c "
import json,sys
l=[x for x in open('$out/${tag}_$f.log') if x.startswith('{')][-1]; d=json.loads(l)
print(d.get('value'), d.get('ms_per_step'), d.get('ingest',{}).get('ms'), d.get('ingest',{}).get('GBps'))")"; done
