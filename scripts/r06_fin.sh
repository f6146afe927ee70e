#!/bin/bash
# Round-6 closing run: full GPU suite, smoke, the default bench line (as the
# driver runs it) with its kernel trace, configs 3 / 5 (with the CPU
# sort-join parity) / 1 / 4, the 2-member in-process rehearsal, one-stream
# traces of configs 2 and 5.
tag=${1:-r06fin}
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
step default 600 python -u bench.py
step trace_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c2 -o k -- python3 bench.py --no-cpu --no-pmc --no-api
step trace_c2s1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c2s1 -o k -- python3 bench.py --no-cpu --no-pmc --no-api --streams 1
step c3 500 python -u bench.py --config 3 --check
step c5 600 python -u bench.py --config 5 --check
step trace_c5s1 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c5s1 -o k -- python3 bench.py --config 5 --no-cpu --no-pmc --no-api --streams 1
step c1 500 python -u bench.py --config 1
step c4 500 python -u bench.py --config 4
step inproc2 500 python -u bench.py --inproc 2 --steps 30
step trace_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace_c4 -o k -- python3 bench.py --config 4 --no-cpu --no-pmc --steps 3 --warmup 1
step inproc4q4 500 python -u bench.py --inproc 4 --steps 30 --no-cpu --no-pmc --no-api --hw-queues 4
