#!/bin/bash
# Round-4 evidence run: GPU suite, bench lines (default = config 2 with its
# PMC passes, configs 1, 3, 4, 5, the multi-GPU rehearsals), kernel traces of
# the default bench on two streams and on one, of config 3, and config 3's
# FETCH_SIZE / WRITE_SIZE passes kept as CSV.  Each step under its own time
# limit; stops at the first fault / abort / timeout (exit codes other than 0
# and 1).
tag=${1:-r04f}
part=${2:-all}  # a: suite + bench lines, b: multi-GPU rehearsals, traces, PMC
out=gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/${tag}_$name.log 2> $out/${tag}_$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/${tag}_$name.err; exit $rc; fi
}
if [ $part != b ]; then
step pytest 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread
tail -2 $out/${tag}_pytest.log
step bench 600 python -u bench.py
step config1 300 python -u bench.py --config 1
step config3 400 python -u bench.py --config 3
step config5 500 python -u bench.py --config 5
step config4 500 python -u bench.py --config 4
fi
[ $part = a ] && exit 0
step inproc2 300 python -u bench.py --inproc 2 --steps 30
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 step rank1 300 python -u bench.py --rank-path --steps 50
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_trace -o k -- python3 bench.py --steps 10 --no-cpu --no-pmc --no-api
step trace_s1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_s1 -o k -- python3 bench.py --steps 10 --streams 1 --no-cpu --no-pmc --no-api
step trace_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_c3trace -o k -- python3 bench.py --config 3 --steps 10 --no-cpu --no-pmc --no-api
step pmc_c3_fetch 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $out/${tag}_c3pmc_fetch -o run -- python3 bench.py --pmc-child --config 3
step pmc_c3_write 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $out/${tag}_c3pmc_write -o run -- python3 bench.py --pmc-child --config 3
