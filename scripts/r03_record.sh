#!/bin/bash
# Round-3 record run (one GPU box): the GPU suite and smoke, kernel traces of
# the default bench on two streams and on one (rocprofv3 --kernel-trace
# --stats; overlap summaries), the default bench with its CPU baseline, PMC
# traffic passes and API leg, configs 3 and 5 with their CPU baselines and
# parity checks, config 1 with its fold legs.  Every GPU step has its own time
# limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r03r}
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${T}_$name.log" 2> "gpurun_out/${T}_$name.err"
  local rc=$?
  echo "== $name rc=$rc"
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/${T}_$name.err"; tail -5 "gpurun_out/${T}_$name.log"; exit $rc; }
  return 0
}
if [ -z "$NO_TESTS" ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  tail -1 gpurun_out/${T}_pytest_gpu.log
  run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
run kt2 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_kt2 -o run -- python3 bench.py --no-cpu --no-pmc --no-api --steps 20
python3 scripts/overlap.py ${T}_kt2 | head -12
run kt1 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_kt1 -o run -- python3 bench.py --no-cpu --no-pmc --no-api --steps 20 --streams 1
python3 scripts/overlap.py ${T}_kt1 | head -12
run bench 600 python3 bench.py
python3 scripts/benchsum.py gpurun_out/${T}_bench.log
run config3 600 python3 bench.py --config 3 --check
python3 scripts/benchsum.py gpurun_out/${T}_config3.log
run config5 700 python3 bench.py --config 5 --check
python3 scripts/benchsum.py gpurun_out/${T}_config5.log
run config1 400 python3 bench.py --config 1
# the N > 1 path rehearsed with two ranks on this one GPU (gloo barrier and
# max-over-ranks; the 8-GPU node runs are the driver's)
for cfg in 2 5; do
  HSC_BENCH_BACKEND=gloo run dist2_c$cfg 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config $cfg --no-cpu --no-pmc --no-api
  python3 scripts/benchsum.py gpurun_out/${T}_dist2_c$cfg.log
done
echo record done
