cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_sq3kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/sq3kt.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -T --output-format csv -d gpurun_out/prof_sq3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/sq3.log 2>&1
echo rc=$?
