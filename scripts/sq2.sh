cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -T --output-format csv -d gpurun_out/prof_sq2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/sq2.log 2>&1
echo rc=$?
