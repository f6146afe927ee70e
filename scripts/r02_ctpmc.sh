#!/bin/bash
# Config 3 (compact tiles) one-stream PMC passes + kernel trace of the probe kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ctpmc}
ARGS="--pmc-child --config 3 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt.log; exit 1; }
head -14 gpurun_out/${TAG}_kt/run_kernel_stats.csv | cut -d, -f1-4
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -T --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob, os
tag = os.environ.get("TAG", "ctpmc")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    if not any(x in k for x in ("locate", "scatter", "join", "plan", "bounds", "pack")):
        continue
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
