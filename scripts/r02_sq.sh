#!/bin/bash
# SQ counter passes over the probe kernels (bench.py --pmc-child: config-2
# window, batch 0 probed 10x on one stream).  One pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02sq}
mkdir -p gpurun_out
[ -n "$LIST" ] && { timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1; grep -c . gpurun_out/${TAG}_counters.txt; }
# counter sets: arguments, one quoted set each
[ $# -eq 0 ] && set -- "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d gpurun_out/prof_${TAG}_$i -o run -- python3 bench.py --pmc-child ${CHILD_ARGS:-} > gpurun_out/${TAG}_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_$i.log; exit 1; }
done
python3 - "$TAG" "$i" <<'PY'
import csv, sys, collections
tag, n = sys.argv[1], int(sys.argv[2])
agg = collections.defaultdict(list)
for k in range(1, n + 1):
    for r in csv.DictReader(open(f"gpurun_out/prof_{tag}_{k}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("hsc::", "").split("<")[0]
        agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in agg if k.startswith(("k_locate", "k_plan", "k_scatter", "k_join", "k_pack"))})
ctrs = sorted({c for _, c in agg})
print("kernel," + ",".join(ctrs))
for k in kern:
    print(k + "," + ",".join(f"{sum(agg.get((k, c), [0])) / max(1, len(agg.get((k, c), [0]))):.4g}" for c in ctrs))
PY
