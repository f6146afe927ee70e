"""Summarise scripts/kt.sh output: per-kernel average duration (us) and, if a
PMC pass ran, per-kernel counter averages per dispatch."""
import collections, csv, os, sys
tag = sys.argv[1] if len(sys.argv) > 1 else "kt"
base = os.path.join(os.path.dirname(__file__), "..", "gpurun_out")
rows = list(csv.DictReader(open(os.path.join(base, tag, "run_kernel_stats.csv"))))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(f'{r["Name"][:40]:40s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.2f} us')
pmc = os.path.join(base, tag + "_pmc", "run_counter_collection.csv")
if os.path.exists(pmc):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(pmc)):
        agg[(r["Kernel_Name"].split("(")[0].replace("hsc::", "").split("<")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    cn = sorted({c for _, c in agg})
    print("kernel".ljust(22), *[c.replace("SQ_", "")[:14].rjust(14) for c in cn])
    for k in sorted({k for k, _ in agg}):
        if not any(x in k for x in ("_t", "colscan", "plan", "pack")):
            continue
        print(k[:22].ljust(22), *[("%.4g" % (sum(agg[(k, c)]) / len(agg[(k, c)]))).rjust(14) if agg[(k, c)] else "-".rjust(14) for c in cn])
