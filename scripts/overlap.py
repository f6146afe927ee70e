"""Overlap of the probe-phase kernels in a rocprofv3 kernel trace
(gpurun_out/TAG/run_kernel_trace.csv): for the densest run of probe kernels,
wall time, summed kernel time, per-kernel average and the time each kernel
spends alone vs. beside another probe kernel."""
import csv, os, sys, collections
tag = sys.argv[1] if len(sys.argv) > 1 else "kt"
path = os.path.join(os.path.dirname(__file__), "..", "gpurun_out", tag, "run_kernel_trace.csv")
PROBE = ("k_locate_t", "k_plan_t", "k_plan_s", "k_scatter_t", "k_join_t", "k_join_f", "k_pack_flags", "k_pack", "k_probe_delta")
rows = []
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].split("(")[0].replace("hsc::", "").split("<")[0]
    if n.startswith(("void ", )):
        n = n[5:]
    if n in PROBE:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
rows.sort()
# the timed loop: longest run of probe kernels with small gaps
best, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if b[0] - max(x[1] for x in cur) < 20000:
        cur.append(b)
    else:
        best = max(best, cur, key=len)
        cur = [b]
best = max(best, cur, key=len)
t0, t1 = best[0][0], max(x[1] for x in best)
print(f"dispatches {len(best)}  wall {(t1 - t0) / 1e3:.1f} us  queues {sorted({x[3] for x in best})}")
tot = collections.defaultdict(float); cnt = collections.Counter(); alone = collections.defaultdict(float)
events = []
for s, e, n, q in best:
    tot[n] += e - s; cnt[n] += 1
    events += [(s, 1, n), (e, -1, n)]
events.sort()
active = collections.Counter(); last = t0; busy = 0.0
for t, d, n in events:
    live = [k for k, v in active.items() if v > 0]
    if live:
        busy += t - last
        if sum(active.values()) == 1:
            alone[live[0]] += t - last
    active[n] += d
    last = t
print(f"busy {busy / 1e3:.1f} us ({100 * busy / (t1 - t0):.0f}% of wall), summed kernel time {sum(tot.values()) / 1e3:.1f} us")
for n in PROBE:
    if cnt[n]:
        print(f"  {n:14s} n={cnt[n]:4d} avg {tot[n] / cnt[n] / 1e3:6.2f} us  alone {100 * alone[n] / tot[n]:4.0f}%")
