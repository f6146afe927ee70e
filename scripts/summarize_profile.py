"""Summarize rocprofv3 output of scripts/profile.sh into profiles/.

  python scripts/summarize_profile.py TAG

reads gpurun_out/prof_TAG_{kt,fetch,write,sq}/ and writes
  profiles/TAG_kernel_stats.csv   (the --kernel-trace --stats summary)
  profiles/TAG_summary.md         (per-kernel avg time, HBM bytes, SQ counters)
  profiles/traffic.json           (HBM bytes per probe batch over the probe-phase
                                   kernels, read by bench.py as roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide (16 B/lane)
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024 (the join's
tile staging and record loads are 16-B-per-lane loads); WRITE_SIZE is exact
for 16-B-per-lane stores.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE_KERNELS = ("k_locate", "k_colscan", "k_plan", "k_scatter", "k_join", "k_pack")


def short(name):
    n = name.split("(")[0]
    n = n.replace("hsc::", "")
    return n.split("<")[0] + ("<" + n.split("<")[1] if "<" in n else "")


def counters(path):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main(tag):
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    kt = os.path.join(out, f"prof_{tag}_kt", "run_kernel_stats.csv")
    stats = list(csv.DictReader(open(kt)))
    shutil.copy(kt, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = counters(os.path.join(out, f"prof_{tag}_fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(out, f"prof_{tag}_write", "run_counter_collection.csv"))
    sq = counters(os.path.join(out, f"prof_{tag}_sq", "run_counter_collection.csv"))
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "Command: `scripts/profile.sh` passes over `python3 bench.py --steps 20 --warmup 3 "
             "--no-cpu` (config 2, 1 GPU).", "",
             "| kernel | calls | avg µs | HBM read MB (2×FETCH_SIZE) | HBM write MB | GB/s |",
             "|---|---|---|---|---|---|"]
    traffic = {"tag": tag, "kernels": {}, "probe_hbm_bytes_per_step": 0.0}
    for r in stats:
        k = short(r["Name"])
        avg_us = float(r["AverageNs"]) / 1e3
        f = fetch.get((k, "FETCH_SIZE"))
        w = write.get((k, "WRITE_SIZE"))
        rd = 2 * 1024 * sum(f) / len(f) if f else None
        wr = 1024 * sum(w) / len(w) if w else None
        gbs = ((rd or 0) + (wr or 0)) / (avg_us * 1e-6) / 1e9 if (rd or wr) else None
        fmt = lambda x: "" if x is None else f"{x / 1e6:.1f}"
        lines.append(f"| {k} | {r['Calls']} | {avg_us:.2f} | {fmt(rd)} | {fmt(wr)} | "
                     f"{'' if gbs is None else f'{gbs:.0f}'} |")
        if any(k.startswith(p) for p in PROBE_KERNELS) and rd is not None:
            traffic["kernels"][k] = {"read_bytes": rd, "write_bytes": wr, "avg_us": avg_us}
            traffic["probe_hbm_bytes_per_step"] += rd + (wr or 0)
    if sq:
        lines += ["", "SQ counters (per dispatch average):", "",
                  "| kernel | " + " | ".join(sorted({c for _, c in sq})) + " |",
                  "|---|" + "---|" * len({c for _, c in sq})]
        for k in sorted({k for k, _ in sq}):
            if not any(k.startswith(p) for p in PROBE_KERNELS):
                continue
            vals = [sq.get((k, c), [0]) for c in sorted({c for _, c in sq})]
            lines.append(f"| {k} | " + " | ".join(f"{sum(v) / len(v):.3g}" for v in vals) + " |")
    # wall time per batch over the densest run of probe dispatches (batches
    # on several streams overlap, so per-kernel averages above are inflated
    # and do not add up to the time per batch)
    trace = os.path.join(out, f"prof_{tag}_kt", "run_kernel_trace.csv")
    if os.path.exists(trace):
        import subprocess
        ov = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "overlap.py"),
                             f"prof_{tag}_kt"], capture_output=True, text=True).stdout
        lines += ["", "Probe-phase overlap (scripts/overlap.py over the kernel trace):", "",
                  "```", ov.rstrip(), "```"]
    open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    if traffic["kernels"]:
        json.dump(traffic, open(os.path.join(prof, "traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
