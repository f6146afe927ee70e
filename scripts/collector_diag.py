"""Diagnostic: the concurrent-caller legs of the bench's api section on a
config-2 window, each with the cgroup CPU statistics around it (cpu.stat:
periods, throttled periods, throttled time) and the caller-visible latency
percentiles -- to tell scheduler / quota stalls from collector waits.
usage: python scripts/collector_diag.py [n_commits] [threads ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (HIP initialised by torch first, as the bench does)

from comdb2_amd import hsc  # noqa: E402
from comdb2_amd.workloads import config2  # noqa: E402


def cpu_stat():
    out = {}
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            out[k] = int(v)
    except OSError:
        pass
    return out


def cpu_max():
    try:
        return open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        return "?"


n_commits = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
threads = [int(x) for x in sys.argv[2:]] or [1, 16, 64, 256]
c2 = config2(n_commits=n_commits, n_txn=100_000)
v = hsc.Validator(0)
v.ingest_log(c2.log)
arrs = hsc.NativeCurRangeArrs(c2.readsets)
want = v.check_readsets(c2.readsets) != 0
print(f"cpu.max {cpu_max()}  affinity {len(os.sched_getaffinity(0))}  nproc {os.cpu_count()}  "
      , flush=True)
for nth in threads:
    for inflight in [int(x) for x in os.environ.get("DIAG_INFLIGHT", "0").split(",")]:
        s0 = cpu_stat()
        t0 = time.perf_counter()
        got, st = v.concurrent_check(arrs, nth, inflight=inflight)
        el = time.perf_counter() - t0
        s1 = cpu_stat()
        d = {k: s1.get(k, 0) - s0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec",
                                                     "usage_usec", "user_usec", "system_usec")}
        keep = ("checks_per_s", "lat_p50_us", "lat_p99_us", "mean_batch", "device_pass_us",
                "busy_frac", "gate_us", "handout_us")
        print(f"threads {nth} inflight {inflight or 4}: parity {bool(np.array_equal(got != 0, want))} wall {el:.2f}s "
              f"cpu {d['usage_usec'] / 1e6 / max(el, 1e-9):.2f} cores "
              f"(user {d['user_usec'] / 1e6:.2f}s sys {d['system_usec'] / 1e6:.2f}s) "
              f"periods {d['nr_periods']} throttled {d['nr_throttled']} ({d['throttled_usec'] / 1e3:.1f} ms) | "
              + " ".join(f"{k} {st[k]:.1f}" if isinstance(st.get(k), float) else f"{k} {st.get(k)}"
                         for k in keep)
              + (" | small " + " ".join(f"{k} {v:.1f}" for k, v in st["small_path"].items()
                                       if isinstance(v, float)) if "small_path" in st else ""),
              flush=True)
arrs.close()
v.close()
