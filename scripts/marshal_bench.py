"""Host half of hip_serial_check_batch on config 2's 100k CurRangeArr* (the
bench's api leg): hsc_marshal_arrs on a host-only context, timed per call,
with 1 and with all host threads.  Runs on any machine (no GPU)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from comdb2_amd import hsc  # noqa: E402
from comdb2_amd.workloads import config2  # noqa: E402

c2 = config2(n_commits=20_000, n_txn=int(sys.argv[1]) if len(sys.argv) > 1 else 100_000,
             value_bits=40, build_log=True)
v = hsc.Validator(-1)
v.ingest_log(c2.log)
v.append_writes([])  # as the bench's device window: no DB_SET record rule
arrs = hsc.NativeCurRangeArrs(c2.readsets)
snaps = np.asarray(c2.readsets.snap, np.uint64)
want = v.marshal(c2.readsets)
got = v.marshal_arrs(arrs, snaps)
assert os.environ.get("HSC_LIB") or got["n"] == want["n"] and np.array_equal(got["lo"], want["lo"]) and \
    np.array_equal(got["txn"], want["txn"])
prev = v.batch_stats()
for th in (1, 0):
    v.set_threads(th)
    v.marshal_arrs(arrs, snaps, copy=False)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        v.marshal_arrs(arrs, snaps, copy=False)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    b0 = v.batch_stats()
    n = c2.readsets.ntxn
    print(f"threads {th or 'all'}: {t * 1e3:.2f} ms per {n} read sets = {n / t / 1e6:.2f} M/s, "
          f"{t / want['n'] * 1e9 * (os.cpu_count() if th == 0 else 1):.0f} ns per range per thread")
    k = b0["marshals"] - prev["marshals"]
    print("   per call ms:", {x: round((b0[x] - prev[x]) / k, 3) for x in ("parts_ns", "alloc_ns", "assemble_ns")})
    prev = b0
arrs.close()
v.close()
# the same read sets as flat arrays (hsc_marshal_readsets): no pointer walk
import ctypes as C  # noqa: E402
v = hsc.Validator(-1)
v.ingest_log(c2.log)
v.append_writes([])
s, keep = hsc.readsets_struct(c2.readsets)
mp = C.POINTER(hsc.Marshalled)()
for th in (1, 0):
    v.set_threads(th)
    v.lib.hsc_marshal_readsets(v.ctx, C.byref(s), C.byref(mp))
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        v.lib.hsc_marshal_readsets(v.ctx, C.byref(s), C.byref(mp))
        ts.append(time.perf_counter() - t0)
    print(f"flat, threads {th or 'all'}: {np.median(ts) * 1e3:.2f} ms")
v.close()
