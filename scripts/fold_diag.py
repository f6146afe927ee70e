"""Config-1 commit stream with small background folds: per-call times of the
checks and appends around the slow ones, with the library's fold trace
(HSC_FOLD_TRACE) on stderr stamped by the same steady clock."""
import gc
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ.setdefault("HSC_FOLD_TRACE", "1")


def main():
    import ctypes as C

    from comdb2_amd import formats as F
    from comdb2_amd import hsc
    from comdb2_amd.workloads import SEED_CONFIG1, config1_events
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    n_txn = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    ev = config1_events(seed=SEED_CONFIG1, n_txn=n_txn)
    v = hsc.Validator(0)
    v.set_fold(rows, background=True)
    lb = F.LogBuilder()
    v.ingest_log(lb.build())
    txns = {t.name: t for e, t in ev if e == "begin"}
    arrs = {nm: hsc.CurRangeArrays([t.reads], [0]) for nm, t in txns.items()}
    f, o = C.c_uint(), C.c_uint()
    check, append, ctx = v.lib.hip_bdb_osql_serial_check, v.lib.hsc_window_append_log, v.ctx
    nul = v.lib.hsc_window_delta_rows
    log = []
    gc.collect()
    gc.disable()
    k = 0
    for e, t in ev:
        if e == "begin":
            s = lb.next_lsn()
            a = arrs[t.name].arrs[0]
            a.file, a.offset = s >> 32, s & 0xFFFFFFFF
            continue
        if not t.writes:
            continue
        a = arrs[t.name].arrs[0]
        pa = C.cast(C.pointer(a), C.c_void_p)
        c0 = time.monotonic_ns()
        rc = check(ctx, pa, C.byref(f), C.byref(o), 0)
        c1 = time.monotonic_ns()
        log.append(("check", k, c0 / 1e3, (c1 - c0) / 1e3))
        if rc == 0:
            start = len(lb.rows)
            lb.begin(t.name)
            for rt, tb, ix, key in t.writes:
                lb.write(t.name, rt, tb, ix, key)
            lb.commit(t.name)
            st, keep = hsc.llog_struct(lb.build(start))
            c0 = time.monotonic_ns()
            append(ctx, C.byref(st))
            c1 = time.monotonic_ns()
            log.append(("append", k, c0 / 1e3, (c1 - c0) / 1e3))
        # host noise baseline: a native call that touches no GPU and no lock
        c0 = time.monotonic_ns()
        nul(ctx)
        c1 = time.monotonic_ns()
        log.append(("null", k, c0 / 1e3, (c1 - c0) / 1e3))
        k += 1
    gc.enable()
    print("fold stats", v.fold_stats(), file=sys.stderr)
    v.close()
    slow = [x for x in log if x[3] > 200 and x[1] > 0]
    for x in slow:
        print(f"[call] {x[2]:.0f} {x[0]} #{x[1]} {x[3]:.0f} us", file=sys.stderr)
    ch = np.array([x[3] for x in log if x[0] == "check"][1000:])
    ap = np.array([x[3] for x in log if x[0] == "append"])
    nu = np.array([x[3] for x in log if x[0] == "null"])
    print(f"null native call: p50 {np.median(nu):.2f} p99.9 {np.percentile(nu, 99.9):.1f} max {nu.max():.0f} us, "
          f"{int((nu > 100).sum())} calls over 100 us", file=sys.stderr)
    print(f"checks after 1000: p50 {np.median(ch):.1f} max {ch.max():.0f}; appends p50 {np.median(ap):.1f} "
          f"max {ap.max():.0f}", file=sys.stderr)


if __name__ == "__main__":
    main()
