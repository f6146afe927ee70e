"""bench.py -- serializable conflict checks/sec on MI355X (BASELINE.json config 2).

One step = one batch of read sets (config 2: 100k read sets x 10 ranges per
GPU) fully verdicted against the resident write window (1M commits x 10
int64 keys per GPU) by the HIP join.  Inputs are resident in HBM when the
timed region starts; marshalling (CurRangeArr -> probe SoA, done by the
native library) happens before it.

Multi-GPU (weak scaling, bench_multi): the native multi-GPU context
(hsc_multi_*; one process per GPU over RCCL under torchrun, or --gpus N
members in this process on devices 0..N-1): every GPU holds its piece of an
N-times larger window and owns 100k read sets of each global batch; the
ranges were routed to the pieces they overlap when the batch was marshalled,
and a step probes every piece and ORs the verdict bitmaps onto each read
set's owner (RCCL across ranks).  The device-routed step (routing +
exchange inside the timed region) is reported beside it.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "serializable conflict checks/sec at 1–8 GPUs, % HBM roofline, vs host CPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def upload_batch(torch, dev, m):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return dict(lo=t(m["lo"]), hi=t(m["hi"]), gid=t(m["gid"]), snap=t(m["snap"]),
                txn=t(m["txn"]), n=m["n"], lock_table=t(m["lock_table"]),
                lock_snap=t(m["lock_snap"]), lock_txn=t(m["lock_txn"]), n_lock=m["n_lock"],
                forced=m["forced"])


def probe_struct(hsc, b, verdict, bitmap, T):
    return hsc.ProbeBatch(b["n"], b["lo"].data_ptr(), b["hi"].data_ptr(), b["gid"].data_ptr(),
                          b["snap"].data_ptr(), b["txn"].data_ptr(), b["n_lock"],
                          b["lock_table"].data_ptr(), b["lock_snap"].data_ptr(),
                          b["lock_txn"].data_ptr(), T, verdict.data_ptr(),
                          bitmap.data_ptr() if bitmap is not None else None)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(log, readsets, gpu_verdict, threads, target_s, m0=None, window=None,
                 table_max=None, ngroups=1, log_note=""):
    """Oracle port of bdb_osql_serial_check (per-read-set log rescan, hash
    lookups, linear range scan, early exit) on a deterministic evenly spaced
    sample of the same batch, on `threads` pthreads and on one core; also
    checks those verdicts against the GPU's.  `log` may be a tail of the log
    that starts before the batch's oldest snapshot: a check only reads the
    records after its snapshot (bdb/serializable.c:390-539), so the tail gives
    the same verdicts and the same work.  With m0 (the marshalled batch) and
    window (gid, words, lsn rows) adds the build's own CPU sort-join over the
    full batch (SURVEY.md §8(d) second CPU line: same algorithm class as the
    GPU, on the host cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ol = oracle.OracleLog(log)
    T = readsets.ntxn

    def timed_sample(nthreads, budget_s):
        cal = np.arange(0, T, max(1, T // (8 * nthreads)))[: 8 * nthreads]
        _, _, secs = oracle.check(ol, readsets.subset(cal), nthreads=nthreads)
        rate = len(cal) / max(secs, 1e-6)
        n = int(min(T, max(len(cal), rate * budget_s)))
        sample = np.unique(np.linspace(0, T - 1, n).astype(np.int64))
        rc, _, secs = oracle.check(ol, readsets.subset(sample), nthreads=nthreads)
        ok = bool(np.array_equal(rc != 0, gpu_verdict[sample] != 0))
        return sample, secs, ok

    sample, secs, ok = timed_sample(threads, target_s)
    step = T / len(sample)
    out = dict(value=len(sample) / secs, unit="checks/s", cores=threads, kind="port",
               sample=f"{len(sample)} of {T} read sets (evenly spaced, 1 in {step:.1f}), "
                      f"oracle/serial_oracle.c restatement of bdb_osql_serial_check over the "
                      f"{log.nrec}-record log{log_note}, {threads} pthreads, {secs:.1f} s; "
                      f"cpu: {cpu_model()}",
               parity_with_gpu=ok)
    s1, secs1, ok1 = timed_sample(1, max(2.0, target_s / 3))
    out["single_core"] = dict(value=len(s1) / secs1, unit="checks/s", cores=1,
                              sample=f"{len(s1)} read sets, {secs1:.1f} s", parity_with_gpu=ok1)
    if m0 is not None and window is not None:
        gid, words, lsn = window
        sj = oracle.SortJoin(gid, words, lsn, ngroups)
        if table_max is None:
            table_max = np.array([lsn.max() if len(lsn) else 0], np.uint64)  # one table (t1)
        res = {}
        for nt in (threads, 1):
            verdict, secs_sj = sj.probe(m0, table_max, nthreads=nt)
            reps = max(1, int(min(target_s / 3, 10.0) / max(secs_sj, 1e-3)))
            tot = secs_sj
            for _ in range(reps - 1):
                _, s_ = sj.probe(m0, table_max, nthreads=nt)
                tot += s_
            res[nt] = (T * reps / tot, bool(np.array_equal(verdict != 0, gpu_verdict != 0)), reps)
        out["sortjoin"] = dict(
            value=res[threads][0], unit="checks/s", cores=threads, kind="build CPU sort-join",
            single_core=res[1][0], parity_with_gpu=res[threads][1] and res[1][1],
            sample=f"full batch ({T} read sets, {m0['n']} ranges), probe phase over a resident "
                   f"sorted window of {sj.rows} rows (window build {sj.build_s:.1f} s, not timed); "
                   f"oracle/sortjoin.c")
        sj.close()
    return out


def log_tail_commit(commit_lsn, snaps):
    """First commit of the log tail a batch's checks read: the commit whose
    regop is the oldest snapshot (or the one before it)."""
    s = int(np.min(snaps))
    c0 = int(np.searchsorted(commit_lsn, s))
    if c0 >= len(commit_lsn) or int(commit_lsn[c0]) != s:
        c0 = max(0, c0 - 1)
    return c0


def _native_stream(ev, v):
    """Replay a config-1 event stream through the drop-in entry of v, timing
    only the native calls: per commit one hip_bdb_osql_serial_check on a
    prebuilt CurRangeArr (snapshot = the log's end at the txn's begin) and,
    when it passes, one hsc_window_append_log of its records (the C struct
    built outside the timed call, as comdb2 hands it over).
    -> (check seconds[], append seconds[], {txn: rc}, wall seconds)."""
    import ctypes as C

    from comdb2_amd import formats as F
    from comdb2_amd import hsc
    lb = F.LogBuilder()
    v.ingest_log(lb.build())
    names = [t.name for e, t in ev if e == "begin"]
    txns = {t.name: t for e, t in ev if e == "begin"}
    arrs = {nm: hsc.CurRangeArrays([txns[nm].reads], [0]) for nm in names}
    f, o = C.c_uint(), C.c_uint()
    pf, po = C.byref(f), C.byref(o)
    check, append, ctx = v.lib.hip_bdb_osql_serial_check, v.lib.hsc_window_append_log, v.ctx
    t_check, t_app, rcs = [], [], {}
    # the collector would pause this loop at random calls (a gen-2 pass over
    # the log builder's rows takes milliseconds): off while the stream runs
    import gc
    gc.collect()
    gc.disable()
    t0 = time.perf_counter()
    for e, t in ev:
        if e == "begin":
            s = lb.next_lsn()
            a = arrs[t.name].arrs[0]
            a.file, a.offset = s >> 32, s & 0xFFFFFFFF
            continue
        if not t.writes:
            continue
        a = arrs[t.name].arrs[0]
        f.value, o.value = a.file, a.offset
        pa = C.cast(C.pointer(a), C.c_void_p)  # the call's arguments as comdb2 holds them
        c0 = time.perf_counter()
        rc = check(ctx, pa, pf, po, 0)
        t_check.append(time.perf_counter() - c0)
        rcs[t.name] = int(rc)
        if rc == 0:
            start = len(lb.rows)
            lb.begin(t.name)
            for rt, tb, ix, key in t.writes:
                lb.write(t.name, rt, tb, ix, key)
            lb.commit(t.name)
            part = lb.build(start)
            st, keep = hsc.llog_struct(part)  # the C struct, as comdb2 would hand it over
            pst = C.byref(st)
            c0 = time.perf_counter()
            rca = append(ctx, pst)
            t_app.append(time.perf_counter() - c0)
            if rca != 0:
                raise RuntimeError(f"hsc_window_append_log -> {rca}")
        del arrs[t.name]
    wall = time.perf_counter() - t0
    gc.enable()
    return np.array(t_check), np.array(t_app), rcs, wall


def _pct(x, slow_us=None):
    x = np.asarray(x) * 1e6
    out = {"mean": float(x.mean()), "p50": float(np.median(x)), "p99": float(np.percentile(x, 99)),
           "p999": float(np.percentile(x, 99.9)), "max": float(x.max()), "max_at": int(np.argmax(x))}
    if slow_us is not None:  # the calls above slow_us: (index, us), at most 20
        idx = np.nonzero(x > slow_us)[0]
        out["slow"] = [(int(i), round(float(x[i]), 1)) for i in idx[:20]]
        out["n_slow"] = int(len(idx))
    return out


def _commit_stream_fold_leg(ev, rows, background):
    """The stream with the delta run folded into the main window every `rows`
    rows (one keyed write per commit: about one fold per `rows` commits), in
    the background or inline, timed natively like the main leg."""
    from comdb2_amd import hsc
    v = hsc.Validator(0)
    if rows:
        v.set_fold(rows, background=background)
    tc, ta, rcs, wall = _native_stream(ev, v)
    st = v.fold_stats()
    v.close()
    w = min(1000, len(tc) // 10)  # the stream's start: the first write to the index builds the window
    return {"check_us": _pct(tc, slow_us=500), "append_us": _pct(ta, slow_us=500),
            "check_us_after_first_1000": _pct(tc[w:]), "folds": st,
            "value": len(tc) / (tc.sum() + ta.sum()), "unit": "commits/s", "checks": len(tc),
            "wall_s": wall}, rcs


def _protocol_leg(args, golden):
    """The master's commit protocol (db/toblock.c:4757-4836) replayed natively
    over the config-1 stream at 1 / 16 / 64 threads (hsc_harness_commit_protocol):
    per commit a regop_only probe under the commit_lock write lock, a full
    check outside it when newer commits exist (then the probe again), the
    writes appended under the lock.  Verdicts: 1 thread = the oracle replay's
    golden; every thread count checked by workloads.protocol_replay_check
    against oracle/serial_oracle.c on the log as it stood at each verdict."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    from comdb2_amd import formats as F
    from comdb2_amd import hsc
    from comdb2_amd.workloads import SEED_CONFIG1, config1_events, protocol_replay_check
    ev = config1_events(seed=SEED_CONFIG1, n_txn=args.n_txn_c1)
    txns = [t for e, t in ev if e == "begin"]
    out = {}
    for nth in (1, 16, 64):
        v = hsc.Validator(0)
        v.ingest_log(F.LogBuilder().build())
        e0 = v.end_lsn
        rc, seq, snap, cend, st = v.commit_protocol(txns, ev, nth)
        v.close()
        chk = protocol_replay_check(txns, rc, seq, snap, cend, e0,
                                    lambda log, rs: oracle.check(log, rs)[0])
        st["parity_with_oracle"] = chk["mismatches"] == 0
        st["oracle_checked"] = chk["checked"]
        st["not_serializable"] = int((rc != 0).sum())
        if nth == 1 and golden is not None:
            st["parity_with_oracle_golden"] = golden == {t.name: int(rc[i]) for i, t in enumerate(txns)
                                                          if t.writes}
        out[f"threads_{nth}"] = st
    out["note"] = ("commits_per_s = (commits + aborts) / wall time of the run; regop_* = the "
                   "regop_only probe under the write lock (answered from the context's published "
                   "snapshot: no collector queue, no context lock); hold_* = commit_lock write-held "
                   "time per commit; full_* = full checks (the context's collector batches "
                   "concurrent ones)")
    return out


def bench_commit_stream(args):
    """Config 1: the tests/tools/serial.c-shaped commit stream (10k txns, 20
    ids x 5 accounts, seed 0xC0FFEE01) replayed through the drop-in entry on
    one GPU with the window kept up to date incrementally: per commit one
    bdb_osql_serial_check (CurRangeArr, regop_only = 0) and, when it passes,
    its log records appended (hsc_window_append_log: decoded on the host,
    rows into the device delta run).  The reference path per commit is the
    same check + the txn's logging (db/toblock.c:4779-4836,
    bdb/tran.c:1545-1560).  Reports the stream rate and the per-call times of
    checks and appends; verdicts are compared with the oracle replay's golden
    (tests/golden/config1_replay.json).  `steady_state`: a 100k-txn stream of
    the same generator with the default fold threshold (32768 rows), so the
    window folds during the run, background vs inline folds (same verdicts)."""
    from comdb2_amd import hsc
    from comdb2_amd.workloads import SEED_CONFIG1, config1_events
    ev = config1_events(seed=SEED_CONFIG1, n_txn=args.n_txn_c1)
    v = hsc.Validator(0)
    tc, ta, rcs, wall = _native_stream(ev, v)
    layout = {hsc.LAYOUT_NARROW: "narrow", hsc.LAYOUT_COMPACT: "compact",
              hsc.LAYOUT_WIDE: "wide"}.get(v.layout, str(v.layout))
    small = v.small_stats()
    appends = v.append_stats()
    v.close()
    parity = None
    gpath = os.path.join(ROOT, "tests", "golden", "config1_replay.json")
    if os.path.exists(gpath) and args.n_txn_c1 == 10_000:
        parity = json.load(open(gpath))["rc"] == rcs
    native = tc.sum() + ta.sum()
    fb, rb = _commit_stream_fold_leg(ev, 1000, True)
    fi, ri = _commit_stream_fold_leg(ev, 1000, False)
    fb["parity_with_oracle_golden"] = parity is not None and rb == rcs and parity
    fi["parity_with_oracle_golden"] = parity is not None and ri == rcs and parity
    golden = json.load(open(gpath))["rc"] if os.path.exists(gpath) and args.n_txn_c1 == 10_000 else None
    protocol = _protocol_leg(args, golden)
    steady = None
    if args.c1_steady:
        ev2 = config1_events(seed=SEED_CONFIG1 + 1, n_txn=args.c1_steady)
        sb, rsb = _commit_stream_fold_leg(ev2, 0, True)      # default threshold, background
        si, rsi = _commit_stream_fold_leg(ev2, 32768, False)  # the same threshold, inline
        steady = {"txns": args.c1_steady, "fold_rows": 32768, "background": sb, "inline": si,
                  "verdicts_equal": rsb == rsi,
                  "not_serializable": int(sum(r != 0 for r in rsb.values())),
                  "note": "seed 0xC0FFEE02 stream of the config-1 generator; the default fold "
                          "threshold folds the delta run into the main window every 32768 "
                          "appended rows (two keyed rows per passing commit)"}
    out = {"metric": "commit-stream serializable checks/sec (drop-in entry + incremental window)",
           "value": len(tc) / native, "unit": "commits/s", "n_gpus": 1, "steps": len(tc),
           "warmup": 0, "ms_per_step": native / len(tc) * 1e3, "higher_is_better": True,
           "scaling": "none", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic config 1 stream (seed 0xC0FFEE01)",
           "window_layout": layout, "small_path": small, "append_path": appends,
           "config": {"workload": f"config1: {args.n_txn_c1} txns of tests/tools/serial.c shape, "
                                  "one check per commit, passing txns appended",
                      "checks": len(tc), "not_serializable": int(sum(r != 0 for r in rcs.values())),
                      "appends": len(ta)},
           "check_us": _pct(tc), "append_us_per_commit": _pct(ta),
           "stream_wall_s": wall, "parity_with_oracle_golden": parity,
           "cpu_baseline": None if args.no_cpu else commit_stream_cpu_baseline(args),
           "fold_every_1k_commits": {"background": fb, "inline": fi},
           "commit_protocol": protocol,
           "steady_state": steady,
           "note": "value = commits / (time inside the native check and append calls: "
                   "hip_bdb_osql_serial_check and hsc_window_append_log on prebuilt C structs); "
                   "the wall time also holds the Python log builder and struct marshalling that "
                   "stand in for comdb2's logging.  An append returns after its host decode "
                   "and the copy of its rows into the pending tail (mapped host memory the "
                   "next check's kernel scans); every 256 rows one merge launch moves the "
                   "tail into the device delta run"}
    print(json.dumps(out), flush=True)


def bench_graph(args):
    """Config 4: WR/WW/RW dependency graph + SCC of a Jepsen bank/register
    style history (SURVEY.md §8(a) A10, 100M ops by default), sharded by key
    over the ranks (comdb2_amd/shard.py sharded_scc): each rank builds the
    edges of its keys from device-resident ops, the ranks OR their covers
    (all_reduce MAX), all-gather the edges between covered txns and colour
    that graph.  Strong scaling: the history is fixed, value = its ops / the
    max-over-ranks wall time of one step (inputs resident in HBM)."""
    import torch
    import torch.distributed as dist

    from comdb2_amd import hsc, shard
    from comdb2_amd.workloads import config4_history
    world_env = max(1, int(os.environ.get("WORLD_SIZE", "1")))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("HSC_BENCH_BACKEND", "nccl")
    if world_env > 1 and args.gpus > 1 and args.gpus != world_env:
        print(f"bench.py --gpus {args.gpus} under WORLD_SIZE {world_env}", file=sys.stderr, flush=True)
        sys.exit(2)
    # without a launcher, --gpus N (devices 0..N-1) / --inproc N (the visible
    # GPUs round robin): N members of one in-process multi context
    devs = None
    if world_env == 1 and (args.gpus > 1 or args.inproc > 1):
        if backend != "nccl":
            print("bench.py --config 4 --gpus N: in-process members need the HIP path",
                  file=sys.stderr, flush=True)
            sys.exit(2)
        ndev = torch.cuda.device_count()
        if args.gpus > 1 and ndev < args.gpus:
            print(f"bench.py --gpus {args.gpus}: only {ndev} GPU(s) visible", file=sys.stderr, flush=True)
            sys.exit(2)
        devs = list(range(args.gpus)) if args.gpus > 1 else [i % ndev for i in range(args.inproc)]
    world = len(devs) if devs else world_env
    if backend != "nccl":
        local = 0
    if devs:
        local = devs[0]
    if args.pmc_child:  # one step of member 0's shard under rocprofv3 --pmc (graph_pmc_traffic)
        return graph_pmc_child(args)
    h = config4_history(n_txn=args.history_txns, n_keys=args.c4_keys or max(1000, args.history_txns // 10),
                        concurrent_frac=args.c4_concurrent, max_lag=args.c4_max_lag)
    traffic = None
    if rank == 0 and backend == "nccl" and not args.no_pmc:
        traffic = graph_pmc_traffic(args, h, world, local)  # before this process touches the GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world_env > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    hs = shard.history_shard(h, rank, world)
    dh = shard.device_history(hs, dev)
    dhs = [dh]
    if devs:  # every member's key shard on its device
        dhs += [shard.device_history(shard.history_shard(h, r, world), torch.device("cuda", devs[r]))
                for r in range(1, world)]
    native = backend == "nccl"  # the sharded step behind the C ABI (hsc_multi_graph_scc)
    if devs:
        mv = hsc.MultiValidator(devs)
    elif native and world > 1:
        ids = torch.zeros(hsc.MULTI_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            ids.copy_(torch.frombuffer(bytearray(hsc.MultiValidator.unique_ids()), dtype=torch.uint8))
        dist.broadcast(ids, 0)
        mv = hsc.MultiValidator(rank=rank, world=world, ids=bytes(ids.cpu().numpy().tobytes()),
                                device=local)
    elif native:
        mv = hsc.MultiValidator([local])
    else:
        mv = None
    v = mv.member(0) if mv is not None else hsc.Validator(local)
    g = shard.GpuGraph(v, dev)
    scc = torch.zeros(max(h.ntxn, 1), dtype=torch.int32, device=dev)

    def barrier():
        if world_env > 1:
            dist.barrier()

    def sync():
        for d in sorted(set(devs or [local])):
            torch.cuda.synchronize(d)

    ptrs = [scc.data_ptr()] + [None] * (len(dhs) - 1)
    times, st = [], None
    for k in range(args.warmup + args.steps):
        barrier()
        sync()
        t0 = time.perf_counter()
        if mv is not None:
            ss = mv.graph_scc(dhs, h.ntxn, ptrs)
            st = {"build": {"build_ms": ss["build_ms"]}, "scc": ss, "cut_rows": ss["edges"]}
        else:
            scc, st = shard.sharded_scc(g, dh, h.ntxn, dev)
        sync()
        dt = time.perf_counter() - t0
        barrier()
        if k >= args.warmup:
            times.append(dt)
    dt = torch.tensor([float(np.mean(times))], dtype=torch.float64,
                      device=dev if backend == "nccl" else "cpu")
    if world_env > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    ms = float(dt.item()) * 1e3
    out = None
    if rank == 0:
        # the unsharded call on the whole history must give the same components
        full, fst = v.dep_graph_scc(h)
        same = bool(np.array_equal(full, scc[:h.ntxn].cpu().numpy().astype(np.uint32)))
        # algorithmic bytes: every op's columns read once (txn u32, key u64,
        # is_write u8, observed u32 = 17 B) + per txn the cover byte and the
        # scc word written (5 B); the build's sorts come on top
        B4 = h.nops * 17 + h.ntxn * 5
        out = {"metric": "dependency-graph ops analysed/sec (WR/WW/RW edges + SCC)",
               "value": h.nops / (ms * 1e-3), "unit": "ops/s",
               "n_gpus": len(set(devs)) if devs else world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "u32/u64", "data": "synthetic config-4 history (seed 0xC0FFEE04)",
               "config": {"workload": f"config4: {h.ntxn} txns, {h.nops} ops, key shards x{world}",
                          "parallelism": f"key shards x{world} (cover all_reduce MAX + cut all_gather)",
                          "edges": fst["edges"], "ww": fst["ww"], "wr": fst["wr"], "rw": fst["rw"],
                          "nontrivial_sccs": st["scc"]["nontrivial_sccs"],
                          "txns_in_cycles": st["scc"]["txns_in_cycles"],
                          "cut_nodes": st["scc"]["cut_nodes"], "cut_rows": st["cut_rows"],
                          "rank0_ops": hs.nops, "rank0_build_ms": st["build"]["build_ms"],
                          "scc_cut_ms": st["scc"]["scc_ms"], "rounds": st["scc"]["rounds"],
                          "unsharded_build_ms": fst["build_ms"], "unsharded_scc_ms": fst["scc_ms"],
                          "parity_with_unsharded_gpu": same,
                          "members": world, "devices": devs or [local],
                          "path": ("hsc_multi_graph_scc (C ABI; in-process members: cover OR "
                                   "kernel + peer copies of the cuts)" if devs else
                                   "hsc_multi_graph_scc (C ABI; RCCL cover all-reduce + cut "
                                   "all-gather across ranks)" if mv is not None else
                                   "shard.sharded_scc over torch.distributed (" + backend + ")"),
                          "phase_ms": st["scc"].get("phase_ms") if mv is not None else None},
               "roofline": {"bound": "hbm", "kernel": "sharded SCC step (raw build: writer sort + "
                                                        "edge rows; cover; cut; colouring SCC)",
                            "achieved": B4 / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": B4 / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                            "traffic": traffic.get("bytes_per_step") if traffic else None,
                            "measured_frac": (traffic["bytes_per_step"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                              if traffic and traffic.get("bytes_per_step") else None),
                            "algorithmic_bytes": B4,
                            "note": "B = ops x 17 B (txn, key, is_write, observed read once) + "
                                    "txns x 5 B (cover byte, scc word); rank 0's step time.  "
                                    "traffic = FETCH_SIZE + WRITE_SIZE bytes of every hsc:: kernel "
                                    "of one step of member 0's shard (rocprofv3 --pmc passes of "
                                    "bench.py --config 4 --pmc-child; at N > 1 the SCC runs over "
                                    "that shard's cut only, not the union of the cuts)"}}
        if traffic:
            out["roofline"]["traffic_detail"] = traffic
    (mv if mv is not None else v).close()
    if world_env > 1:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        if not args.no_cpu:  # the host's throughput: the same line at every N
            out["cpu_baseline"] = graph_cpu_baseline(args)
        print(json.dumps(out), flush=True)


def graph_pmc_traffic(args, h, world, device):
    """HBM bytes of one config-4 step (member 0's key shard: raw build, cover,
    cut, colouring SCC) from rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes
    of `bench.py --config 4 --pmc-child` over the same history (saved for the
    child with numpy, no pickles), summed over every hsc:: kernel of the
    step; the gfx950 FETCH_SIZE correction as in pmc_traffic."""
    import csv
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="hsc_c4_")
    out = {"kind": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --config 4 "
                   "--pmc-child (one step of member 0's shard, every hsc:: kernel)", "kernels": {}}
    try:
        for k in ("txn", "key", "is_write", "observed"):
            np.save(os.path.join(d, k + ".npy"), getattr(h, k))
        per = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            od = os.path.join(d, "pmc_" + ctr)
            cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "-T", "--output-format",
                   "csv", "-d", od, "-o", "run", "--", sys.executable, os.path.abspath(__file__),
                   "--pmc-child", "--config", "4", "--c4-dir", d, "--c4-ntxn", str(h.ntxn),
                   "--c4-world", str(world), "--pmc-device", str(device)]
            env = {k: v for k, v in os.environ.items()
                   if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                                "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
            print(f"[bench] config-4 pmc pass {ctr}", file=sys.stderr, flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            path = os.path.join(od, "run_counter_collection.csv")
            if r.returncode != 0 or not os.path.exists(path):
                out["error"] = f"{ctr}: rc {r.returncode}: {(r.stderr or '')[-300:]}"
                return out
            vals = {}
            for row in csv.DictReader(open(path)):
                # (-T: truncated names, no namespace; every kernel of the library is k_*)
                name = row["Kernel_Name"]
                k = name.split("(")[0].replace("hsc::", "").replace("(anonymous namespace)::", "")
                k = (k[5:] if k.startswith("void ") else k).split("<")[0]
                if not k.startswith("k_") or row["Counter_Name"] != ctr:
                    continue
                vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
            per[ctr] = vals
        tot = 0.0
        for k in sorted(set(per["FETCH_SIZE"]) | set(per["WRITE_SIZE"])):
            rd, wr = 2 * 1024 * per["FETCH_SIZE"].get(k, 0.0), 1024 * per["WRITE_SIZE"].get(k, 0.0)
            out["kernels"][k] = {"read_bytes": rd, "write_bytes": wr}
            tot += rd + wr
        out["bytes_per_step"] = tot
    except (OSError, subprocess.SubprocessError) as e:
        out["error"] = str(e)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return out


def graph_pmc_child(args):
    """The profiled child of graph_pmc_traffic: member 0's shard of the saved
    history, one hsc_multi_graph_scc step on one GPU."""
    import torch

    from comdb2_amd import hsc, shard
    from comdb2_amd.workloads import History
    ld = lambda k: np.load(os.path.join(args.c4_dir, k + ".npy"))
    h = History(ld("txn"), ld("key"), ld("is_write"), ld("observed"), args.c4_ntxn)
    hs = shard.history_shard(h, 0, max(1, args.c4_world))
    torch.cuda.set_device(args.pmc_device)
    dev = torch.device("cuda", args.pmc_device)
    dh = shard.device_history(hs, dev)
    scc = torch.zeros(max(h.ntxn, 1), dtype=torch.int32, device=dev)
    mv = hsc.MultiValidator([args.pmc_device])
    torch.cuda.synchronize(dev)
    mv.graph_scc([dh], h.ntxn, [scc.data_ptr()])
    torch.cuda.synchronize(dev)
    mv.close()


def graph_cpu_baseline(args, threads=None):
    """oracle/scc_oracle.c (Adya edges + Tarjan) on histories of the same
    generator, sized to finish in seconds: one history on one core, and on
    every host CPU at once (one independent history per thread -- Tarjan is
    sequential, so the box's throughput is the per-core work side by side;
    ctypes drops the GIL inside the C calls)."""
    from concurrent.futures import ThreadPoolExecutor

    from comdb2_amd.workloads import config4_history
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = max(1000, min(args.history_txns, 1_000_000))
    mk = lambda seed: config4_history(seed=seed, n_txn=n, n_keys=args.c4_keys or max(1000, n // 10),
                                      concurrent_frac=args.c4_concurrent, max_lag=args.c4_max_lag)

    def run(h):
        t0 = time.perf_counter()
        s_, d_, _ = O.dep_edges(h.txn, h.key, h.is_write, h.observed)
        O.scc(h.ntxn, s_, d_)
        return h.nops, time.perf_counter() - t0
    h = mk(0xC0FFEE04)
    ops1, dt1 = run(h)
    threads = threads or box_cpus()["threads"]
    hs = [mk(0xC0FFEE04 + i) for i in range(threads)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(run, hs))
    wall = time.perf_counter() - t0
    tot = sum(r[0] for r in res)
    return {"value": tot / wall, "unit": "ops/s", "cores": threads, "kind": "port",
            "sample": f"{threads} independent histories of {n} txns (~{h.nops} ops each) of the "
                      f"config-4 generator, oracle/scc_oracle.c edges + Tarjan, one per thread, "
                      f"{wall:.1f} s wall; cpu: {cpu_model()}",
            "single_core": {"value": ops1 / dt1, "unit": "ops/s", "cores": 1,
                            "sample": f"{h.ntxn} txns / {ops1} ops, {dt1:.1f} s"}}


def commit_stream_cpu_baseline(args):
    """Config 1 on the host: the oracle (oracle/serial_oracle.c, the
    reference algorithm: per check a log rescan from the snapshot, chain walks,
    range scans) replayed over a bounded stream of the same generator -- each
    commit checked against the whole log so far, passing txns logged -- timing
    only the checks (the Python log builder stands in for comdb2's logging)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    from comdb2_amd.workloads import SEED_CONFIG1, config1_events, replay
    n = min(args.n_txn_c1, 2000)
    acc = [0.0, 0]

    def chk(log, rs):
        rc, _, secs = oracle.check(log, rs)
        acc[0] += secs
        acc[1] += 1
        return rc
    replay(config1_events(seed=SEED_CONFIG1, n_txn=n), chk)
    return {"value": acc[1] / acc[0], "unit": "commits/s", "cores": 1, "kind": "port",
            "sample": f"the first {n}-txn stream of the config-1 generator ({acc[1]} checks, "
                      f"{acc[0]:.2f} s inside the checks), one core: the reference checks one "
                      f"commit at a time under commit_lock (db/toblock.c:4757-4836); "
                      f"cpu: {cpu_model()}"}


def kernel_bytes(layout, W, n_keys, n_r, T, tm, WG=0, bitmap=False):
    """Per-kernel event times and each kernel's own algorithmic bytes (what it
    must read and write in this build's layout) for the probe phase.  Events
    add a few microseconds per slot; the rocprofv3 summaries in profiles/ give
    the undisturbed durations."""
    recs = tm["records"]
    tiles = tm["tiles"]
    chunk = 2048 if WG else 4096  # probes per locate workgroup
    chunks = (n_r + chunk - 1) // chunk
    hist = 4 * tiles * ((chunks + 7) // 8 * 8)
    if layout == 2:
        # narrow tiles, chunk-sorted records: the locate writes them in place
        # (+ its chunk's row of run starts / counts), no scatter pass
        own = {
            "k_locate_t": n_r * (4 + 8 + 4 + 16 * W) + 16 * recs + hist,
            "k_plan_s": hist + 6 * tiles * ((chunks + 7) // 8 * 8) + 2 * T,
            None: 0,
            "k_join_t": 8 * n_keys + 16 * recs + 6 * tiles * ((chunks + 7) // 8 * 8),
            "k_pack": (T + (T + 7) // 8) if bitmap else 0,
        }
    elif WG:
        # compact tiles, chunk-sorted 64-byte records written by the locate
        cols = 6 * tiles * ((chunks + 7) // 8 * 8)
        own = {
            "k_compact_bounds+k_locate_c": n_r * (4 + 8 + 4 + 16 * W) + 64 * recs + hist,
            "k_plan_s": hist + cols + 2 * T,
            None: 0,
            "k_join_c": n_keys * (8 * WG + 4) + 64 * recs + cols,
            "k_pack": (T + (T + 7) // 8) if bitmap else 0,
        }
    else:  # wide tiles (compact: W = code words): key words + lsn + gid per row
        own = {
            "k_locate": n_r * (4 + 8 + 16 * W) + 8 * n_r,
            "k_plan": 0,
            "k_scatter": n_r * (4 + 8 + 16 * W) + recs * 8 * (2 * W + 2),
            "k_join": n_keys * (8 * W + 12) + recs * 8 * (2 * W + 2),
            "k_pack": T + (T + 7) // 8,
        }
    ms = [tm["locate_ms"], tm["plan_ms"], tm["scatter_ms"], tm["join_ms"], tm["pack_ms"]]
    out = {}
    for (name, b), t in zip(own.items(), ms):
        if not name:  # no such pass in this layout
            continue
        out[name] = {"event_ms": t, "bytes": int(b),
                     "GBps": b / (t * 1e-3) / 1e9 if t > 0 else None}
    return out


def api_leg(hsc, v, rs, device_verdict, args):
    """The drop-in entry end to end: hip_serial_check_batch on the batch's
    read sets as CurRangeArr* (heap CurRange's with their own name and key
    allocations, as a comdb2 master holds them), each call = host marshal on
    the box's CPUs into pinned staging, upload, the join, verdict download and
    rc_out -- pipelined in 32k-read-set chunks (db/toblock.c:4779-4836 calls
    the check per transaction; a batching collector hands it n at once).
    Snapshots are passed as file/offset arrays (full mode overwrites them with
    the end LSN), one fresh pair per call, filled outside the timed region."""
    arrs = hsc.NativeCurRangeArrs(rs)
    T = rs.ntxn
    K = max(3, min(args.steps, 10))
    snaps = np.asarray(rs.snap, np.uint64)
    fo = [(np.ascontiguousarray(snaps >> np.uint64(32), np.uint32),
           np.ascontiguousarray(snaps & np.uint64(0xFFFFFFFF), np.uint32)) for _ in range(K + 1)]
    v.set_stream(0)  # the context's own stream
    rc = v.check_batch(arrs, file=fo[0][0], offset=fo[0][1])
    b0 = v.batch_stats()
    t0 = time.perf_counter()
    for k in range(K):
        v.check_batch(arrs, file=fo[k + 1][0], offset=fo[k + 1][1])
    el = time.perf_counter() - t0
    b1 = v.batch_stats()
    # phase split of a call (hsc_batch_stats: wall time of each phase summed
    # over the call's pipeline chunks; launch and wait overlap the next
    # chunk's marshal)
    phases = {k[:-3] + "_ms": (b1[k] - b0[k]) / K for k in b1 if k.endswith("_ns")}
    phases["ranges_per_call"] = (b1["ranges"] - b0["ranges"]) / K
    phases["chunks_per_call"] = (b1["marshals"] - b0["marshals"]) / K
    # the per-transaction call pattern: C threads each calling the one-set
    # entry (hsc_collector_check, bdb_osql_serial_check's signature) on their
    # share of the read sets; the collector batches whatever arrives together
    conc = {}
    want = np.asarray(device_verdict) != 0
    v.concurrent_check(arrs, 64)  # warm-up: the callers' threads, slots and staging
    for nth in (64, 256):
        runs = []
        for _ in range(3):  # the median run of three (run-to-run spread ~5 %)
            got, st = v.concurrent_check(arrs, nth)
            st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want))
            runs.append(st)
        runs.sort(key=lambda x: x["checks_per_s"])
        st = dict(runs[1])
        st["runs_checks_per_s"] = [r["checks_per_s"] for r in runs]
        st["parity_with_device_batch"] = all(r["parity_with_device_batch"] for r in runs)
        conc[f"threads_{nth}"] = st
    # passes in flight other than the default 4 (one run each)
    sweep = {}
    for inf in (2, 6, 8):
        got, s2 = v.concurrent_check(arrs, 64, inflight=inf)
        sweep[str(inf)] = {"checks_per_s": s2["checks_per_s"], "lat_p50_us": s2["lat_p50_us"],
                           "lat_p99_us": s2["lat_p99_us"], "mean_batch": s2.get("mean_batch"),
                           "parity_with_device_batch": bool(np.array_equal(got != 0, want))}
    conc["threads_64_inflight"] = sweep
    # one batch on the device at a time (the collector before round 3)
    got, st = v.concurrent_check(arrs, 64, inflight=1)
    st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want))
    conc["threads_64_inflight1"] = st
    # the plain drop-in entry (hip_bdb_osql_serial_check) from 64 threads: by
    # default it joins the context's own collector
    got, st = v.concurrent_check(arrs, 64, collect=False)
    st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want))
    st["entry"] = "hip_bdb_osql_serial_check (context-owned collector, the default)"
    conc["threads_64_dropin"] = st
    m = min(T, 2000)  # uncollected: one device pass per call, a bounded sample
    sub = hsc.NativeCurRangeArrs(_readsets_head(rs, m))
    got, st = v.concurrent_check(sub, 1, collect=False)  # a lone caller of the default entry
    st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want[:m]))
    st["sample"] = f"first {m} read sets"
    conc["threads_1_dropin"] = st
    v.set_autocollect(False)
    for nth in (1, 64):
        got, st = v.concurrent_check(sub, nth, collect=False)
        st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want[:m]))
        st["sample"] = f"first {m} read sets"
        conc[f"threads_{nth}_uncollected"] = st
    v.set_autocollect(True)
    sub.close()
    arrs.close()
    ok = bool(np.array_equal(rc != 0, want))
    return {"entry": "hip_serial_check_batch (CurRangeArr* x n, full checks)",
            "value": T * K / el, "unit": "checks/s", "calls": K, "read_sets_per_call": T,
            "ms_per_call": el / K * 1e3, "host_threads": box_cpus()["threads"],
            "phases": phases, "parity_with_device_batch": ok,
            "note": "marshal + pinned upload + probe + download + rc_out, timed over whole calls",
            "concurrent_callers": conc}


def _readsets_head(rs, m):
    """The first m read sets of rs (same key buffer)."""
    from comdb2_amd.formats import ReadSets
    e = int(rs.txn_off[m])
    return ReadSets(rs.txn_off[:m + 1], rs.snap[:m], rs.table[:e], rs.idxnum[:e],
                    rs.lflag[:e], rs.rflag[:e], rs.islocked[:e], rs.lkeylen[:e],
                    rs.rkeylen[:e], rs.lkey_off[:e], rs.rkey_off[:e], rs.keys, rs.tbnames)


def box_cpus():
    """The host CPUs this run may use: the affinity mask, the cgroup v2 CPU
    quota (a GPU box grants 16 CPUs of a larger machine) and nproc; the CPU
    baseline runs on min(affinity, quota) threads."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        nproc = None
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return dict(threads=threads, nproc=nproc, affinity_cpus=aff, cgroup_cpu_quota=quota,
                cpu=cpu_model())


PROBE_KERNELS = ("k_locate_t", "k_plan_s", "k_join_t", "k_pack_flags",  # narrow
                 "k_locate_c", "k_join_c",  # compact tiles
                 "k_compact_bounds", "k_locate", "k_colscan", "k_plan", "k_scatter", "k_join",
                 "k_pack", "k_probe_delta")  # compact / wide, delta run


def pmc_traffic(args, members=1, device=0):
    """HBM bytes per probe batch from rocprofv3 PMC passes of this same
    workload (`bench.py --pmc-child`: the window and the same ring of distinct
    batches as the timed loop, each probed once, rotating over the same
    streams; members > 1: `--multi-pmc`, the N-member partition on `device`
    with member 0 probing its routed share of two batches), one pass per
    counter as MI355X_MICROARCH.md
    prescribes (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2).  FETCH_SIZE /
    WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
    coalesced read, so read bytes = 2 x 1024 x FETCH_SIZE, write bytes = 1024 x
    WRITE_SIZE.  FETCH_SIZE counts Infinity-Cache hits too (L2 misses), so the
    figure is what the kernels pull from beyond L2.  Runs before this process
    touches the GPU."""
    import csv
    import shutil
    import tempfile
    out = {"kind": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --pmc-child "
                   "(same window, the timed loop's ring of batches and streams; per-kernel "
                   "means over the ring's launches)", "kernels": {}}
    per = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hsc_pmc_")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "-T", "--output-format",
               "csv", "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__),
               "--pmc-child", "--config", str(args.config), "--n-commits", str(args.n_commits),
               "--n-txn", str(args.n_txn), "--c3-writes", str(args.c3_writes),
               "--c5-keys", str(args.c5_keys), "--streams", str(args.streams), "--paths", str(args.paths)]
        cmd += (["--compact-wide"] if args.compact_wide else [])
        if members > 1:
            cmd += ["--multi-pmc", str(members), "--pmc-device", str(device), "--batches", "2",
                    "--ring-gb", "0"]
        else:
            cmd += ["--ring-gb", str(args.ring_gb)]
        # the child is a one-process run whatever launched this one
        env = {k: v for k, v in os.environ.items()
               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                            "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
        print(f"[bench] pmc pass {ctr}", file=sys.stderr, flush=True)
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            path = os.path.join(d, "run_counter_collection.csv")
            if r.returncode != 0 or not os.path.exists(path):
                out["error"] = f"{ctr}: rc {r.returncode}: {(r.stderr or '')[-300:]}"
                return out
            vals = {}
            for row in csv.DictReader(open(path)):
                k = row["Kernel_Name"].split("(")[0].replace("hsc::", "").split("<")[0]
                k = k[5:] if k.startswith("void ") else k
                if k in PROBE_KERNELS and row["Counter_Name"] == ctr:
                    vals.setdefault(k, []).append(float(row["Counter_Value"]))
            per[ctr] = {k: float(np.mean(v)) for k, v in vals.items()}
        except (OSError, subprocess.SubprocessError) as e:
            out["error"] = f"{ctr}: {e}"
            return out
        finally:
            shutil.rmtree(d, ignore_errors=True)
    tot = 0.0
    for k in PROBE_KERNELS:
        f, w = per["FETCH_SIZE"].get(k), per["WRITE_SIZE"].get(k)
        if f is None and w is None:
            continue
        rd, wr = 2 * 1024 * (f or 0.0), 1024 * (w or 0.0)
        out["kernels"][k] = {"read_bytes": rd, "write_bytes": wr}
        tot += rd + wr
    out["bytes_per_batch"] = tot
    return out


def bench_multi(args):
    """N > 1: the native multi-GPU context (include/hip_serial.h hsc_multi_*).
    Weak scaling: every member holds its piece of an N-times larger window
    (composite-key splitters: config 2 key ranges, config 5 sampled global
    splitters, config 3 work quantiles over the 32 groups' rows and ranges)
    and owns 100k read sets of each global batch (N x 100k read sets).

    Timed step (the headline): hsc_multi_probe_routed -- every member probes
    the ranges of the global batch that overlap its piece (routed on the host
    when the batch was marshalled: the drop-in path's routing),
    then the members' verdict bitmaps are OR-ed onto each read set's owner
    (RCCL send / receive of the owners' slices across ranks; peer reads in one
    process).  Secondary leg `device_routed`: the same global batch resident
    unrouted (each member its own 100k read sets) and routed inside the step
    (hsc_multi_probe_device: route kernels, exchange, probe, merge).

    Under torchrun: one process per GPU (RCCL).  Without it: `--gpus N` runs N
    members in this process on devices 0..N-1 (exits non-zero when fewer are
    visible); `--inproc N` is the rehearsal that lets members share a GPU."""
    import torch
    import torch.distributed as dist

    from comdb2_amd import hsc, shard
    from comdb2_amd.workloads import (SEED_CONFIG2, config2, config2_rank_window, config5_log,
                                      lsn_to_index)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --pmc-child --multi-pmc N: the rocprofv3 counter pass of member 0's
    # probes (pmc_traffic): N members in this process on one device, every
    # ring batch's routed share probed once by member 0
    pmc_child = bool(args.pmc_child and args.multi_pmc > 1)
    inproc = pmc_child or (world_env == 1 and not args.rank_path)
    traffic = None
    if inproc and not pmc_child:
        ndev = torch.cuda.device_count()  # (does not initialise the GPU on this image)
        N = args.gpus if args.gpus > 1 else args.inproc
        if args.gpus > 1 and ndev < N:
            print(f"bench.py --gpus {N}: only {ndev} GPU(s) visible", file=sys.stderr, flush=True)
            sys.exit(2)
    else:
        N = args.multi_pmc if pmc_child else world_env
    if (not pmc_child and not args.no_pmc and args.config in (2, 3) and (inproc or rank == 0)):
        # member 0's HBM bytes per step, before this process touches the GPU
        # (under torchrun the other ranks wait for rank 0 at the rendezvous)
        traffic = pmc_traffic(args, members=N, device=local if not inproc else 0)
    if pmc_child:
        devs = [args.pmc_device] * N
        v = hsc.MultiValidator(devs)
        mine = list(range(N))
        dev_of = {g: torch.device("cuda", devs[g]) for g in mine}
    elif inproc:
        ndev = torch.cuda.device_count()
        devs = list(range(N)) if args.gpus > 1 else [i % ndev for i in range(N)]
        v = hsc.MultiValidator(devs)
        mine = list(range(N))
        dev_of = {g: torch.device("cuda", devs[g]) for g in mine}
    else:
        N = world_env
        if args.gpus > 1 and args.gpus != N:
            print(f"bench.py --gpus {args.gpus} under WORLD_SIZE {N}", file=sys.stderr, flush=True)
            sys.exit(2)
        torch.cuda.set_device(local)
        dev0 = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=dev0)
        ids = torch.zeros(hsc.MULTI_ID_BYTES, dtype=torch.uint8, device=dev0)
        if rank == 0:
            ids.copy_(torch.frombuffer(bytearray(hsc.MultiValidator.unique_ids()), dtype=torch.uint8))
        dist.broadcast(ids, 0)
        v = hsc.MultiValidator(rank=rank, world=N, ids=bytes(ids.cpu().numpy().tobytes()),
                               device=local)
        mine = [rank]
        dev_of = {rank: dev0}
        devs = [local]
    if args.loopback and inproc:
        v.set_transport(True)

    def sync_all():
        for d in sorted(set(dev_of[g].index for g in mine)):
            torch.cuda.synchronize(d)

    T = args.n_txn
    rows = {}  # member -> (gid, words, lsn)
    seg_vals = {}  # member -> its written int64 values in its commit order (configs 2 / 5: the log)
    if args.config == 2:
        value_bits = 40
        assert v.register_group("t1", 0, 9) == 0
        c2 = config2(seed=SEED_CONFIG2, n_commits=args.n_commits, n_txn=T, rank=mine[0], world=N,
                     build_log=False)
        end_lsn = c2.params["end_lsn"]
        first_rs = c2.readsets
        c2 = None
        for g in mine:  # (the same rows as config2(rank=g), without its read sets)
            gid_, words_, lsn_, seg_vals[g] = config2_rank_window(SEED_CONFIG2, args.n_commits, g, N)
            rows[g] = (gid_, words_, lsn_)
        more_rs = lambda bi: config2(seed=SEED_CONFIG2 + 7919 * bi, n_commits=args.n_commits,
                                     n_txn=T, rank=0, world=N, build_log=False).readsets
        sp_g, sp_w = shard.int64_splitter_keys([j << value_bits for j in range(1, N)], 2)
        workload = (f"config2 x{N}: per member 100k read sets x 10 ranges vs its key-range piece "
                    f"of an {N}x window (1M commits x 10 int64 keys per member), one index")
        data = "synthetic (BASELINE config 2 generator, seed 0xC0FFEE02, weak scaling per member)"
        groups = [("t1", 0, 9)]
    elif args.config == 5:
        from comdb2_amd.workloads import SEED_CONFIG5, config5_scaled, int64_words
        assert v.register_group("t1", 0, 9) == 0
        segs = {}
        for g in mine:
            c5 = config5_scaled(seed=SEED_CONFIG5, keys_per_gpu=args.c5_keys, n_txn=T, rank=g,
                                world=N)
            segs[g] = (c5.keys, c5.lsn)
            seg_vals[g] = c5.keys
            end_lsn = c5.end_lsn
            first_rs = c5.readsets
            range_keys = c5.range_keys
        if inproc:
            allk = np.concatenate([segs[g][0] for g in mine])
            alll = np.concatenate([segs[g][1] for g in mine])
            split = shard.sampled_splitters(allk, range_keys, N, 0, shard.ROW_COST,
                                            shard.RANGE_COST)["splitters"]
            own = np.searchsorted(split, allk, side="right")
            for g in mine:
                sel = own == g
                k = allk[sel]
                rows[g] = (np.zeros(len(k), np.uint32), int64_words(k), alll[sel])
        else:
            k, l = segs[rank]
            split = shard.sampled_splitters(k, range_keys, N, rank, shard.ROW_COST,
                                            shard.RANGE_COST)["splitters"]
            k, l = shard.exchange_rows(k, l, split)
            rows[rank] = (np.zeros(len(k), np.uint32), int64_words(k), l)
        segs = None
        more_rs = lambda bi: config5_scaled(seed=SEED_CONFIG5 + 7919 * bi, keys_per_gpu=args.c5_keys,
                                            n_txn=T, rank=0, world=N, window=False).readsets
        sp_g, sp_w = shard.int64_splitter_keys(split, 2)
        workload = (f"config5 x{N}: one global Zipf(1.2) law over 2^32 keys, {args.c5_keys} logged "
                    f"writes per member, sampled global splitters, 100k read sets x 10 ranges "
                    f"per member")
        data = "synthetic (config 5 generator, seed 0xC0FFEE05, weak scaling per member)"
        groups = [("t1", 0, 9)]
    else:
        from comdb2_amd.workloads import SEED_CONFIG3, config3_arrays
        c3 = config3_arrays(seed=SEED_CONFIG3, n_writes=args.c3_writes * N, n_txn=T * N)
        for g, (tbn, ix, L) in enumerate(c3.groups):
            assert v.register_group(tbn, ix, L) == g
        gid, words, lsn = c3.window()
        hv = hsc.Validator(-1)
        for (tbn, ix, L) in c3.groups:
            hv.register_group(tbn, ix, L)
        hv.set_end(c3.end_lsn)
        sp_g, sp_w = shard.composite_splitters(gid, words, N, hv.marshal(c3.readsets))
        hv.close()
        own = shard.composite_owner(gid, words, sp_g, sp_w)
        for g in mine:
            sel = own == g
            rows[g] = (gid[sel], np.ascontiguousarray(words[:, sel]), lsn[sel])
        end_lsn = c3.end_lsn
        first_rs = c3.readsets
        more_rs = lambda bi: config3_arrays(seed=SEED_CONFIG3, n_writes=args.c3_writes * N,
                                            n_txn=T * N, rs_seed=bi).readsets
        workload = (f"config3 x{N}: {len(c3.groups)} (table, index) groups of composite keys "
                    f"(9-64 B), {args.c3_writes} index writes and {T} read sets per member, "
                    f"composite-key pieces at work quantiles (hot groups cut)")
        data = "synthetic (config 3 generator, seed 0xC0FFEE03, weak scaling per member)"
        groups = c3.groups
    # the CPU baseline's log (rank 0): every record after the oldest snapshot
    # of owner 0's read sets -- configs 2 / 5: the members' writes from local
    # commit c_start on, gathered across ranks (config 3: the global arrays)
    want_cpu = not args.no_cpu and not pmc_child
    tails, c_start = None, 0
    if want_cpu and args.config in (2, 5):
        K5 = 10
        snap0 = np.asarray(first_rs.snap[:T], np.uint64)
        gc0 = int((int(lsn_to_index(snap0.min())) - (K5 + 2)) // (K5 + 3))  # its regop's commit
        c_start = max(0, gc0) // N
        mine_tail = {g: np.ascontiguousarray(seg_vals[g][c_start * K5:]) for g in mine}
        if inproc:
            tails = [mine_tail[g] for g in range(N)]
        else:
            tails = [None] * N
            dist.all_gather_object(tails, mine_tail[rank])
    seg_vals = None
    v.set_splitters(sp_g, sp_w)
    for i, g in enumerate(mine):
        gid, words, lsn = rows[g]
        d = dev_of[g]
        tg = torch.from_numpy(np.ascontiguousarray(gid)).to(d)
        tw = torch.from_numpy(np.ascontiguousarray(words).reshape(-1).view(np.int64)).to(d)
        tl = torch.from_numpy(np.ascontiguousarray(lsn).view(np.int64)).to(d)
        sync_all()
        v.member(i).ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(),
                                  tl.data_ptr(), end_lsn)
        del tg, tw, tl
    n_w = {g: len(rows[g][2]) for g in mine}
    # the replicated drop-in leg (in process, config 2): every member holds
    # the whole global window
    rows_all = ([rows[g] for g in mine] if inproc and not pmc_child and args.config == 2
                and not args.no_api else None)
    rows = None
    v.adopt()
    if args.config == 3:
        v.merge_table_max(c3.table_max)  # data-row writes lock tables too
    W = v.words
    TP = (T + 63) // 64 * 64  # each owner's read sets start at a multiple of 64
    # resident batches, per member: `routed` = its ranges of the whole global
    # batch (routed at marshal), `dev` = its own 100k read sets unrouted
    batches, ring_bytes, bi = [], 0, 0
    t_setup = time.perf_counter()
    while bi < max(2, args.batches) or ring_bytes < args.ring_gb * 1e9:
        rs = first_rs if bi == 0 else more_rs(bi)
        shares = [rs.subset(np.arange(g * T, (g + 1) * T)) for g in range(N)]
        routed = v.routed_shares(shares, mine)
        per = {}
        for li, g in enumerate(mine):
            dv = dev_of[g]
            r = routed[g]
            b = upload_batch(torch, dv, r)
            b["bits"] = torch.zeros(TP // 64, dtype=torch.int64, device=dv)
            b["verdict"] = torch.zeros(N * TP, dtype=torch.uint8, device=dv)
            b["struct"] = hsc.ProbeBatch(b["n"], b["lo"].data_ptr(), b["hi"].data_ptr(),
                                         b["gid"].data_ptr(), b["snap"].data_ptr(),
                                         b["txn"].data_ptr(), b["n_lock"],
                                         b["lock_table"].data_ptr(), b["lock_snap"].data_ptr(),
                                         b["lock_txn"].data_ptr(), N * TP,
                                         b["verdict"].data_ptr(), b["bits"].data_ptr())
            b["owner_base"] = r["owner_base"]
            b["forced"] = r["forced"][g]
            b["bytes"] = sum(int(b[k].numel() * b[k].element_size())
                             for k in ("lo", "hi", "gid", "snap", "txn", "lock_table", "lock_snap",
                                       "lock_txn"))
            if pmc_child:
                per[g] = {"routed": b}
                continue
            m = v.marshal(shares[g])
            d = upload_batch(torch, dv, m)
            d["bits"] = torch.zeros((T + 63) // 64, dtype=torch.int64, device=dv)
            d["verdict"] = torch.zeros(T, dtype=torch.uint8, device=dv)
            d["struct"] = probe_struct(hsc, d, d["verdict"], d["bits"], T)
            per[g] = {"routed": b, "dev": d}
        ring_bytes += per[mine[0]]["routed"]["bytes"]
        batches.append(per)
        bi += 1
        if bi % 8 == 0:
            print(f"[bench] {bi} batches, {ring_bytes / 1e9:.2f} GB per member", file=sys.stderr,
                  flush=True)
    setup_s = time.perf_counter() - t_setup
    NB = len(batches)
    ob = batches[0][mine[0]]["routed"]["owner_base"]
    sync_all()
    if pmc_child:
        # counted by the parent's rocprofv3 --pmc pass: member 0 probes its
        # routed share of every ring batch once (the kernels of its step's probe)
        m0 = v.member(0)
        for i in range(NB):
            b = batches[i][0]["routed"]
            m0.probe_device(probe_struct(hsc, b, b["verdict"], None, N * TP))
        m0.synchronize()
        v.close()
        return

    # each batch's call arguments built once: a step is one foreign call (the
    # Python list + ctypes array per call cost ~30 us, more than the C enqueue)
    prep_routed = [v.prepare_routed([batches[i][g]["routed"]["struct"] for g in mine], ob)
                   for i in range(NB)]
    prep_dev = [v.prepare_device([batches[i][g]["dev"]["struct"] for g in mine]) for i in range(NB)]

    def step_routed(k, lanes, nbatch):
        v.probe_routed_prepared(prep_routed[k % nbatch], k % lanes)

    def step_device(k, lanes, nbatch):
        v.probe_device_prepared(prep_dev[k % nbatch], k % lanes)

    def timed(step, lanes, nbatch):
        for k in range(args.warmup):
            step(k, lanes, nbatch)
        sync_all()
        if not inproc:
            dist.barrier()
        sync_all()
        t0 = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            step(k, lanes, nbatch)
        sync_all()
        if not inproc:
            dist.barrier()
        sync_all()
        el = time.perf_counter() - t0
        if not inproc:
            e = torch.tensor([el], dtype=torch.float64, device=dev_of[rank])
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el

    elapsed = timed(step_routed, 2, NB)
    serial = float(np.median([timed(step_routed, 1, NB) for _ in range(3)]))
    dev_elapsed = timed(step_device, 2, NB)
    dev_serial = float(np.median([timed(step_device, 1, NB) for _ in range(3)]))
    # merged verdicts of batch 0, member mine[0]'s read sets, both routings
    g0 = mine[0]
    step_device(0, 1, NB)
    sync_all()
    d0 = batches[0][g0]["dev"]
    dbits = np.unpackbits(d0["bits"].cpu().numpy().view(np.uint8), bitorder="little")[:T]
    step_routed(0, 1, NB)
    sync_all()
    r0 = batches[0][g0]["routed"]
    rbits = np.unpackbits(r0["bits"].cpu().numpy().view(np.uint8), bitorder="little")[:T]
    v0 = np.maximum(rbits, r0["forced"])
    routings_equal = bool(np.array_equal(np.maximum(dbits, d0["forced"]) != 0, v0 != 0))
    # the routed step's host cost: its phases over the timed legs, and the
    # pure enqueue -- calls that start on an idle GPU (no queue backpressure)
    rps = v.routed_phase_stats()
    idle = []
    for k in range(min(max(args.steps, 5), NB)):
        sync_all()
        t0 = time.perf_counter()
        step_routed(k, 1, NB)
        idle.append(time.perf_counter() - t0)
    sync_all()
    # per-member probe time of the routed step (imbalance across the pieces)
    v.enable_member_timing(True)
    pm = []
    for k in range(min(args.steps, NB)):
        step_routed(k, 1, NB)
        pm.append(v.member_probe_ms())
    v.enable_member_timing(False)
    sync_all()
    pm = np.mean(np.array(pm, np.float64), axis=0)
    if not inproc:
        t = torch.tensor(pm, dtype=torch.float64, device=dev_of[rank])
        allt = [torch.zeros_like(t) for _ in range(N)]
        dist.all_gather(allt, t)
        pm = torch.cat(allt).cpu().numpy()
    cnt = v.last_counts().astype(np.int64)
    n_keys = v.member(0).keys
    n_r = int(r0["n"])
    Lhat = 8 * W
    B = n_keys * (Lhat + 12) + n_r * (2 * Lhat + 16) + (N * T + 7) // 8
    ms = elapsed / args.steps * 1e3
    rec = 16 * W + 16
    off_diag = int(cnt.sum() - np.trace(cnt))
    routed_rows = [int(batches[0][g]["routed"]["n"]) for g in mine]
    own_rows = [int(batches[0][g]["dev"]["n"]) for g in mine]
    out = {
        "metric": METRIC,
        "value": N * T * args.steps / elapsed,
        "unit": "checks/s",
        "n_gpus": len(set(devs)) if inproc else N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": data,
        "config": {
            "workload": workload,
            "members": N,
            "devices": devs,
            "transport": ("in-process (xGMI peer reads / same GPU)" + (", loopback copies" if args.loopback else ""))
                         if inproc else "RCCL (C, grouped send/recv)",
            "read_sets_per_step_per_member": T,
            "ranges_routed_to_member0": n_r,
            "window_keys_member0": n_keys,
            "logged_writes_per_member": n_w,
            "parallelism": f"composite-key pieces x{N}: ranges routed to the pieces they overlap "
                           "at marshal time (host), probe + bitmap OR per owner in the timed step",
            "lanes": 2,
            "serial_ms_per_step": serial / args.steps * 1e3,
            "ring_batches": NB,
            "setup_s": setup_s,
            "groups": len(groups),
            "conflict_rate": float((v0 != 0).mean()),
        },
        "routing": {
            "mode": "host, at marshal (hsc_multi_marshal_routed; not in the timed step, like the "
                    "marshal itself)",
            "routed_rows_per_member_batch0": routed_rows,
            "own_rows_per_member_batch0": own_rows,
            "routed_over_own": float(sum(routed_rows)) / max(1, sum(own_rows)),
            "verdicts_equal_device_routed": routings_equal,
            "host_enqueue_us_per_step": v.phase_stats()["routed_enqueue_us"],
            "host_phases_us_per_step": rps,
            "host_enqueue_idle_us": {"p50": float(np.median(idle) * 1e6), "min": float(np.min(idle) * 1e6),
                                     "per_member_p50": float(np.median(idle) * 1e6) / max(1, len(mine)),
                                     "note": "hsc_multi_probe_routed calls that start on an idle GPU "
                                             "(no queue backpressure): the pure host enqueue"},
        },
        "imbalance": {
            "member_probe_ms": [float(x) for x in pm],
            "max_over_mean": float(pm.max() / pm.mean()) if pm.size and pm.mean() > 0 else None,
        },
        "device_routed": {
            "value": N * T * args.steps / dev_elapsed,
            "ms_per_step": dev_elapsed / args.steps * 1e3,
            "serial_ms_per_step": dev_serial / args.steps * 1e3,
            "counts_last_batch": cnt.tolist(),
            "exchanged_bytes_per_step": off_diag * rec,
            "host_phases_us": v.phase_stats(),
            "note": "the same global batch resident unrouted (member g: its own 100k read sets); "
                    "the step routes on the devices (k_route_count / k_route_scatter), exchanges "
                    "(RCCL or in-process stores), probes and merges",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "routed step per member (probe phase of its routed ranges + OR merge)",
            "achieved": B / (ms * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": B / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frac_1lane": B / (serial / args.steps) / 1e9 / HBM_PEAK_GBS,
            "traffic": traffic.get("bytes_per_batch") if traffic else None,
            "measured_frac": (traffic["bytes_per_batch"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                              if traffic and traffic.get("bytes_per_batch") else None),
            "algorithmic_bytes": B,
            "note": "B = member 0's probe-phase bytes (SURVEY 8(d): its window keys, the ranges "
                    "routed to it, the global batch's verdict bits); with members sharing a GPU "
                    "(--inproc rehearsal) the GPU runs every member's B in one step.  traffic = "
                    "member 0's probe kernels' FETCH_SIZE + WRITE_SIZE bytes per batch "
                    "(rocprofv3 --pmc passes of bench.py --pmc-child --multi-pmc N: the same "
                    "partition, member 0 probing its routed share of each batch)",
        },
        "cpu_baseline": None,
    }
    if traffic:
        out["roofline"]["traffic_detail"] = traffic
    if inproc and args.config == 2 and not args.no_api:
        out["api"] = multi_api_leg(hsc, v, first_rs.subset(np.arange(0, T)), v0)
        v.close()
        out["api_replicas"] = replicas_api_leg(hsc, torch, devs, rows_all, end_lsn,
                                               first_rs.subset(np.arange(0, T)), v0)
        rows_all = None
    v.close()
    if not inproc:
        dist.destroy_process_group()
    if want_cpu and rank == 0:
        # the reference algorithm over the N-times larger log, owner 0's read
        # sets (an evenly spaced sample), against the merged GPU verdicts
        cpus = box_cpus()
        threads = args.cpu_threads or cpus["threads"]
        share0 = first_rs.subset(np.arange(0, T))
        print(f"[bench] cpu baseline on {threads} threads ({cpus})", file=sys.stderr, flush=True)
        if args.config == 3:
            from comdb2_amd.workloads import config3_log
            c0 = log_tail_commit(c3.commit_lsn, share0.snap)
            log = config3_log(c3, from_commit=c0)
            note = (f" (the global log's tail from commit {c0} of {len(c3.commit_lsn)}: every "
                    f"record after the oldest snapshot of owner 0's read sets)")
        else:
            log = config5_log(tails, keys_per_commit=10, commit_base=c_start)
            note = (f" (the global log of all {N} members' writes from global commit "
                    f"{c_start * N} on: every record after the oldest snapshot of owner 0's "
                    f"read sets)")
        tails = None
        cpu = cpu_baseline(log, share0, v0, threads, args.cpu_seconds, log_note=note)
        cpu["host"] = cpus
        cpu["read_sets"] = "owner 0's share of the global batch (member 0's merged verdicts)"
        out["cpu_baseline"] = cpu
        out["parity"] = {"kind": "owner 0's merged verdicts vs oracle/serial_oracle.c on the "
                                 "cpu_baseline sample (the global log)",
                         "equal": bool(cpu["parity_with_gpu"] and cpu["single_core"]["parity_with_gpu"])}
    if rank == 0:
        print(json.dumps(out), flush=True)


def replicas_api_leg(hsc, torch, devs, rows_all, end_lsn, rs, want):
    """The drop-in entry on a replicated multi context (HSC_MULTI_REPLICAS):
    every member ingests the whole global window from device rows, a lone
    call or a collector pass goes whole to one member (the one with the
    fewest passes in flight), a large batch is sliced over the members -- the
    same legs as multi_api_leg, same read sets, same expected verdicts."""
    rv = hsc.MultiValidator(devs)
    try:
        assert rv.register_group("t1", 0, 9) == 0
        rv.set_mode(hsc.MULTI_REPLICAS)
        gid = np.concatenate([r[0] for r in rows_all])
        words = np.concatenate([r[1] for r in rows_all], axis=1)
        lsn = np.concatenate([r[2] for r in rows_all])
        for i, d in enumerate(devs):
            dv = torch.device("cuda", d)
            tg = torch.from_numpy(np.ascontiguousarray(gid)).to(dv)
            tw = torch.from_numpy(np.ascontiguousarray(words).reshape(-1).view(np.int64)).to(dv)
            tl = torch.from_numpy(np.ascontiguousarray(lsn).view(np.int64)).to(dv)
            torch.cuda.synchronize(dv)
            rv.member(i).ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(),
                                       tl.data_ptr(), end_lsn)
            del tg, tw, tl
        rv.adopt()
        out = multi_api_leg(hsc, rv, rs, want)
        out["mode"] = "replicas" if rv.mode == hsc.MULTI_REPLICAS else "pieces"
        out["window_keys_per_member"] = rv.member(0).keys
        return out
    finally:
        rv.close()


def multi_api_leg(hsc, v, rs, want):
    """The drop-in entry on the in-process multi context, the per-transaction
    call pattern of db/toblock.c:4777-4800: a lone caller (one
    hip_bdb_osql_serial_check at a time), 64 threads through the collector,
    64 uncollected.  Each call is routed on the host while marshalled; only
    the members its ranges overlap run their small kernels."""
    arrs = hsc.NativeCurRangeArrs(rs)
    want = np.asarray(want) != 0
    conc = {}
    v.concurrent_check(arrs, 64)  # warm-up
    r0 = v.route_stats()
    got, st = v.concurrent_check(arrs, 64)
    st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want))
    conc["threads_64"] = st
    # collector passes in flight (default 4): each pass launches and waits on
    # every member its ranges touch, so a multi pass is longer than a one-GPU one
    sweep = {}
    for inf in (2, 3, 6):
        got, s2 = v.concurrent_check(arrs, 64, inflight=inf)
        sweep[str(inf)] = {"checks_per_s": s2["checks_per_s"], "lat_p50_us": s2["lat_p50_us"],
                           "lat_p99_us": s2["lat_p99_us"], "mean_batch": s2.get("mean_batch"),
                           "parity_with_device_batch": bool(np.array_equal(got != 0, want))}
    conc["threads_64_inflight"] = sweep
    # the plain drop-in entry from 64 threads (the context's own collector)
    got, st = v.concurrent_check(arrs, 64, collect=False)
    st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want))
    st["entry"] = "hip_bdb_osql_serial_check (context-owned collector, the default)"
    conc["threads_64_dropin"] = st
    m = min(rs.ntxn, 2000)
    sub = hsc.NativeCurRangeArrs(_readsets_head(rs, m))
    v.set_autocollect(False)
    for nth in (1, 64):
        got, st = v.concurrent_check(sub, nth, collect=False)
        st["parity_with_device_batch"] = bool(np.array_equal(got != 0, want[:m]))
        st["sample"] = f"first {m} read sets"
        conc[f"threads_{nth}_uncollected"] = st
    v.set_autocollect(True)
    r1 = v.route_stats()
    sub.close()
    arrs.close()
    calls = max(1, r1["calls"] - r0["calls"])
    return {"entry": "hip_bdb_osql_serial_check / hsc_collector_check on the multi context",
            "members": v.world, "concurrent_callers": conc,
            "members_per_call": (r1["member_checks"] - r0["member_checks"]) / calls,
            "host_route_us_per_call": r1["route_us_per_call"],
            "host_launch_us_per_call": r1["launch_us_per_call"],
            "wait_us_per_call": r1["wait_us_per_call"],
            "front_small_stats": v.small_stats(), "front_batch_stats": v.batch_stats(),
            "member_small_stats": [v.member(i).small_stats() for i in range(v.nlocal)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", type=int, default=2,
                    help="distinct resident read-set batches (at least; see --ring-gb)")
    ap.add_argument("--ring-gb", type=float, default=None,
                    help="cycle distinct resident batches whose probe inputs total at least this "
                         "many GB (default: 1.1 for config 2 -- past the 256 MiB Infinity Cache "
                         "-- else 0); the 2-batch L3-resident ring is timed alongside")
    ap.add_argument("--n-commits", type=int, default=1_000_000)
    ap.add_argument("--n-txn", type=int, default=100_000)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: the box's CPUs, min(affinity, cgroup quota))")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    ap.add_argument("--no-api", action="store_true",
                    help="skip the drop-in entry leg (hip_serial_check_batch end to end)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--multi-pmc", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--c4-dir", default="", help=argparse.SUPPRESS)
    ap.add_argument("--c4-ntxn", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--c4-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--wide", action="store_true", help="force the wide window layout")
    ap.add_argument("--paths", type=int, default=0,
                    help="hsc_set_paths flags of the one-GPU context, set before the build (A/B runs; "
                         "64 = HSC_PATH_NO_CT_POINTS)")
    ap.add_argument("--compact-wide", action="store_true",
                    help="compact windows: probe through the wide tile pipeline instead of "
                         "the compact tiles (A/B)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the batches rotate over (each with its own outputs and "
                         "probe lane), so consecutive batches' kernels can overlap (default 2; "
                         "3 for config 3, r05p: 74.4 vs 77.3 us per batch, while configs 2 / 5 "
                         "measured 45.0 / 52.3 us on 2 against 48.2 / 54.5 on 3)")
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4, 5),
                    help="1: the config-1 commit stream through the drop-in entry with "
                         "incremental appends; 2: the headline check batch; 3: composite keys over "
                         "32 (table, index) "
                         "groups, group shards; 4: dependency graph + SCC of a history; "
                         "5: Zipf hot keys over a large window (per-GPU imbalance reported)")
    ap.add_argument("--n-txn-c1", type=int, default=10_000, help="config 1: txns in the stream")
    ap.add_argument("--c1-steady", type=int, default=100_000,
                    help="config 1: txns of the steady-state leg (default fold threshold; 0: skip)")
    ap.add_argument("--c3-writes", type=int, default=4_000_000,
                    help="config 3: index writes per GPU (log-normal group sizes)")
    ap.add_argument("--c5-keys", type=int, default=125_000_000,
                    help="config 5: window writes per GPU (125M x 8 GPUs = SURVEY's 1B)")
    ap.add_argument("--check", action="store_true",
                    help="config 3 / 5, N = 1: full-batch CPU sort-join parity (oracle/sortjoin.c)")
    ap.add_argument("--history-txns", type=int, default=16_700_000,
                    help="config 4: transactions (x ~6 ops: 16.7M = SURVEY's 100M-op history)")
    ap.add_argument("--c4-concurrent", type=float, default=0.02,
                    help="config 4: fraction of txns reading a stale snapshot")
    ap.add_argument("--c4-max-lag", type=int, default=64, help="config 4: max snapshot lag")
    ap.add_argument("--c4-keys", type=int, default=0, help="config 4: keys (0: txns / 10)")
    ap.add_argument("--inproc", type=int, default=0,
                    help="without torchrun: N members of one multi context in this process "
                         "(the visible GPUs round robin; members share a GPU when there are "
                         "fewer) -- the in-process multi-GPU path")
    ap.add_argument("--loopback", action="store_true",
                    help="in-process multi context: the per-rank exchange with peer copies "
                         "(hsc_multi_set_transport) for the device-routed leg and the merge")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="multi legs: GPU_MAX_HW_QUEUES for this process (0: max(the box's, 8))")
    ap.add_argument("--rank-path", action="store_true",
                    help="run the per-rank (RCCL) multi-GPU path even at WORLD_SIZE 1 (its "
                         "world-1 rehearsal on one GPU)")
    args = ap.parse_args()
    if args.streams is None:
        args.streams = 3 if args.config == 3 else 2
    if args.ring_gb is None:
        args.ring_gb = 1.1 if args.config in (2, 3, 5) else 0.0

    if args.config == 4:
        return bench_graph(args)
    if args.config == 1:
        return bench_commit_stream(args)
    if (int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.gpus > 1 or args.inproc > 1
            or args.rank_path or args.multi_pmc > 1):
        # the multi context runs more streams per process than HIP's default 4
        # hardware queues (per member: its lanes' streams, its small-batch
        # slots; RCCL's): with 4, streams share queues and serialise (r05ae:
        # 2 members on one GPU 119.5 -> 100.7 us per step with 8).  Read by the
        # HIP runtime at its initialisation, so set before anything touches the
        # GPU; a larger setting is kept.
        try:
            q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        except ValueError:
            q = 4
        # (--hw-queues N: exactly N, e.g. the box's default 4 for an A/B)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues if args.hw_queues > 0 else max(q, 8))
        return bench_multi(args)
    # one GPU (N > 1 runs bench_multi)
    world, rank = 1, 0
    traffic = None
    if args.config in (2, 3, 5) and not args.no_pmc and not args.pmc_child and not args.wide:
        traffic = pmc_traffic(args)  # child processes, before this one touches the GPU
    import torch

    from comdb2_amd import hsc, shard
    from comdb2_amd.workloads import SEED_CONFIG2, config2, config2_device_window

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    want_cpu = not args.no_cpu and args.config in (2, 3, 5) and not args.pmc_child
    batches = []
    v = hsc.Validator(local)
    if args.paths:
        v.set_paths(args.paths)
    if args.wide:
        v.set_layout(hsc.LAYOUT_WIDE)
    elif args.compact_wide:
        v.set_layout(hsc.LAYOUT_COMPACT_WIDE)
    if args.config != 3:
        gid_t = v.register_group("t1", 0, 9)
        assert gid_t == 0
    c3 = None
    if args.config == 3:
        from comdb2_amd.workloads import SEED_CONFIG3, config3_arrays
        c3 = config3_arrays(seed=SEED_CONFIG3, n_writes=args.c3_writes * world,
                            n_txn=args.n_txn * world)
        for g, (tbn, ix, L) in enumerate(c3.groups):
            assert v.register_group(tbn, ix, L) == g
        gid, words, lsn = c3.window()
        mine = list(range(len(c3.groups)))
        end_lsn = c3.end_lsn
        first_rs = c3.readsets
        more_rs = lambda bi: config3_arrays(seed=SEED_CONFIG3, n_writes=args.c3_writes * world,
                                            n_txn=args.n_txn * world, rs_seed=bi).readsets
        workload = (f"config3: {len(c3.groups)} (table, index) groups of composite keys "
                    f"(9-64 B, log-normal sizes), {args.c3_writes} index writes and "
                    f"{args.n_txn} read sets per GPU (points, ranges, prefixes, table locks)")
        data = "synthetic (config 3 generator, seed 0xC0FFEE03, weak scaling per GPU)"
    elif args.config == 2:
        value_bits = 40
        c2 = config2(seed=SEED_CONFIG2, n_commits=args.n_commits, n_txn=args.n_txn, rank=rank,
                     world=world, build_log=want_cpu)
        gid, words, lsn = config2_device_window(c2)
        end_lsn = c2.params["end_lsn"]
        first_rs = c2.readsets
        more_rs = lambda bi: config2(seed=SEED_CONFIG2 + 7919 * bi, n_commits=args.n_commits,
                                     n_txn=args.n_txn, rank=rank, world=world,
                                     build_log=False).readsets
        workload = ("config2: per GPU 100k read sets x 10 ranges (1M ranges) vs a window of "
                    "1M commits x 10 int64 index keys (10M logged keys), one index")
        data = ("synthetic (BASELINE config 2 generator, seed 0xC0FFEE02; int64 keys in memcmp "
                "order as big-endian u64 words)")
    else:
        from comdb2_amd.workloads import SEED_CONFIG5, config5_scaled, int64_words
        c5 = config5_scaled(seed=SEED_CONFIG5, keys_per_gpu=args.c5_keys, n_txn=args.n_txn,
                            rank=rank, world=world)
        keys5, lsn, end_lsn = c5.keys, c5.lsn, c5.end_lsn
        first_rs = c5.readsets
        more_rs = lambda bi: config5_scaled(seed=SEED_CONFIG5 + 7919 * bi,
                                            keys_per_gpu=args.c5_keys, n_txn=args.n_txn,
                                            rank=rank, world=world, window=False).readsets
        words = int64_words(keys5)
        gid = np.zeros(len(keys5), dtype=np.uint32)
        del keys5
        workload = (f"config5: one global Zipf(1.2) law over 2^32 keys, {args.c5_keys} logged "
                    f"writes per GPU (hot keys collapse under dedupe), sampled global splitters, "
                    f"100k read sets x 10 ranges per GPU (width {c5.params['width']}, 3 % of the "
                    f"points on Zipf-drawn hot keys)")
        data = "synthetic (config 5 generator, seed 0xC0FFEE05, weak scaling per GPU)"
    n_w = len(lsn)
    tg = torch.from_numpy(gid).to(dev)
    tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
    tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
    v.ingest_device(n_w, words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), end_lsn)
    ingest_cold_ms = v.timing()["ingest_ms"]  # first build: its buffers are allocated inside
    # the same rows again: a rebuild over allocated buffers (a fold, a re-ingest)
    v.ingest_device(n_w, words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), end_lsn)
    ingest_ms = v.timing()["ingest_ms"]
    del tg, tw, tl
    if c3 is not None:
        v.merge_table_max(c3.table_max)  # data-row writes lock tables too
    W = v.words
    T = first_rs.ntxn
    m0 = None
    ring_bytes = 0
    bi = 0
    nb_min = max(2, args.batches)
    while bi < nb_min or ring_bytes < args.ring_gb * 1e9:
        rs = first_rs if bi == 0 else more_rs(bi)
        m = v.marshal(rs)
        if bi == 0 and (want_cpu or args.check):
            m0 = m
        b = upload_batch(torch, dev, m)
        b["bytes"] = sum(int(b[k].numel() * b[k].element_size())
                         for k in ("lo", "hi", "gid", "snap", "txn", "lock_table", "lock_snap",
                                   "lock_txn"))
        ring_bytes += b["bytes"]
        batches.append(b)
        bi += 1
        if bi % 8 == 0:
            print(f"[bench] {bi} batches, {ring_bytes / 1e9:.2f} GB", file=sys.stderr, flush=True)
    S = max(1, args.streams)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(S - 1)]
    verdicts = [torch.zeros(T, dtype=torch.uint8, device=dev) for _ in range(S)]
    # the verdict bytes are the result, no bitmap (the pack is folded into the plan kernel)
    structs = [[probe_struct(hsc, b, verdicts[si], None, T) for si in range(S)] for b in batches]
    torch.cuda.synchronize()

    if args.pmc_child:  # profiled by the parent's rocprofv3 --pmc pass: the ring, S streams
        for k in range(len(batches)):
            v.set_stream(streams[k % S].cuda_stream)
            v.probe_device(structs[k][k % S])
        v.synchronize()
        v.close()
        return

    def step(k, nstreams, nbatch):
        si = k % nstreams
        st = streams[si]
        v.set_stream(st.cuda_stream)
        v.probe_device(structs[k % nbatch][si])

    def timed(nstreams, nbatch):
        for k in range(args.warmup):
            step(k, nstreams, nbatch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            step(k, nstreams, nbatch)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return el

    NB = len(batches)
    # the ring: every timed step probes a batch no other step of the region touches
    # (warmup + steps <= NB) or, with a longer run, the least recently probed one
    elapsed = timed(S, NB)
    # the secondary legs (one stream; cache-resident): the median of 5 timed
    # regions each, so one host hiccup inside a ~1 ms region does not move them
    def med(nstreams, nbatch):
        return float(np.median([timed(nstreams, nbatch) for _ in range(5)]))
    serial_elapsed = med(1, NB) if S > 1 else elapsed
    # L3-resident: two batches alternate (window + both batches fit the 256 MiB cache)
    l3_elapsed = med(S, 2) if NB > 2 else elapsed
    l3_serial = med(1, 2) if NB > 2 else serial_elapsed
    v.set_stream(streams[0].cuda_stream)

    # verdicts of batch 0 (for the conflict rate and the CPU parity sample)
    step(0, 1, NB)
    torch.cuda.synchronize()
    v0 = verdicts[0].cpu().numpy().copy()
    forced = batches[0]["forced"]
    v0 = np.maximum(v0, forced)

    # per-kernel device time (separate pass over the ring; events on the launch stream)
    v.enable_timing(True)
    acc = {}
    for k in range(args.steps):
        v.probe_device(structs[k % NB][0])
        v.synchronize()
        for key, val in v.timing().items():
            acc.setdefault(key, []).append(val)
    v.enable_timing(False)
    tm = {k: float(np.mean(vals)) for k, vals in acc.items()}

    n_keys = v.keys
    n_r = int(np.mean([b["n"] for b in batches]))
    # B = N_w s_w + N_r s_r + ceil(N_t / 8), s_w = L^ + 12, s_r = 2 L^ + 16
    Lhat = 8 * W
    s_w, s_r = Lhat + 12, 2 * Lhat + 16
    B = n_keys * s_w + n_r * s_r + (T + 7) // 8
    if args.config == 3:  # per group L^ = 8 ceil(L / 8): window keys and ranges of each group
        lhat = np.array([8 * ((L + 7) // 8) for (_, _, L) in c3.groups], np.int64)
        keys_g = np.zeros(len(c3.groups), np.int64)
        for g in mine:
            kb = c3.keys_of[g][np.unique(c3.w_row[c3.w_group == g])]
            keys_g[g] = len(np.unique(np.ascontiguousarray(kb).view(np.dtype((np.void, kb.shape[1])))))
        host = lambda x: x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
        rng_g = np.mean([np.bincount(host(b["gid"]), minlength=len(c3.groups)) for b in batches],
                        axis=0)
        B = int((keys_g * (lhat + 12)).sum() + (rng_g * (2 * lhat + 16)).sum() + (T + 7) // 8)
    WG = v.tile_key_words if v.layout == hsc.LAYOUT_COMPACT and not args.compact_wide else 0
    kern = kernel_bytes(v.layout, W if WG else v.code_words, n_keys, n_r, T, tm, WG, False)
    ms_per_step = elapsed / args.steps * 1e3
    frac = lambda el: B / (el / args.steps) / 1e9 / HBM_PEAK_GBS
    checks = T * args.steps
    out = {
        "metric": METRIC,
        "value": checks / elapsed,
        "unit": "checks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": data,
        "config": {
            "workload": workload,
            "read_sets_per_step": T,
            "ranges_per_gpu": n_r,
            "window_keys_per_gpu": n_keys,
            "logged_writes_per_gpu": n_w,
            "parallelism": "one GPU (bench.py --gpus N: the multi-GPU context, bench_multi)",
            "streams": S,
            "serial_ms_per_step": serial_elapsed / args.steps * 1e3,
            "ring_batches": NB,
            "window_layout": {hsc.LAYOUT_NARROW: "narrow (u32 tile-relative keys)",
                              hsc.LAYOUT_COMPACT: (f"compact tiles ({WG}-word keys gid || code, "
                                                   f"{v.code_words}-word codes of {W}-word keys)"
                                                   if WG else
                                                   f"compact ({v.code_words}-word codes of "
                                                   f"{W}-word keys, wide tile pipeline)"),
                              hsc.LAYOUT_WIDE: "wide"}.get(v.layout, "?"),
            "conflict_rate": float((v0 != 0).mean()),
        },
        "roofline": {
            # the probe phase as SURVEY 8(d) defines it: B over the device time of
            # one batch (the timed loop runs batches back to back over the ring)
            "bound": "hbm",
            "kernel": "probe phase (" + ", ".join(kern) + ")",
            "achieved": B / (ms_per_step * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": frac(elapsed),
            "frac_1stream": frac(serial_elapsed),
            "secondary_legs": "frac_1stream and l3_resident: the median of 5 timed regions each",
            "traffic": traffic.get("bytes_per_batch") if traffic else None,
            # the same time against the PMC-measured bytes (FETCH_SIZE counts
            # Infinity-Cache hits too): how much of HBM's peak the probe phase
            # actually moves; frac above is the algorithmic-bytes roofline
            "measured_frac": (traffic["bytes_per_batch"] / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS
                              if traffic and traffic.get("bytes_per_batch") else None),
            "algorithmic_bytes": B,
            "avg_ms": ms_per_step,
            "working_set": {
                "ring_batches": NB,
                "ring_input_bytes": int(sum(b["bytes"] for b in batches)),
                "note": "distinct resident probe batches cycled by the timed loop (every step "
                        "a batch no other step of the region touches) plus the resident window; "
                        "past the 256 MiB Infinity Cache"},
            "l3_resident": {
                "batches": 2,
                "input_bytes": int(batches[0]["bytes"] + batches[min(1, NB - 1)]["bytes"]),
                "ms_per_step": l3_elapsed / args.steps * 1e3,
                "serial_ms_per_step": l3_serial / args.steps * 1e3,
                "frac": frac(l3_elapsed),
                "frac_1stream": frac(l3_serial),
                "value": checks / l3_elapsed},
        },
        "probe_phase": {
            "event_total_ms": tm["probe_total_ms"],
            "kernels": kern,
            "join_records": tm["records"], "tiles": tm["tiles"],
        },
        "ingest_ms": ingest_ms,
        # window build (sort + dedupe + summaries), SURVEY 8(d): reported apart
        # from the probe phase; bytes = N_w * (L^ + 8 LSN + 4 group)
        "ingest": {"rows": int(n_w), "algorithmic_bytes": int(n_w) * (8 * W + 12),
                   "GBps": int(n_w) * (8 * W + 12) / (ingest_ms * 1e-3) / 1e9 if ingest_ms else None,
                   "ms": ingest_ms, "cold_ms": ingest_cold_ms,
                   "note": "window build (device_build: sort, dedupe, summaries, narrow index) "
                           "of rows already in HBM, timed by events around it; ms = a rebuild "
                           "over allocated buffers, cold_ms = the context's first build"},
        "cold_e2e_ms": ingest_cold_ms + ms_per_step,
        "cpu_baseline": None,
    }
    if traffic:
        out["roofline"]["traffic_detail"] = traffic
    if args.config == 3:
        if args.check:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            sj = oracle.SortJoin(gid, words, lsn, len(c3.groups))
            want, secs = sj.probe(m0, v.table_max(), nthreads=box_cpus()["threads"])
            sj.close()
            out["parity"] = {"kind": "full batch 0 vs oracle/sortjoin.c (CPU sort-join)",
                             "equal": bool(np.array_equal(want != 0, v0 != 0)), "cpu_s": secs}
    if args.config == 5:
        if args.check:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            sj = oracle.SortJoin(gid, words, lsn, 1)
            want, secs = sj.probe(m0, np.array([lsn.max()], np.uint64),
                                  nthreads=box_cpus()["threads"])
            sj.close()
            out["parity"] = {"kind": "full batch 0 vs oracle/sortjoin.c (CPU sort-join)",
                             "equal": bool(np.array_equal(want != 0, v0 != 0)),
                             "cpu_s": secs}
    if args.config == 2 and not args.no_api:
        out["api"] = api_leg(hsc, v, first_rs, v0, args)
    if want_cpu:
        cpus = box_cpus()
        threads = args.cpu_threads or cpus["threads"]
        print(f"[bench] cpu baseline on {threads} threads ({cpus})", file=sys.stderr, flush=True)
        if args.config == 2:
            out["cpu_baseline"] = cpu_baseline(c2.log, c2.readsets, v0, threads, args.cpu_seconds,
                                               m0=m0, window=config2_device_window(c2))
        elif args.config == 3:
            from comdb2_amd.workloads import config3_log
            c0 = log_tail_commit(c3.commit_lsn, first_rs.snap)
            out["cpu_baseline"] = cpu_baseline(
                config3_log(c3, from_commit=c0), first_rs, v0, threads, args.cpu_seconds, m0=m0,
                window=(gid, words, lsn), table_max=c3.table_max, ngroups=len(c3.groups),
                log_note=f" (the tail from commit {c0} of {len(c3.commit_lsn)}: every record "
                         f"after the batch's oldest snapshot)")
        else:
            from comdb2_amd.workloads import config5_log
            K5 = c5.params["keys_per_commit"]
            c0 = log_tail_commit(c5.lsn[K5 - 1::K5], first_rs.snap)
            out["cpu_baseline"] = cpu_baseline(
                config5_log([c5.keys], keys_per_commit=K5, from_commit=c0), first_rs, v0,
                threads, args.cpu_seconds, m0=m0, window=(gid, words, lsn),
                log_note=f" (the tail from commit {c0} of {len(c5.lsn) // K5}: every record "
                         f"after the batch's oldest snapshot)")
        out["cpu_baseline"]["host"] = cpus
    print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
