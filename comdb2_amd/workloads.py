"""Synthetic workloads of BASELINE.json's configs (seeded, numpy-vectorised).

* :func:`config2` -- 1xMI355X: N_t read sets x 10 ranges vs a log window of
  1M commits x 10 int64 index keys on one index.
* :func:`config1_events` -- the ``tests/tools/serial.c`` shaped commit stream
  (20 ids x 5 accounts, read ``sum where id``, read one row, update it).
* :func:`random_case` -- small adversarial logs + read sets exercising every
  record type and every rule of the check (parity tests).
* :func:`replay` -- drive a commit stream through a checker in commit order,
  appending each passing write txn to the log (SURVEY.md §7 hard part 7a).
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import formats as F
from .formats import LLog, LogBuilder, Range, ReadSets, lsn

SEED_CONFIG1 = 0xC0FFEE01
SEED_CONFIG2 = 0xC0FFEE02


def ranges_in_set_order(lo_u: np.ndarray, T: int, per_txn: int) -> np.ndarray:
    """Permutation that sorts every read set's `per_txn` consecutive ranges by
    lo_u, stably (= np.lexsort((lo_u, txn_of_range)) for equal-size read sets,
    without the global sort: 5.3 s -> 0.3 s for 8M ranges)."""
    o = np.argsort(np.asarray(lo_u).reshape(T, per_txn), axis=1, kind="stable")
    return (o + (np.arange(T, dtype=np.int64) * per_txn)[:, None]).reshape(-1)


def lsn_to_index(lsn) -> np.ndarray:
    """Inverse of lsn_of_index (same defaults)."""
    lsn = np.asarray(lsn, dtype=np.uint64)
    f = lsn >> np.uint64(32)
    o = lsn & np.uint64(0xFFFFFFFF)
    return (f - np.uint64(1)) * np.uint64(1 << 26) + (o - np.uint64(28)) // np.uint64(64)


def lsn_of_index(idx: np.ndarray, per_file: int = 1 << 26, step: int = 64) -> np.ndarray:
    """LSN of the idx-th record when records are `step` bytes apart and a file
    holds `per_file` records."""
    idx = np.asarray(idx, dtype=np.uint64)
    f = np.uint64(1) + idx // np.uint64(per_file)
    o = np.uint64(28) + (idx % np.uint64(per_file)) * np.uint64(step)
    return (f << np.uint64(32)) | o


# ---------------------------------------------------------------------------
# config 2
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class Config2:
    log: LLog
    readsets: ReadSets
    commit_lsn: np.ndarray      # uint64[n_commits] regop LSN of each commit
    key_values: np.ndarray      # int64[n_commits * k] written values (log order)
    params: dict


def config2(seed: int = SEED_CONFIG2, n_commits: int = 1_000_000, keys_per_commit: int = 10,
            n_txn: int = 100_000, ranges_per_txn: int = 10, value_bits: int = 40,
            width: int = 1 << 20, snap_recent: float = 0.01, build_log: bool = True,
            rank: int = 0, world: int = 1) -> Config2:
    """Writes: values uniform in [0, 2^value_bits), n_commits x keys_per_commit
    undo_upd_ix records on table "t1" index 0, one committed txn per commit.
    Ranges (per read set, sorted by lower bound like a coalesced CurRangeArr):
    50% point (half on a written key), 40% [v, v + width], 8% prefix ranges
    (lower/upper endpoint = the first 6 or 7 bytes of a key), 2% open on one
    side.  Snapshots: the regop LSN of a commit drawn uniformly from the most
    recent `snap_recent` fraction of commits (recent snapshots keep the
    conflict rate inside the 20-60% band SURVEY.md §8(d) asks for).

    Sharded form (world > 1, weak scaling): the key space is range-partitioned,
    rank r's window holds the keys [r, r+1) * 2^value_bits written by its own
    n_commits commits (global commit g = c * world + r, so LSNs interleave);
    the read sets are the global world * n_txn ones over the whole key space."""
    K = keys_per_commit
    R = K + 3  # ltran_start, K undo records, ltran_commit, regop
    vals_all = [np.random.default_rng([seed, r]).integers(r << value_bits, (r + 1) << value_bits,
                                                           size=n_commits * K, dtype=np.int64)
                for r in range(world)]
    vals = vals_all[rank]
    gcommit = np.arange(n_commits, dtype=np.uint64) * np.uint64(world) + np.uint64(rank)
    commit_lsn = lsn_of_index(gcommit * np.uint64(R) + np.uint64(R - 1))
    end_lsn = int(lsn_of_index(np.array([world * n_commits * R]))[0])
    log = None
    if build_log:
        nrec = n_commits * R
        idx = (np.repeat(gcommit, R) * np.uint64(R) + np.tile(np.arange(R, dtype=np.uint64), n_commits))
        lsns = lsn_of_index(idx)
        j = np.tile(np.arange(R, dtype=np.int64), n_commits)
        rectype = np.full(nrec, F.REC_UNDO_UPD_IX, dtype=np.uint32)
        rectype[j == 0] = F.REC_LTRAN_START
        rectype[j == R - 2] = F.REC_LTRAN_COMMIT
        rectype[j == R - 1] = F.REC_TXN_REGOP
        prev = np.zeros(nrec, dtype=np.uint64)
        prev[1:] = lsns[:-1]
        prev[j == 0] = 0
        is_undo = (j >= 1) & (j <= K)
        table = np.where(is_undo, 0, -1).astype(np.int32)
        ix = np.zeros(nrec, dtype=np.int16)
        keylen = np.where(is_undo, 9, 0).astype(np.int32)
        key_off = np.zeros(nrec, dtype=np.uint64)
        key_off[is_undo] = np.arange(n_commits * K, dtype=np.uint64) * np.uint64(9)
        keys = F.enc_int64_array(vals).reshape(-1)
        log = LLog(lsns, rectype, prev, np.zeros(nrec, dtype=np.int16), table, ix, key_off,
                   keylen, keys, ["t1"], end_lsn)

    # read ranges (global: identical on every rank)
    rng = np.random.default_rng([seed, 1 << 20])
    T = n_txn * world
    nr = T * ranges_per_txn
    kind = rng.choice(4, size=nr, p=[0.5, 0.4, 0.08, 0.02])
    v = rng.integers(0, world << value_bits, size=nr, dtype=np.int64)
    hit = rng.random(nr) < 0.5
    allv = vals_all[0] if world == 1 else np.concatenate(vals_all)
    v = np.where((kind == 0) & hit, allv[rng.integers(0, len(allv), size=nr)], v)
    lo = F.enc_int64_array(v)
    hi = F.enc_int64_array(np.where(kind == 1, v + width, v))
    lkeylen = np.full(nr, 9, dtype=np.int32)
    rkeylen = np.full(nr, 9, dtype=np.int32)
    plen = rng.integers(6, 8, size=nr).astype(np.int32)
    lkeylen[kind == 2] = plen[kind == 2]
    rkeylen[kind == 2] = plen[kind == 2]
    lflag = np.zeros(nr, dtype=np.int32)
    rflag = np.zeros(nr, dtype=np.int32)
    side = rng.random(nr) < 0.5
    lflag[(kind == 3) & side] = 1
    rflag[(kind == 3) & ~side] = 1
    lkeylen[lflag == 1] = 0
    rkeylen[rflag == 1] = 0
    # sort each read set's ranges by lower bound (currange_cmp order: lflag first)
    lo_u = np.where(lflag == 1, -1, v.astype(np.int64))
    order = ranges_in_set_order(lo_u, T, ranges_per_txn)
    lo, hi = lo[order], hi[order]
    lkeylen, rkeylen, lflag, rflag = lkeylen[order], rkeylen[order], lflag[order], rflag[order]
    keys = np.concatenate([lo.reshape(-1), hi.reshape(-1)])
    lkey_off = np.arange(nr, dtype=np.uint64) * np.uint64(9)
    rkey_off = np.uint64(nr * 9) + np.arange(nr, dtype=np.uint64) * np.uint64(9)
    ncg = world * n_commits
    recent = max(1, int(round(ncg * snap_recent)))
    gi = np.uint64(ncg - 1) - rng.integers(0, recent, size=T).astype(np.uint64)
    snap = lsn_of_index(gi * np.uint64(R) + np.uint64(R - 1))
    rs = ReadSets(txn_off=np.arange(0, nr + 1, ranges_per_txn, dtype=np.int64), snap=snap,
                  table=np.zeros(nr, np.int32), idxnum=np.zeros(nr, np.int32), lflag=lflag,
                  rflag=rflag, islocked=np.zeros(nr, np.int32), lkeylen=lkeylen, rkeylen=rkeylen,
                  lkey_off=lkey_off, rkey_off=rkey_off, keys=keys, tbnames=["t1"])
    return Config2(log, rs, commit_lsn, vals,
                   dict(seed=seed, n_commits=n_commits, keys_per_commit=K, n_txn=n_txn,
                        ranges_per_txn=ranges_per_txn, value_bits=value_bits, width=width,
                        snap_recent=snap_recent, rank=rank, world=world, end_lsn=end_lsn))


def config2_rank_window(seed: int = SEED_CONFIG2, n_commits: int = 1_000_000, rank: int = 0,
                        world: int = 1, keys_per_commit: int = 10, value_bits: int = 40):
    """Rank `rank`'s window of config2(seed, ..., rank, world) without its read
    sets: (gid, words, lsn) as config2_device_window gives them, and the
    written values (key_values).  The same rows as the full call."""
    K = keys_per_commit
    R = K + 3
    vals = np.random.default_rng([seed, rank]).integers(rank << value_bits, (rank + 1) << value_bits,
                                                        size=n_commits * K, dtype=np.int64)
    gcommit = np.arange(n_commits, dtype=np.uint64) * np.uint64(world) + np.uint64(rank)
    commit_lsn = lsn_of_index(gcommit * np.uint64(R) + np.uint64(R - 1))
    c2 = Config2(None, None, commit_lsn, vals, dict(keys_per_commit=K))
    gid, words, lsn = config2_device_window(c2)
    return gid, words, lsn, vals


def config2_device_window(c2: Config2) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The decoded window of config 2 as (gid u32[n], words u64[2][n], lsn u64[n])
    in log order -- the rows hsc_window_ingest_log would stage (one group)."""
    n = len(c2.key_values)
    b = F.enc_int64_array(c2.key_values)
    pad = np.zeros((n, 16), dtype=np.uint8)
    pad[:, :9] = b
    words = pad.view(">u8").astype(np.uint64).reshape(n, 2).T.copy()
    lsn = np.repeat(c2.commit_lsn, c2.params["keys_per_commit"])
    return np.zeros(n, dtype=np.uint32), words, lsn


# ---------------------------------------------------------------------------
# commit-stream replay
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class Txn:
    name: str
    reads: List[Range]
    writes: List[Tuple[int, str, int, Optional[bytes]]]  # (rectype, table, ix, key)


def replay(events: Sequence[Tuple[str, Txn]], check: Callable[[LLog, ReadSets], np.ndarray],
           tbnames: Sequence[str] = ()) -> dict:
    """events: ('begin', txn) / ('commit', txn) in time order.  At begin the
    snapshot is the end-of-log LSN (bdb_get_current_lsn, bdb/tran.c:2662).  At
    commit a write txn is checked (read-only txns never ship a read set,
    db/sqloffload.c:280-287,357-363); if serializable its writes are logged
    as one committed txn.  Returns {txn name: rc} for checked txns."""
    lb = LogBuilder(tbnames)
    snaps, rcs = {}, {}
    for ev, t in events:
        if ev == "begin":
            snaps[t.name] = lb.next_lsn()
            continue
        if not t.writes:
            continue
        log = lb.build()
        rs = ReadSets.from_lists([t.reads], [snaps[t.name]], tbnames=lb.tbnames)
        rc = int(check(log, rs)[0])
        rcs[t.name] = rc
        if rc == 0:
            lb.begin(t.name)
            for rt, tb, ix, key in t.writes:
                lb.write(t.name, rt, tb, ix, key)
            lb.commit(t.name)
    return rcs


def replay_incremental(events: Sequence[Tuple[str, Txn]], v, tbnames: Sequence[str] = (),
                       mode: str = "log", on_check=None, check_times=None) -> dict:
    """The commit stream of :func:`replay` against one validator whose window
    is kept up to date incrementally: an empty log is ingested once, then
    every passing write txn's records are appended -- as the continuation of
    the log (``mode="log"``: hsc_window_append_log, the chains decoded on the
    device side's host decoder) or as decoded writes (``mode="writes"``:
    hsc_window_append + hsc_window_set_end).  Each check is the drop-in entry
    bdb_osql_serial_check on a CurRangeArr.  Returns {txn name: rc};
    check_times (a list) collects each check's wall time in seconds."""
    import time
    from .hsc import CurRangeArrays, bdb_osql_serial_check
    lb = LogBuilder(tbnames)
    v.ingest_log(lb.build())
    snaps, rcs = {}, {}
    for ev, t in events:
        if ev == "begin":
            snaps[t.name] = lb.next_lsn()
            continue
        if not t.writes:
            continue
        arrs = CurRangeArrays([t.reads], [snaps[t.name]])
        if on_check:
            on_check()
        t0 = time.perf_counter()
        rc = int(bdb_osql_serial_check(v, arrs.arrs[0]))
        if check_times is not None:
            check_times.append(time.perf_counter() - t0)
        rcs[t.name] = rc
        if rc == 0:
            start = len(lb.rows)
            lb.begin(t.name)
            for rt, tb, ix, key in t.writes:
                lb.write(t.name, rt, tb, ix, key)
            c_lsn = lb.commit(t.name)
            if mode == "log":
                v.append_log(lb.build(start))
            else:
                v.append_writes([(tb, ix if key is not None else -2,
                                  None if rt in F.DTA_TYPES else key, c_lsn)
                                 for rt, tb, ix, key in t.writes], end_lsn=lb.next_lsn())
    return rcs


def protocol_replay_check(txns: Sequence[Txn], rc, commit_seq, snap, check_end, e0: int,
                          check: Callable[[LLog, ReadSets], np.ndarray]) -> dict:
    """Verify a commit-protocol run (Validator.commit_protocol, the harness
    of db/toblock.c:4757-4836) against `check` (the oracle): the committed
    txns' writes form the log in commit order (LSNs of the harness: commit k
    at e0 + 2k + 1, the end after k commits e0 + 2k, so a snapshot or a
    returned end S has seen (S - e0) / 2 commits).  Every verdict must be the
    reference's answer on the log as it stood when it was made:
      committed txn, commit k   -> check(log of commits < k, snapshot) == 0
      aborted txn               -> check(log its last full check saw) != 0
    (the final regop probe under the write lock saw no commit after the
    last full check's end, so the log before commit k is that check's log).
    -> {"checked", "mismatches", "first_mismatch"}."""
    n = len(txns)
    rc, commit_seq = np.asarray(rc), np.asarray(commit_seq)
    k_of = lambda S: (int(S) - int(e0)) // 2
    order = sorted((int(commit_seq[i]), i) for i in range(n) if commit_seq[i] >= 0)
    assert [k for k, _ in order] == list(range(len(order))), "commit sequence has gaps"
    lb = LogBuilder()
    ends, nrec = [lb.next_lsn()], [0]
    for _, i in order:
        t = txns[i]
        lb.begin(t.name)
        for rt, tb, ix, key in t.writes:
            lb.write(t.name, rt, tb, ix, key)
        lb.commit(t.name)
        ends.append(lb.next_lsn())
        nrec.append(len(lb.rows))
    full = lb.build()

    def prefix(p):
        m = nrec[p]
        return LLog(full.lsn[:m], full.rectype[:m], full.prev[:m], full.isabort[:m], full.table[:m],
                    full.ix[:m], full.key_off[:m], full.keylen[:m], full.keys, full.tbnames, ends[p])
    groups = {}
    for i in range(n):
        if not txns[i].writes:
            continue
        if commit_seq[i] >= 0:
            p, want = int(commit_seq[i]), 0
        else:
            p, want = k_of(check_end[i]), 1
        j = k_of(snap[i])
        assert 0 <= j <= p <= len(order), (i, j, p)
        groups.setdefault(p, []).append((i, j, want))
    bad, first = 0, None
    for p, items in sorted(groups.items()):
        rs = ReadSets.from_lists([txns[i].reads for i, _, _ in items], [ends[j] for _, j, _ in items],
                                 tbnames=full.tbnames)
        got = np.asarray(check(prefix(p), rs)) != 0
        for (i, j, want), g in zip(items, got):
            if int(g) != want or int(rc[i] != 0) != want:
                bad += 1
                if first is None:
                    first = {"txn": txns[i].name, "commits_seen": p, "snapshot_commits": j,
                             "protocol_rc": int(rc[i]), "oracle_rc": int(g)}
    return {"checked": sum(len(v) for v in groups.values()), "mismatches": bad, "first_mismatch": first}


def config1_events(seed: int = SEED_CONFIG1, n_txn: int = 10_000, n_ids: int = 20,
                   n_accts: int = 5, concurrency: int = 20) -> List[Tuple[str, Txn]]:
    """tests/tools/serial.c-shaped stream: table "accounts" with unique index 0
    = (id, acct) as two int64 fields (18-byte keys).  Each txn reads
    sum(bal) where id=? (prefix range over the 9-byte id field), reads one
    account row (point), and updates it (upd_dta + upd_ix).  `concurrency`
    txns are in flight; they begin/commit in a seeded random interleaving."""
    rng = np.random.default_rng(seed)
    tb = "accounts"
    txns = []
    for i in range(n_txn):
        idv = int(rng.integers(0, n_ids))
        acct = int(rng.integers(0, n_accts))
        pre = F.enc_int64(idv)
        key = pre + F.enc_int64(acct)
        reads = [Range(tb, 0, pre, pre), Range(tb, 0, key, key)]
        writes = [(F.REC_UNDO_UPD_DTA, tb, -2, None), (F.REC_UNDO_UPD_IX, tb, 0, key)]
        txns.append(Txn(f"T{i}", reads, writes))
    events, live, nxt = [], [], 0
    while nxt < n_txn or live:
        if nxt < n_txn and (len(live) < concurrency and (not live or rng.random() < 0.5)):
            events.append(("begin", txns[nxt]))
            live.append(txns[nxt])
            nxt += 1
        else:
            k = int(rng.integers(0, len(live)))
            events.append(("commit", live.pop(k)))
    return events


# ---------------------------------------------------------------------------
# random adversarial cases
# ---------------------------------------------------------------------------
def random_case(seed: int, n_commits: int = 60, n_txn: int = 40, tables=("ta", "tb", "tc"),
                n_ix: int = 3, keylens=(9, 18, 5), max_ranges: int = 8, value_range: int = 64,
                broken: bool = False) -> Tuple[LLog, ReadSets]:
    """Small log + read sets covering: all undo record types (dta and ix, _lk
    variants), comprec, aborted txns, read-only logical txns, regops whose
    prev is not an ltran_commit, interleaved txns, table locks (first-range
    rule), unsorted read sets (span quirk), prefix / over-long / open bounds,
    empty read sets, groups with several key lengths, snapshots at every kind
    of record and at/after the end of the log, and (broken=True) broken
    chains and dangling regops."""
    rng = np.random.default_rng(seed)
    lb = LogBuilder(list(tables) + ["never_written"])

    def key_for(ix):
        kl = keylens[ix % len(keylens)]
        v = int(rng.integers(0, value_range))
        k = F.enc_int64(v)
        if kl <= 9:
            return k[:kl]
        return (k + F.enc_int64(int(rng.integers(0, 4))) + bytes(64))[:kl]

    ix_types = F.IX_TYPES
    dta_types = F.DTA_TYPES
    live = []
    snaps_pool = [lb.next_lsn()]
    c = 0
    while c < n_commits:
        if live and (len(live) > 3 or rng.random() < 0.35):
            t = live.pop(int(rng.integers(0, len(live))))
            r = rng.random()
            regop = [F.REC_TXN_REGOP, F.REC_TXN_REGOP_GEN, F.REC_TXN_REGOP_ROWLOCKS][int(rng.integers(0, 3))]
            if r < 0.1:
                lb.commit(t, isabort=1, regop=regop)
            else:
                lb.commit(t, regop=regop)
            c += 1
        elif rng.random() < 0.06:
            # read-only logical txn: commit with prevllsn.file == 0
            lb.commit(("ro", c), empty=True)
            c += 1
        elif rng.random() < 0.05:
            # a regop whose prev record is not an ltran_commit
            s = lb.begin(("x", c))
            lb.raw(F.REC_TXN_REGOP, prev=s)
        else:
            t = ("t", c, int(rng.integers(0, 1 << 30)))
            lb.begin(t)
            live.append(t)
            for _ in range(int(rng.integers(1, 5))):
                tb = tables[int(rng.integers(0, len(tables)))]
                if rng.random() < 0.25:
                    lb.write(t, dta_types[int(rng.integers(0, len(dta_types)))], tb)
                else:
                    ix = int(rng.integers(0, n_ix))
                    lb.write(t, ix_types[int(rng.integers(0, len(ix_types)))], tb, ix, key_for(ix))
                if rng.random() < 0.1:
                    lb.comprec(t)
        snaps_pool.append(lb.rows[-1][0] if lb.rows else lb.next_lsn())
    for t in live:
        lb.commit(t)
    if broken:
        # dangling regop (prev points nowhere) and a committed txn whose chain breaks
        lb.raw(F.REC_TXN_REGOP, prev=(1 << 32) | 7)
        t = ("broken",)
        lb.begin(t)
        lb.write(t, F.REC_UNDO_UPD_IX, tables[0], 0, key_for(0))
        lb._last[t] = (1 << 32) | 13  # chain head points at a non-record
        lb.commit(t)
    log = lb.build()
    all_lsn = [int(x) for x in log.lsn] + [int(log.end_lsn), int(log.end_lsn) + 64]

    sets, snaps = [], []
    for i in range(n_txn):
        rs = []
        nr = int(rng.integers(0, max_ranges + 1))
        for _ in range(nr):
            tb = (list(tables) + ["never_written", "unknown_tb"])[int(rng.integers(0, len(tables) + 2))]
            u = rng.random()
            if u < 0.08:
                rs.append(Range(tb, int(rng.choice([-1, -2, 0])), None, None, 1, 1, 1))
                continue
            ix = int(rng.integers(-1, n_ix + 1))
            kl = keylens[ix % len(keylens)] if ix >= 0 else 9

            def bound():
                k = key_for(max(ix, 0))
                m = int(rng.integers(0, len(k) + 6))
                return (k + bytes(rng.integers(0, 256, size=6).astype(np.uint8)))[:m]

            lk, rk = bound(), bound()
            if rng.random() < 0.5 and lk > rk:
                lk, rk = rk, lk
            lf = int(rng.random() < 0.1)
            rf = int(rng.random() < 0.1)
            rs.append(Range(tb, ix, None if lf and rng.random() < 0.5 else lk,
                            None if rf and rng.random() < 0.5 else rk, lf, rf,
                            int(rng.random() < 0.05)))
        if rng.random() < 0.5:
            rs.sort(key=lambda r: (r.tbname, -r.islocked, r.idxnum, r.lkey or b""))
        sets.append(rs)
        pool = all_lsn if rng.random() < 0.9 else [int(x) + 1 for x in log.lsn[:5]] or all_lsn
        snaps.append(pool[int(rng.integers(0, len(pool)))])
    return log, ReadSets.from_lists(sets, snaps, tbnames=lb.tbnames)


# ---------------------------------------------------------------------------
# config 4: Jepsen bank/register-style histories for the dependency graph
# ---------------------------------------------------------------------------
SEED_CONFIG4 = 0xC0FFEE04


@dataclasses.dataclass
class History:
    """Micro-ops of committed transactions.  txn ids are commit order; a read
    records the writer txn of the version it observed (-1 = initial value),
    as a Jepsen rw-register history with unique write values does."""
    txn: np.ndarray        # uint32[nops]
    key: np.ndarray        # uint64[nops]
    is_write: np.ndarray   # uint8[nops]
    observed: np.ndarray   # int64[nops]
    ntxn: int
    snap: Optional[np.ndarray] = None  # int64[ntxn] snapshot (reads see writers < snap)

    @property
    def nops(self) -> int:
        return int(len(self.txn))


def config4_history(seed: int = SEED_CONFIG4, n_txn: int = 1_000_000, n_keys: int = 100_000,
                    ops_per_txn: int = 4, write_frac: float = 0.5, concurrent_frac: float = 0.02,
                    max_lag: int = 64, zipf: float = 0.0) -> History:
    """Txn t commits t-th and reads from snapshot s_t: s_t = t for most txns
    (serial), s_t = t - lag (lag <= max_lag) for `concurrent_frac` of them, so
    stale reads create rw anti-dependencies (write skew / G2 cycles).  Every
    txn touches ops_per_txn distinct-ish keys; each op is a read (observes the
    latest writer < s_t) followed, with probability write_frac, by a write
    (the bank transfer shape: read-modify-write)."""
    rng = np.random.default_rng(seed)
    n = n_txn * ops_per_txn
    txn = np.repeat(np.arange(n_txn, dtype=np.uint32), ops_per_txn)
    if zipf > 0:
        key = (rng.zipf(1.0 + zipf, size=n) % n_keys).astype(np.uint64)
    else:
        key = rng.integers(0, n_keys, size=n, dtype=np.uint64)
    lag = np.where(rng.random(n_txn) < concurrent_frac, rng.integers(1, max_lag + 1, size=n_txn), 0)
    snap = np.maximum(np.arange(n_txn, dtype=np.int64) - lag, 0)
    w = rng.random(n) < write_frac
    # writes sorted by (key, txn) as one composite
    wc = np.sort((key[w] << np.uint64(32)) | txn[w].astype(np.uint64))
    rc = (key << np.uint64(32)) | np.repeat(snap, ops_per_txn).astype(np.uint64)
    qo = np.argsort(rc)  # sorted queries: searchsorted walks wc in order
    idx = np.empty(n, np.int64)
    idx[qo] = np.searchsorted(wc, rc[qo], side="left")
    idx -= 1
    ok = idx >= 0
    cand = wc[np.maximum(idx, 0)]
    ok &= (cand >> np.uint64(32)) == key
    observed = np.where(ok, (cand & np.uint64(0xFFFFFFFF)).astype(np.int64), -1)
    # op stream: each op is a read; written keys also get a write micro-op.
    # Per txn: its ops_per_txn reads, then its writes (in op order) -- placed
    # directly (the order of a stable sort by txn).
    P = ops_per_txn
    nw_t = w.reshape(n_txn, P).sum(axis=1)
    start = np.cumsum(P + nw_t) - (P + nw_t)
    pos_r = (np.repeat(start, P) + np.tile(np.arange(P), n_txn)).astype(np.int64)
    wi = np.nonzero(w)[0]
    wt = wi // P
    wk = np.arange(len(wi)) - (np.cumsum(nw_t) - nw_t)[wt]
    pos_w = start[wt] + P + wk
    m = n + len(wi)
    o_txn = np.empty(m, np.uint32)
    o_key = np.empty(m, np.uint64)
    o_w = np.empty(m, np.uint8)
    o_obs = np.empty(m, np.int64)
    o_txn[pos_r], o_key[pos_r], o_w[pos_r], o_obs[pos_r] = txn, key, 0, observed
    o_txn[pos_w], o_key[pos_w], o_w[pos_w], o_obs[pos_w] = txn[wi], key[wi], 1, -1
    return History(o_txn, o_key, o_w, o_obs, n_txn, snap)


@dataclasses.dataclass
class HistoryWindow:
    """A History as the validator sees it: txn i commits
    at LSN commit_lsn[i]; the window holds every write (int64 key value, commit
    LSN); txn t's reads are point ranges of read set t at the snapshot LSN just
    below commit snap[t] -- so the join's (t, writer) pairs are exactly the
    writers a read of t did not see, the history's rw antidependencies."""
    keys: np.ndarray        # int64[nw] window rows
    lsn: np.ndarray         # uint64[nw]
    readsets: ReadSets      # one read set per txn (txn order; empty without reads)
    commit_lsn: np.ndarray  # uint64[ntxn] strictly increasing
    end_lsn: int


def history_window(h: History) -> HistoryWindow:
    assert h.snap is not None, "history without snapshots"
    commit = lsn_of_index(np.arange(h.ntxn + 1, dtype=np.uint64))
    w = h.is_write != 0
    keys = h.key[w].astype(np.int64)
    lsn_w = commit[h.txn[w].astype(np.int64)]
    r = np.nonzero(~w)[0]
    rt = h.txn[r].astype(np.int64)
    order = np.argsort(rt, kind="stable")
    r, rt = r[order], rt[order]
    nr = len(r)
    txn_off = np.zeros(h.ntxn + 1, np.int64)
    np.add.at(txn_off, rt + 1, 1)
    txn_off = np.cumsum(txn_off)
    snap_i = np.asarray(h.snap, np.int64)
    snap = np.where(snap_i > 0, commit[np.maximum(snap_i - 1, 0)], np.uint64(0)).astype(np.uint64)
    kb = F.enc_int64_array(h.key[r].astype(np.int64)).reshape(-1)
    off = np.arange(nr, dtype=np.uint64) * np.uint64(9)
    z = np.zeros(nr, np.int32)
    rs = ReadSets(txn_off=txn_off, snap=snap, table=z.copy(), idxnum=z.copy(), lflag=z.copy(),
                  rflag=z.copy(), islocked=z.copy(), lkeylen=np.full(nr, 9, np.int32),
                  rkeylen=np.full(nr, 9, np.int32), lkey_off=off, rkey_off=off.copy(), keys=kb,
                  tbnames=["t1"])
    return HistoryWindow(keys, lsn_w, rs, commit[:h.ntxn].copy(), int(commit[h.ntxn]))


def history_to_edn(h: History, limit: Optional[int] = None) -> str:
    """Jepsen rw-register (Elle) style EDN, one completed txn per line:
    {:type :ok, :f :txn, :value [[:r k v] [:w k v]], :process p, :index i};
    write values are writer txn + 1 (unique per key), nil = initial."""
    lines = []
    starts = np.searchsorted(h.txn, np.arange(h.ntxn + 1))
    for t in range(h.ntxn if limit is None else min(limit, h.ntxn)):
        mops = []
        for i in range(starts[t], starts[t + 1]):
            k = int(h.key[i])
            if h.is_write[i]:
                mops.append(f"[:w {k} {t + 1}]")
            else:
                ob = int(h.observed[i])
                mops.append(f"[:r {k} {'nil' if ob < 0 else ob + 1}]")
        lines.append(f"{{:type :ok, :f :txn, :value [{' '.join(mops)}], :process {t % 16}, :index {t}}}")
    return "\n".join(lines)


def history_from_edn(text: str) -> History:
    """Parse the EDN above (only :ok txns, in history order = commit order)."""
    import re
    txn, key, isw, obs = [], [], [], []
    t = 0
    for line in text.splitlines():
        if ":type :ok" not in line:
            continue
        for kind, k, v in re.findall(r"\[:(r|w) (\d+) (nil|\d+)\]", line):
            txn.append(t)
            key.append(int(k))
            isw.append(1 if kind == "w" else 0)
            obs.append(-1 if (kind == "w" or v == "nil") else int(v) - 1)
        t += 1
    return History(np.array(txn, np.uint32), np.array(key, np.uint64), np.array(isw, np.uint8),
                   np.array(obs, np.int64), t)


# ---------------------------------------------------------------------------
# config 3: composite keys <= 64 B over 32 (table, index) groups
# ---------------------------------------------------------------------------
SEED_CONFIG3 = 0xC0FFEE03
SEED_CONFIG5 = 0xC0FFEE05

# per index: list of fields (kind, size, descending) -> ondisk key bytes
INDEX_SHAPES = [
    [("i64", 9, False)],                                               # 9 B
    [("i64", 9, False), ("i64", 9, True)],                             # 18 B
    [("str", 21, False), ("i64", 9, False)],                           # 30 B
    [("str", 31, False), ("i64", 9, True), ("i64", 9, False), ("i64", 9, False)],  # 58 B
]


def _enc_fields(rng, shape, n, vmax):
    """n keys of an index shape as uint8[n, L] (memcmp-ordered ondisk)."""
    cols = []
    for kind, size, desc in shape:
        if kind == "i64":
            v = rng.integers(0, vmax, size=n, dtype=np.int64)
            b = F.enc_int64_array(v)
        else:
            ln = rng.integers(1, size - 1, size=n)
            letters = rng.integers(ord("a"), ord("a") + 6, size=(n, size - 1)).astype(np.uint8)
            letters[np.arange(size - 1)[None, :] >= ln[:, None]] = 0
            b = np.concatenate([np.full((n, 1), 8, np.uint8), letters], axis=1)
        cols.append(255 - b if desc else b)
    return np.concatenate(cols, axis=1)


@dataclasses.dataclass
class Config3Arrays:
    tbnames: List[str]
    groups: List[Tuple[str, int, int]]  # group g = (table, index, key length)
    keys_of: List[np.ndarray]           # uint8[gsize, L_g] per group
    w_group: np.ndarray                 # int64[n_writes] group of each index write (log order)
    w_row: np.ndarray                   # int64[n_writes] row in keys_of[group]
    w_lsn: np.ndarray                   # uint64[n_writes] regop LSN of the write's commit
    dta: List[Tuple[int, int]]          # (commit, table) of the data-row writes
    commit_lsn: np.ndarray              # uint64[n_commits]
    table_max: np.ndarray               # uint64[n_tables] max commit LSN of any write
    end_lsn: int
    readsets: ReadSets
    keys_per_commit: int

    def window(self, groups=None):
        """Window rows (gid u32[n], words u64[W][n], lsn u64[n]) in log order
        for the given group ids (all if None); gid = group index, W from the
        longest key of any group."""
        W = (max(L for _, _, L in self.groups) + 7) // 8
        sel = np.ones(len(self.w_group), bool) if groups is None else np.isin(self.w_group, list(groups))
        g, r, lsn = self.w_group[sel], self.w_row[sel], self.w_lsn[sel]
        pad = np.zeros((len(g), 8 * W), dtype=np.uint8)
        for gg in np.unique(g):
            m = g == gg
            kb = self.keys_of[gg][r[m]]
            pad[m, :kb.shape[1]] = kb
        words = pad.view(">u8").astype(np.uint64).reshape(len(g), W).T.copy()
        return g.astype(np.uint32), words, lsn.copy()


def config3_group_sizes(rng, n_groups: int, n_writes: int) -> np.ndarray:
    """Log-normal group sizes of config 3 (the first draw of its generator)."""
    w = rng.lognormal(0.0, 1.0, size=n_groups)
    return np.maximum(1, (w / w.sum() * n_writes).astype(np.int64))


def config3_group_keys(seed: int, g: int, n_ix: int, size: int, vmax: int) -> np.ndarray:
    """Group g's distinct-row keys (each written once), from its own stream:
    one group's keys can be drawn without the others'."""
    return _enc_fields(np.random.default_rng([seed, 3, g]), INDEX_SHAPES[g % n_ix], size, vmax)


def config3_arrays(seed: int = SEED_CONFIG3, n_tables: int = 8, n_ix: int = 4,
                   n_writes: int = 200_000, keys_per_commit: int = 8, n_txn: int = 20_000,
                   ranges_per_txn: int = 10, vmax: int = 1 << 12, snap_recent: float = 0.01,
                   lock_frac: float = 0.01, rs_seed: Optional[int] = None,
                   range_rows: int = 8, prefix_drop: int = 2) -> Config3Arrays:
    """Config 3 as arrays (no log): n_tables x n_ix composite-key groups with
    log-normal sizes, commits of keys_per_commit index writes (30% also write
    a data row of a random table), LSNs exactly as LogBuilder assigns them
    (ltran_start, writes, [dta], ltran_commit, regop; 64 bytes apart), and
    read sets of point / range / prefix ranges (and a few table locks) over
    1-3 tables each.  config3() builds the same workload as a log.  rs_seed
    draws the read sets from their own generator (another batch over the same
    window).  range_rows > 0: a range spans 1..range_rows neighbouring keys of
    its group (in key order) instead of two random keys, and prefix_drop > 0:
    a prefix range drops 1..prefix_drop trailing bytes of a key instead of
    keeping a random 1..L-1 of them -- narrow read sets, as config 2's
    (conflict rate 20-60 %)."""
    rng = np.random.default_rng(seed)
    tb = [f"t{i}" for i in range(n_tables)]
    G = n_tables * n_ix
    gsize = config3_group_sizes(rng, G, n_writes)
    keys_of = [config3_group_keys(seed, g, n_ix, int(gsize[g]), vmax) for g in range(G)]
    gid = np.concatenate([np.full(int(gsize[g]), g) for g in range(G)])
    row = np.concatenate([np.arange(int(gsize[g])) for g in range(G)])
    perm = rng.permutation(len(gid))
    gid, row = gid[perm], row[perm]
    K = keys_per_commit
    n_commits = (len(gid) + K - 1) // K
    dta = []
    nrec = np.zeros(n_commits, dtype=np.int64)
    for c in range(n_commits):
        k = min(K, len(gid) - c * K)
        has = rng.random() < 0.3
        if has:
            dta.append((c, int(rng.integers(0, n_tables))))
        nrec[c] = 1 + k + (1 if has else 0) + 2
    # record index of each commit's regop (LogBuilder: file 1, offset 28 + 64 i)
    regop_idx = np.cumsum(nrec) - 1
    assert 28 + 64 * int(nrec.sum()) < (1 << 32) - 64, "one log file"
    commit_lsn = (np.uint64(1) << np.uint64(32)) | (np.uint64(28) + np.uint64(64) * regop_idx.astype(np.uint64))
    start_lsn = int(lsn(1, 28))
    end_lsn = int(lsn(1, 28 + 64 * int(nrec.sum())))
    w_lsn = np.repeat(commit_lsn, K)[:len(gid)]
    table_max = np.zeros(n_tables, dtype=np.uint64)
    np.maximum.at(table_max, gid // n_ix, w_lsn)
    for c, t in dta:
        table_max[t] = max(table_max[t], commit_lsn[c])
    commits = [start_lsn] + [int(x) for x in commit_lsn]
    recent = max(1, int(len(commits) * snap_recent))
    if rs_seed is not None:
        rng = np.random.default_rng([seed, rs_seed])
    sorted_keys = None
    if range_rows > 0:
        sorted_keys = [kg[np.lexsort(kg.T[::-1])] for kg in keys_of]
    sets, snaps = [], []
    for t in range(n_txn):
        rs = []
        for tt in sorted(rng.choice(n_tables, size=int(rng.integers(1, 4)), replace=False)):
            if rng.random() < lock_frac:
                rs.append(Range.locked(tb[tt]))
                continue
            for _ in range(max(1, ranges_per_txn // 3)):
                ix = int(rng.integers(0, n_ix))
                g = tt * n_ix + ix
                a = bytes(keys_of[g][int(rng.integers(0, len(keys_of[g])))])
                u = rng.random()
                if u < 0.5:
                    rs.append(Range(tb[tt], ix, a, a))
                elif u < 0.8:
                    if sorted_keys is not None:
                        sk = sorted_keys[g]
                        i = int(rng.integers(0, len(sk)))
                        j = min(len(sk) - 1, i + int(rng.integers(0, range_rows)))
                        rs.append(Range(tb[tt], ix, bytes(sk[i]), bytes(sk[j])))
                    else:
                        b = bytes(keys_of[g][int(rng.integers(0, len(keys_of[g])))])
                        rs.append(Range(tb[tt], ix, min(a, b), max(a, b)))
                else:
                    if prefix_drop > 0:
                        p = a[: max(1, len(a) - int(rng.integers(1, prefix_drop + 1)))]
                    else:
                        p = a[: int(rng.integers(1, len(a)))]
                    rs.append(Range(tb[tt], ix, p, p))
        rs.sort(key=lambda r: (r.tbname, -r.islocked, r.idxnum, r.lkey or b""))
        sets.append(rs)
        snaps.append(commits[len(commits) - 1 - int(rng.integers(0, recent))])
    groups = [(tb[g // n_ix], g % n_ix, int(keys_of[g].shape[1])) for g in range(G)]
    return Config3Arrays(tb, groups, keys_of, gid, row, w_lsn, dta, commit_lsn, table_max,
                         end_lsn, ReadSets.from_lists(sets, snaps, tbnames=tb), K)


def config3(seed: int = SEED_CONFIG3, n_tables: int = 8, n_ix: int = 4, n_writes: int = 200_000,
            keys_per_commit: int = 8, n_txn: int = 20_000, ranges_per_txn: int = 10,
            vmax: int = 1 << 12, snap_recent: float = 0.01, lock_frac: float = 0.01,
            range_rows: int = 8, prefix_drop: int = 2):
    """Log of commits writing composite index keys (upd_ix) plus dta records
    over n_tables x n_ix groups with log-normal group sizes, and read sets of
    point / range / prefix ranges (and a few full-scan table locks) over 1-3
    tables each (ranges sorted per table like coalesced arrays).  Returns
    (LLog, ReadSets); config3_arrays() is the same workload as arrays."""
    a = config3_arrays(seed, n_tables, n_ix, n_writes, keys_per_commit, n_txn, ranges_per_txn,
                       vmax, snap_recent, lock_frac, range_rows=range_rows, prefix_drop=prefix_drop)
    n_ix_ = n_ix
    lb = LogBuilder(a.tbnames)
    dta = dict(a.dta)
    K = a.keys_per_commit
    for c in range(len(a.commit_lsn)):
        lb.begin(c)
        for g, r in zip(a.w_group[c * K:(c + 1) * K], a.w_row[c * K:(c + 1) * K]):
            lb.write(c, F.REC_UNDO_UPD_IX, a.tbnames[g // n_ix_], int(g % n_ix_), bytes(a.keys_of[g][r]))
        if c in dta:
            lb.write(c, F.REC_UNDO_UPD_DTA, a.tbnames[dta[c]])
        l = lb.commit(c)
        assert l == int(a.commit_lsn[c])
    return lb.build(), a.readsets


def config3_log(a: Config3Arrays, from_commit: int = 0) -> LLog:
    """The log of config3_arrays' workload (the records config3() logs, with
    the same LSNs), vectorised, from commit `from_commit` on: a tail of the
    log is enough for the oracle to check read sets whose snapshots fall
    inside it (each check only reads records after its snapshot)."""
    n_tab = len(a.tbnames)
    n_ix = len(a.groups) // n_tab
    K = a.keys_per_commit
    nc = len(a.commit_lsn)
    kc = np.minimum(K, len(a.w_group) - np.arange(nc, dtype=np.int64) * K)
    has = np.zeros(nc, bool)
    dt = np.full(nc, -1, np.int64)
    for c, t in a.dta:
        has[c], dt[c] = True, t
    nrec = 1 + kc + has.astype(np.int64) + 2
    base = np.concatenate([[0], np.cumsum(nrec)[:-1]])
    c0 = int(from_commit)
    cs = np.arange(c0, nc)
    commit_of = np.repeat(cs, nrec[c0:])
    idx = base[c0] + np.arange(int(nrec[c0:].sum()), dtype=np.int64)
    j = idx - base[commit_of]
    k_of, n_of = kc[commit_of], nrec[commit_of]
    lsns = lsn_of_index(idx.astype(np.uint64))
    rectype = np.full(len(idx), F.REC_UNDO_UPD_IX, np.uint32)
    rectype[j == 0] = F.REC_LTRAN_START
    is_dta = has[commit_of] & (j == k_of + 1)
    rectype[is_dta] = F.REC_UNDO_UPD_DTA
    rectype[j == n_of - 2] = F.REC_LTRAN_COMMIT
    rectype[j == n_of - 1] = F.REC_TXN_REGOP
    prev = lsn_of_index(np.maximum(idx - 1, 0).astype(np.uint64))
    prev[j == 0] = 0
    is_ix = rectype == F.REC_UNDO_UPD_IX
    w = commit_of[is_ix] * K + (j[is_ix] - 1)
    g, r = a.w_group[w], a.w_row[w]
    table = np.full(len(idx), -1, np.int32)
    ix = np.zeros(len(idx), np.int16)
    table[is_ix] = (g // n_ix).astype(np.int32)
    ix[is_ix] = (g % n_ix).astype(np.int16)
    table[is_dta] = dt[commit_of[is_dta]].astype(np.int32)
    glen = np.array([kg.shape[1] for kg in a.keys_of], np.int64)
    klen = glen[g]
    koff = np.concatenate([[0], np.cumsum(klen)[:-1]]).astype(np.int64)
    blob = np.zeros(max(int(klen.sum()), 1), np.uint8)
    for gg in np.unique(g):
        m = g == gg
        L = int(glen[gg])
        blob[(koff[m][:, None] + np.arange(L)[None, :]).reshape(-1)] = a.keys_of[gg][r[m]].reshape(-1)
    key_off = np.zeros(len(idx), np.uint64)
    keylen = np.zeros(len(idx), np.int32)
    key_off[is_ix] = koff.astype(np.uint64)
    keylen[is_ix] = klen.astype(np.int32)
    regop = rectype == F.REC_TXN_REGOP
    assert np.array_equal(lsns[regop], a.commit_lsn[c0:])
    return LLog(lsns, rectype, prev, np.zeros(len(idx), np.int16), table, ix, key_off, keylen,
                blob, list(a.tbnames), int(a.end_lsn))


@dataclasses.dataclass
class Config5Scaled:
    keys: np.ndarray            # int64[n] this rank's segment of the log: written key values
    lsn: np.ndarray             # uint64[n] commit LSN of each row (log order)
    readsets: ReadSets          # global read sets (identical on every rank)
    range_keys: np.ndarray      # int64[nr] lower key value of every range (splitter sampling)
    end_lsn: int
    params: dict

    @property
    def gid(self) -> np.ndarray:
        return np.zeros(len(self.keys), dtype=np.uint32)

    @property
    def words(self) -> np.ndarray:
        return int64_words(self.keys)


def int64_words(vals: np.ndarray) -> np.ndarray:
    """int64 index-key values -> uint64[2][n] big-endian key words of their
    9-byte enc_int64 keys (db/types.c:766-771), zero padded to 16 bytes."""
    n = len(vals)
    pad = np.zeros((n, 16), dtype=np.uint8)
    pad[:, :9] = F.enc_int64_array(vals)
    return pad.view(">u8").astype(np.uint64).reshape(n, 2).T.copy()


def zipf_keys(rng, n: int, s: float, key_bits: int) -> np.ndarray:
    """n draws of a Zipf(s) law truncated to 2^key_bits keys: key k - 1 has
    probability ~ k^-s, so the hot keys are the smallest values (draws past
    the key space are redrawn)."""
    out = rng.zipf(s, size=n).astype(np.uint64)
    lim = np.uint64(1 << key_bits)
    bad = np.nonzero(out > lim)[0]
    while len(bad):
        out[bad] = rng.zipf(s, size=len(bad)).astype(np.uint64)
        bad = bad[out[bad] > lim]
    return (out - np.uint64(1)).astype(np.int64)


def config5_scaled(seed: int = SEED_CONFIG5, keys_per_gpu: int = 125_000_000,
                   keys_per_commit: int = 10, n_txn: int = 100_000, ranges_per_txn: int = 10,
                   zipf_s: float = 1.2, key_bits: int = 32, snap_recent: float = 0.01,
                   rank: int = 0, world: int = 1, window: bool = True,
                   hot_frac: float = 0.03) -> Config5Scaled:
    """Config 5 (a 1B-key log window, Zipf s = 1.2 over 2^32
    keys, ranges as config 2 scaled), weak-scaled: ONE global Zipf(s) law over
    2^key_bits key values (hot keys are the small values, so a fixed split of
    the key space puts nearly every distinct key and every hot range on rank
    0); the log is world x keys_per_gpu writes and rank r generates its
    segment -- global commits g = c * world + r, keys_per_commit writes each,
    config 2's LSN numbering.  Which rank owns which rows is decided later by
    sampled global splitters (shard.sampled_splitters / exchange_rows).  The
    read sets are global: config 2's kind mix over the whole key space, range
    width scaled to the mean key density (about 10 logged writes per range),
    a hot_frac share of the point ranges on Zipf-drawn hot keys.  window=False:
    another batch of read sets over the same log (no rows)."""
    K = keys_per_commit
    R = K + 3
    n_commits = keys_per_gpu // K
    n = n_commits * K if window else 0
    vals = zipf_keys(np.random.default_rng([seed, 5, rank]), n, zipf_s, key_bits)
    gcommit = np.arange(n // K, dtype=np.uint64) * np.uint64(world) + np.uint64(rank)
    lsn = np.repeat(lsn_of_index(gcommit * np.uint64(R) + np.uint64(R - 1)), K)
    end_lsn = int(lsn_of_index(np.array([world * n_commits * R]))[0])

    rng = np.random.default_rng([seed, 1 << 20])
    T = n_txn * world
    nr = T * ranges_per_txn
    space = 1 << key_bits
    width = max(1, int(round(10 * space / max(world * n_commits * K, 1))))
    kind = rng.choice(4, size=nr, p=[0.5, 0.4, 0.08, 0.02])
    v = rng.integers(0, space, size=nr, dtype=np.int64)
    aim = np.nonzero((kind == 0) & (rng.random(nr) < hot_frac))[0]
    v[aim] = zipf_keys(rng, len(aim), zipf_s, key_bits)
    lo = F.enc_int64_array(v)
    hi = F.enc_int64_array(np.where(kind == 1, v + width, v))
    lkeylen = np.full(nr, 9, dtype=np.int32)
    rkeylen = np.full(nr, 9, dtype=np.int32)
    plen = rng.integers(6, 8, size=nr).astype(np.int32)
    lkeylen[kind == 2] = plen[kind == 2]
    rkeylen[kind == 2] = plen[kind == 2]
    lflag = np.zeros(nr, dtype=np.int32)
    rflag = np.zeros(nr, dtype=np.int32)
    side = rng.random(nr) < 0.5
    lflag[(kind == 3) & side] = 1
    rflag[(kind == 3) & ~side] = 1
    lkeylen[lflag == 1] = 0
    rkeylen[rflag == 1] = 0
    order = ranges_in_set_order(np.where(lflag == 1, -1, v), T, ranges_per_txn)
    lo, hi, v = lo[order], hi[order], v[order]
    lkeylen, rkeylen, lflag, rflag = lkeylen[order], rkeylen[order], lflag[order], rflag[order]
    keys = np.concatenate([lo.reshape(-1), hi.reshape(-1)])
    ncg = world * n_commits
    recent = max(1, int(round(ncg * snap_recent)))
    gi = np.uint64(ncg - 1) - rng.integers(0, recent, size=T).astype(np.uint64)
    snap = lsn_of_index(gi * np.uint64(R) + np.uint64(R - 1))
    rs = ReadSets(txn_off=np.arange(0, nr + 1, ranges_per_txn, dtype=np.int64), snap=snap,
                  table=np.zeros(nr, np.int32), idxnum=np.zeros(nr, np.int32), lflag=lflag,
                  rflag=rflag, islocked=np.zeros(nr, np.int32), lkeylen=lkeylen,
                  rkeylen=rkeylen, lkey_off=np.arange(nr, dtype=np.uint64) * np.uint64(9),
                  rkey_off=np.uint64(nr * 9) + np.arange(nr, dtype=np.uint64) * np.uint64(9),
                  keys=keys, tbnames=["t1"])
    range_keys = np.where(lflag == 1, np.int64(-(1 << 63)), v)
    return Config5Scaled(vals, lsn, rs, range_keys, end_lsn,
                         dict(seed=seed, keys_per_gpu=n, zipf_s=zipf_s, key_bits=key_bits,
                              width=width, n_txn=n_txn, rank=rank, world=world,
                              keys_per_commit=K))


def config5_log(segments: Sequence[np.ndarray], keys_per_commit: int = 10,
                from_commit: int = 0, commit_base: int = 0) -> LLog:
    """The global log of config5_scaled's per-rank key segments (rank r's
    commit c is global commit c * world + r): per commit ltran_start, one
    undo_upd_ix per key, ltran_commit, regop -- the LSNs config5_scaled gives
    its rows and snapshots -- from global commit `from_commit` on (a tail
    serves read sets whose snapshots fall inside it).  For oracle checks.
    commit_base: the segments are the ranks' tails from their local commit
    commit_base on (global commit (commit_base + c) * world + r).  Config 2's
    sharded log has the same layout (config2(world=...) key_values)."""
    world, K = len(segments), keys_per_commit
    R = K + 3
    n_commits = len(segments[0]) // K
    ncg = world * n_commits
    gkeys = np.stack([np.asarray(sg, np.int64).reshape(n_commits, K) for sg in segments], axis=1)
    gkeys = gkeys.reshape(ncg * K)[from_commit * K:]  # global commit order: (c, r) -> c * world + r
    nrec = (ncg - from_commit) * R
    first = commit_base * world + from_commit  # global index of the first commit kept
    idx = np.arange(nrec, dtype=np.uint64) + np.uint64(first * R)
    lsns = lsn_of_index(idx)
    j = (idx % np.uint64(R)).astype(np.int64)
    rectype = np.full(nrec, F.REC_UNDO_UPD_IX, dtype=np.uint32)
    rectype[j == 0] = F.REC_LTRAN_START
    rectype[j == R - 2] = F.REC_LTRAN_COMMIT
    rectype[j == R - 1] = F.REC_TXN_REGOP
    prev = np.zeros(nrec, dtype=np.uint64)
    prev[1:] = lsns[:-1]
    prev[j == 0] = 0
    is_undo = (j >= 1) & (j <= K)
    key_off = np.zeros(nrec, dtype=np.uint64)
    key_off[is_undo] = np.arange((ncg - from_commit) * K, dtype=np.uint64) * np.uint64(9)
    return LLog(lsns, rectype, prev, np.zeros(nrec, np.int16),
                np.where(is_undo, 0, -1).astype(np.int32), np.zeros(nrec, np.int16), key_off,
                np.where(is_undo, 9, 0).astype(np.int32), F.enc_int64_array(gkeys).reshape(-1),
                ["t1"], int(lsn_of_index(np.array([(commit_base * world + ncg) * R]))[0]))


def config5(seed: int = SEED_CONFIG5, n_commits: int = 100_000, keys_per_commit: int = 10,
            n_txn: int = 10_000, zipf_s: float = 1.2, key_bits: int = 32, **kw) -> Config2:
    """Config 2's shape with Zipf(s) hot keys over 2^key_bits: a few keys take
    most writes (they collapse under dedupe) and ranges cluster on hot tiles."""
    c2 = config2(seed=seed, n_commits=n_commits, keys_per_commit=keys_per_commit, n_txn=n_txn,
                 value_bits=key_bits, build_log=False, **kw)
    rng = np.random.default_rng([seed, 5])
    z = rng.zipf(zipf_s, size=n_commits * keys_per_commit).astype(np.uint64)
    hot = ((z * np.uint64(0x9E3779B1)) & np.uint64((1 << key_bits) - 1)).astype(np.int64)
    K = keys_per_commit
    R = K + 3
    nrec = n_commits * R
    idx = np.arange(nrec, dtype=np.uint64)
    lsns = lsn_of_index(idx)
    j = (idx % np.uint64(R)).astype(np.int64)
    rectype = np.full(nrec, F.REC_UNDO_UPD_IX, dtype=np.uint32)
    rectype[j == 0] = F.REC_LTRAN_START
    rectype[j == R - 2] = F.REC_LTRAN_COMMIT
    rectype[j == R - 1] = F.REC_TXN_REGOP
    prev = np.zeros(nrec, dtype=np.uint64)
    prev[1:] = lsns[:-1]
    prev[j == 0] = 0
    is_undo = (j >= 1) & (j <= K)
    key_off = np.zeros(nrec, dtype=np.uint64)
    key_off[is_undo] = np.arange(n_commits * K, dtype=np.uint64) * np.uint64(9)
    log = LLog(lsns, rectype, prev, np.zeros(nrec, np.int16), np.where(is_undo, 0, -1).astype(np.int32),
               np.zeros(nrec, np.int16), key_off, np.where(is_undo, 9, 0).astype(np.int32),
               F.enc_int64_array(hot).reshape(-1), ["t1"], int(lsn_of_index(np.array([nrec]))[0]))
    # point ranges aim at the hot keys half of the time
    rs = c2.readsets
    pts = (rs.lkeylen == 9) & (rs.rkeylen == 9)
    sel = np.nonzero(pts & (rng.random(len(pts)) < 0.5))[0]
    keys = rs.keys.copy().reshape(-1)
    hk = F.enc_int64_array(hot[rng.integers(0, len(hot), size=len(sel))])
    for side in ("lkey_off", "rkey_off"):
        off = getattr(rs, side)[sel].astype(np.int64)
        keys[(off[:, None] + np.arange(9)[None, :]).reshape(-1)] = hk.reshape(-1)
    rs = dataclasses.replace(rs, keys=keys)
    return Config2(log, rs, lsns[R - 1::R].copy(), hot, dict(c2.params, zipf_s=zipf_s))
