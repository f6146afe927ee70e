"""Test helpers: fixture loading and an independent pure-Python model of the
check (A0 of SURVEY.md §8(a), written as a set formula rather than as the
reference's walk) used to cross-check the C oracle on small cases."""
import json
import os

import numpy as np

from comdb2_amd import formats as F
from comdb2_amd.formats import LLog, Range, ReadSets
from comdb2_amd.workloads import Txn

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

WRITE_TYPES = {"upd_dta": F.REC_UNDO_UPD_DTA, "upd_ix": F.REC_UNDO_UPD_IX,
               "add_dta": F.REC_UNDO_ADD_DTA, "add_ix": F.REC_UNDO_ADD_IX,
               "del_dta": F.REC_UNDO_DEL_DTA, "del_ix": F.REC_UNDO_DEL_IX}


def serialstep():
    with open(os.path.join(GOLDEN, "serialstep.json")) as f:
        return json.load(f)


def scenario_events(sc):
    txns = {}
    for name, t in sc["txns"].items():
        reads = [Range(r["tb"], r["ix"], None if r["lkey"] is None else bytes.fromhex(r["lkey"]),
                       None if r["rkey"] is None else bytes.fromhex(r["rkey"]),
                       r["lflag"], r["rflag"], r["islocked"]) for r in t["reads"]]
        writes = [(WRITE_TYPES[w[0]], w[1], w[2], None if w[3] is None else bytes.fromhex(w[3]))
                  for w in t["writes"]]
        txns[name] = Txn(name, reads, writes)
    return [(ev, txns[n]) for ev, n in sc["events"]]


def _mc(a, b, n):
    a, b = a[:n], b[:n]
    return (a > b) - (a < b)


def model_check(log: LLog, rs: ReadSets, regop_only=0):
    """Set-formula model: rc(t) = 1 iff S valid-and-before-end and there is a
    committed write txn after S whose writes hit the read set (or an error
    along the way).  Returns (rc, post_lsn)."""
    lsn = [int(x) for x in log.lsn]
    pos = {l: i for i, l in enumerate(lsn)}
    end = int(log.end_lsn)
    # committed write txns: (regop lsn, [writes], broken)
    commits = []
    dangling = []
    for i, t in enumerate(log.rectype):
        if int(t) not in F.REGOP_TYPES:
            continue
        p = pos.get(int(log.prev[i]))
        if p is None:
            dangling.append(lsn[i])
            continue
        if int(log.rectype[p]) != F.REC_LTRAN_COMMIT:
            continue
        if (int(log.prev[p]) >> 32) == 0 or int(log.isabort[p]):
            continue
        writes, broken, cur = [], False, int(log.prev[p])
        while True:
            r = pos.get(cur)
            if r is None:
                broken = True
                break
            rt = int(log.rectype[r])
            if rt == F.REC_LTRAN_START:
                break
            if rt in F.DTA_TYPES:
                writes.append((log.tbnames[log.table[r]], -2, None))
            elif rt in F.IX_TYPES:
                o, n = int(log.key_off[r]), int(log.keylen[r])
                writes.append((log.tbnames[log.table[r]], int(log.ix[r]), bytes(log.keys[o:o + n])))
            cur = int(log.prev[r])
            if (cur >> 32) == 0:
                break
        commits.append((lsn[i], writes, broken))
    rc = np.zeros(rs.ntxn, dtype=np.int32)
    post = np.zeros(rs.ntxn, dtype=np.uint64)
    for t in range(rs.ntxn):
        S = int(rs.snap[t])
        post[t] = S if regop_only else end
        if S >= end:
            continue
        if S not in pos:
            rc[t] = 1
            continue
        if any(d > S for d in dangling):
            rc[t] = 1
            continue
        later = [c for c in commits if c[0] > S]
        if regop_only:
            rc[t] = int(bool(later))
            continue
        rows = range(int(rs.txn_off[t]), int(rs.txn_off[t + 1]))
        ranges = []
        for r in rows:
            lk = bytes(rs.keys[int(rs.lkey_off[r]): int(rs.lkey_off[r]) + int(rs.lkeylen[r])])
            rk = bytes(rs.keys[int(rs.rkey_off[r]): int(rs.rkey_off[r]) + int(rs.rkeylen[r])])
            ranges.append((rs.tbnames[rs.table[r]], int(rs.idxnum[r]), lk, rk, int(rs.lflag[r]),
                           int(rs.rflag[r]), int(rs.islocked[r])))
        first_lock, span = {}, {}
        for i, r in enumerate(ranges):
            first_lock.setdefault(r[0], r[6])
            b, e = span.get((r[0], r[1]), (i, i))
            span[(r[0], r[1])] = (b, i)

        def hit(tb, ix, key):
            if not ranges or tb not in first_lock:
                return False
            if first_lock[tb]:
                return True
            if key is None or (tb, ix) not in span:
                return False
            b, e = span[(tb, ix)]
            for r in ranges[b:e + 1]:
                lo_ok = r[4] or _mc(r[2], key, min(len(r[2]), len(key))) <= 0
                hi_ok = r[5] or _mc(key, r[3], min(len(r[3]), len(key))) <= 0
                if lo_ok and hi_ok:
                    return True
            return False

        for c, writes, broken in later:
            if any(hit(*w) for w in writes) or broken:
                rc[t] = 1
                break
    return rc, post
