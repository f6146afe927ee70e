"""Test-only model of the GPU join at the probe level: evaluates marshalled
probes (as produced by the native marshaller) against the committed-write
window decoded in Python.  Used on CPU to check marshalling + join semantics
(and the sharded routing/merge) against the oracle without a GPU."""
import bisect
from collections import defaultdict

import numpy as np

from comdb2_amd import formats as F


def committed_writes(log):
    """[(regop lsn, [(tbname, ix, key|None)], broken)], dangling regop lsns."""
    lsn = [int(x) for x in log.lsn]
    pos = {l: i for i, l in enumerate(lsn)}
    commits, dangling = [], []
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
    return commits, dangling


class WindowModel:
    """Deduplicated window: (tbname, ix, klen) -> sorted [(words, max lsn)]."""

    def __init__(self, log, key_filter=None):
        commits, _ = committed_writes(log)
        self.table_max = defaultdict(int)
        rows = defaultdict(dict)
        for c, writes, _ in commits:
            for tb, ix, key in writes:
                self.table_max[tb] = max(self.table_max[tb], c)
                if key is None or (key_filter and not key_filter(tb, ix, key)):
                    continue
                d = rows[(tb, ix, len(key))]
                d[key] = max(d.get(key, 0), c)
        self.groups = {}
        for g, d in rows.items():
            items = sorted(d.items())
            self.groups[g] = ([k for k, _ in items], [v for _, v in items])

    def probe(self, tb, ix, klen, lo_words, hi_words, snap, W):
        keys, lsns = self.groups.get((tb, ix, klen), ([], []))
        lo = b"".join(int(x).to_bytes(8, "big") for x in lo_words)[:klen]
        hi = b"".join(int(x).to_bytes(8, "big") for x in hi_words)[:klen]
        a = bisect.bisect_left(keys, lo)
        b = bisect.bisect_right(keys, hi)
        return any(v > snap for v in lsns[a:b])


def evaluate(v, m, model, table_max_by_name=None):
    """Verdict bytes of a marshalled batch m (Validator.marshal) from the model.
    v: the (host-only) Validator that marshalled m, for gid -> group names."""
    names = {}
    verdict = np.zeros(m["n_txn"], dtype=np.uint8)
    tmax = table_max_by_name if table_max_by_name is not None else model.table_max
    tbname = {}
    for i in range(m["n"]):
        g = int(m["gid"][i])
        if g not in names:
            tid, ix, kl = v.group_info(g)
            names[g] = (_tname(v, tid, tbname), ix, kl)
        tb, ix, kl = names[g]
        if model.probe(tb, ix, kl, m["lo"][:, i], m["hi"][:, i], int(m["snap"][i]), m["words"]):
            verdict[int(m["txn"][i])] = 1
    for i in range(m["n_lock"]):
        tb = _tname(v, int(m["lock_table"][i]), tbname)
        if tmax.get(tb, 0) > int(m["lock_snap"][i]):
            verdict[int(m["lock_txn"][i])] = 1
    return verdict


def _tname(v, tid, cache):
    if tid not in cache:
        cache[tid] = v.table_name(tid)
    return cache[tid]
