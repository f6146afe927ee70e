"""Read/write conflict pairs before the OR-reduction (hsc_rw_edges,
comdb2_amd/csrc/hsc_edges.hip) against a Python
restatement over every committed write version of the log (the committed
writes as tests/probe_model.py decodes them), and: a read set has a pair
exactly when the oracle (oracle/serial_oracle.c) says it conflicts, for
read sets whose verdict comes from ranges alone."""
import os
import sys

import numpy as np
import pytest

from comdb2_amd.workloads import config2

sys.path.insert(0, os.path.dirname(__file__))
from probe_model import committed_writes  # noqa: E402
from test_gpu_narrow import keyed_case  # noqa: E402

pytestmark = pytest.mark.gpu


def words_of(key, W):
    b = bytes(key) + bytes(8 * W - len(key))
    return tuple(int.from_bytes(b[8 * j:8 * j + 8], "big") for j in range(W))


def expected_pairs(v, log, m):
    """Every (txn, commit) with a committed index write in one of the txn's
    marshalled ranges and commit > snapshot."""
    W = m["words"]
    commits, _ = committed_writes(log)
    by_group = {}
    for c, writes, _ in commits:
        for tb, ix, key in writes:
            if key is None:
                continue
            by_group.setdefault((tb, ix, len(key)), []).append((words_of(key, W), c))
    ginfo = {}
    pairs = set()
    for q in range(m["n"]):
        g = int(m["gid"][q])
        if g not in ginfo:
            tid, ix, kl = v.group_info(g)
            ginfo[g] = (v.table_name(tid), ix, kl)
        lo = tuple(int(x) for x in m["lo"][:, q])
        hi = tuple(int(x) for x in m["hi"][:, q])
        s = int(m["snap"][q])
        t = int(m["txn"][q])
        for w, c in by_group.get(ginfo[g], ()):
            if lo <= w <= hi and c > s:
                pairs.add((t, c))
    return sorted(pairs)


def check(v, oracle_mod, log, rs):
    v.ingest_log(log)
    m = v.marshal(rs)
    txn, lsn = v.rw_edges(rs)
    got = list(zip(txn.tolist(), lsn.tolist()))
    want = expected_pairs(v, log, m)
    assert got == want
    # the OR of a read set's pairs is its verdict (read sets without locks
    # or host-forced verdicts)
    verdict = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    has = np.zeros(rs.ntxn, bool)
    has[txn] = True
    plain = np.ones(rs.ntxn, bool)
    plain[m["lock_txn"]] = False
    plain &= m["forced"] == 0
    assert plain.sum() > 0
    np.testing.assert_array_equal(has[plain], verdict[plain])
    return len(got)


def test_rw_edges_config2(validator, oracle_mod):
    c2 = config2(n_commits=3000, n_txn=600, value_bits=16, width=1 << 8, snap_recent=0.3)
    assert check(validator, oracle_mod, c2.log, c2.readsets) > 100


def test_rw_edges_hot_keys_many_versions(validator, oracle_mod):
    """Few distinct keys, many versions each: a range sees every later version."""
    from comdb2_amd import formats as F
    from comdb2_amd.formats import Range
    key = lambda rng: F.enc_int64(int(rng.integers(0, 40)))

    def rng_range(rng):
        a = int(rng.integers(0, 40))
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(a + int(rng.integers(0, 4))))
    log, rs = keyed_case(5, 2000, 3, key, rng_range, 300, ranges_per_txn=3, snap_recent=0.2)
    assert check(validator, oracle_mod, log, rs) > 1000
