"""Incremental window, host side (hsc_window_append_log on host-only
contexts): a log taken in pieces -- a prefix ingested, the rest appended in
chunks, logical chains reaching back across the pieces -- leaves the window
in the state the whole log does: table maxima, max commit, end LSN, key groups
and the marshalled probes / forced verdicts of every read set (the
DB_SET-on-a-non-record and broken-chain rules included)."""
import numpy as np
import pytest

from comdb2_amd.formats import LLog
from comdb2_amd.hsc import Validator
from comdb2_amd.workloads import random_case


def log_slice(log: LLog, a: int, b: int) -> LLog:
    """Records [a, b) of log; the end is the next record's LSN (or the log's)."""
    end = int(log.lsn[b]) if b < log.nrec else int(log.end_lsn)
    return LLog(lsn=log.lsn[a:b], rectype=log.rectype[a:b], prev=log.prev[a:b],
                isabort=log.isabort[a:b], table=log.table[a:b], ix=log.ix[a:b],
                key_off=log.key_off[a:b], keylen=log.keylen[a:b], keys=log.keys,
                tbnames=list(log.tbnames), end_lsn=end)


def state(v: Validator, rs):
    m = v.marshal(rs)
    return (v.table_max().tolist(), v.lib.hsc_window_max_commit(v.ctx), v.end_lsn,
            {k: (m[k].tolist() if hasattr(m[k], "tolist") else m[k]) for k in m})


@pytest.mark.parametrize("seed", range(10))
def test_append_log_in_pieces_equals_whole_log(seed):
    log, rs = random_case(300 + seed, n_commits=80, broken=(seed % 3 == 0))
    whole = Validator(-1)
    whole.ingest_log(log)
    want = state(whole, rs)
    whole.close()
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(1, log.nrec, size=4).tolist()))
    pieces = [0] + cuts + [log.nrec]
    v = Validator(-1)
    v.ingest_log(log_slice(log, 0, pieces[1]))
    for a, b in zip(pieces[1:], pieces[2:]):
        v.append_log(log_slice(log, a, b))
    got = state(v, rs)
    v.close()
    assert got == want


def test_append_log_rejects_going_back():
    log, _ = random_case(7, n_commits=20)
    v = Validator(-1)
    v.ingest_log(log_slice(log, 0, log.nrec // 2))
    with pytest.raises(Exception):
        v.append_log(log_slice(log, 0, 3))  # LSNs below the stored ones
    v.close()
