"""CPU: the vectorised logs of configs 3 and 5 (workloads.config3_log,
config5_log with from_commit) that the full-size GPU tests hand the oracle.
config3_log equals config3()'s LogBuilder log record for record, and a tail of
either log gives the oracle (oracle/serial_oracle.c) the verdicts of the
whole log for read sets whose snapshots fall inside the tail: each check only
reads records after its snapshot (bdb/serializable.c:390-539)."""
import numpy as np

from comdb2_amd.workloads import config3, config3_arrays, config3_log, config5_log, config5_scaled


def _same(a, b):
    for f in ("lsn", "rectype", "prev", "isabort", "table", "ix", "keylen"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    for i in range(a.nrec):
        ka = bytes(a.keys[int(a.key_off[i]):int(a.key_off[i]) + int(a.keylen[i])])
        kb = bytes(b.keys[int(b.key_off[i]):int(b.key_off[i]) + int(b.keylen[i])])
        assert ka == kb, i
    assert a.tbnames == b.tbnames and a.end_lsn == b.end_lsn


def test_config3_log_equals_the_builder_log():
    kw = dict(n_writes=6000, n_txn=200)
    log, _ = config3(**kw)
    _same(config3_log(config3_arrays(**kw)), log)


def test_config3_tail_gives_the_whole_logs_verdicts(oracle_mod):
    a = config3_arrays(n_writes=20000, n_txn=600)
    whole = config3_log(a)
    snaps = a.readsets.snap
    c0 = int(np.searchsorted(a.commit_lsn, snaps.min()))
    c0 = max(0, c0 - (0 if c0 < len(a.commit_lsn) and a.commit_lsn[c0] == snaps.min() else 1))
    tail = config3_log(a, from_commit=c0)
    assert tail.nrec < whole.nrec
    want, _, _ = oracle_mod.check(whole, a.readsets)
    got, _, _ = oracle_mod.check(tail, a.readsets)
    np.testing.assert_array_equal(got, want)
    assert 0.02 < (want != 0).mean() < 0.98


def test_config5_tail_gives_the_whole_logs_verdicts(oracle_mod):
    c5 = config5_scaled(keys_per_gpu=200_000, n_txn=500)
    whole = config5_log([c5.keys])
    R = 13
    regops = whole.lsn[R - 1::R]
    c0 = int(np.searchsorted(regops, c5.readsets.snap.min()))
    tail = config5_log([c5.keys], from_commit=c0)
    want, _, _ = oracle_mod.check(whole, c5.readsets)
    got, _, _ = oracle_mod.check(tail, c5.readsets)
    np.testing.assert_array_equal(got, want)
