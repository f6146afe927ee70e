"""GPU pending tail (hsc_host.cpp pend_mirror / k_small_narrow's second
half): on a narrow window whose keys fit 4 words, an append's rows and raised
table maxima stay in mapped host memory that the small-batch kernel scans
beside the delta runs, until 256 rows wait or a batch that is not small merges
them into the live run.  Logs are appended a few records at a time and
checked after every piece against the oracle on the log so far -- small
batches (the tail scanned), a large batch (the tail merged first), wide keys
(no tail: every append merged), and a window of many tables whose first
writes arrive by append."""
import numpy as np
import pytest

from comdb2_amd.hsc import LAYOUT_NARROW
from comdb2_amd.workloads import random_case
from test_incremental import log_slice

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _clamped(rs, end_lsn):
    return rs.with_snaps(np.minimum(rs.snap, np.uint64(end_lsn)))


def _replay_pieces(v, oracle_mod, log, rs, pieces, big=None):
    v.ingest_log(log_slice(log, 0, pieces[1]))
    v.check_readsets(_clamped(rs, log.lsn[pieces[1] - 1]))
    for a, b in zip(pieces[1:], pieces[2:]):
        v.append_log(log_slice(log, a, b))
        sub = log_slice(log, 0, b)
        r = _clamped(rs, sub.lsn[-1])
        want, _, _ = oracle_mod.check(sub, r)
        got = v.check_readsets(r)
        np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"records [0, {b})")
        if big is not None and b % 7 == 0:  # a batch past the small path: the tail is merged
            rb = _clamped(big, sub.lsn[-1])
            wb, _, _ = oracle_mod.check(sub, rb)
            np.testing.assert_array_equal(v.check_readsets(rb) != 0, wb != 0, err_msg=f"big [0, {b})")


@pytest.mark.parametrize("seed", range(4))
def test_small_checks_scan_the_pending_tail(validator, oracle_mod, seed):
    log, rs = random_case(900 + seed, n_commits=300, n_txn=40, value_range=48)
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(40, log.nrec, size=120).tolist()))
    pieces = [0, 40] + [c for c in cuts if c > 40] + [log.nrec]
    _replay_pieces(validator, oracle_mod, log, rs, pieces)
    st = validator.append_stats()
    if validator.layout == LAYOUT_NARROW and validator.words <= 4:
        assert st["pending_appends"] > 0 and st["pending_merges"] > 0, st


def test_large_batches_merge_the_tail_first(validator, oracle_mod):
    log, rs = random_case(950, n_commits=200, n_txn=40, value_range=40)
    _, big = random_case(950, n_commits=200, n_txn=1500, value_range=40)  # same log, 1500 read sets
    cuts = list(range(60, log.nrec, 9))
    _replay_pieces(validator, oracle_mod, log, rs, [0] + cuts + [log.nrec], big=big)


def test_wide_keys_take_no_tail(validator, oracle_mod):
    log, rs = random_case(960, n_commits=150, n_txn=40, keylens=(40, 9), value_range=32)
    cuts = list(range(30, log.nrec, 11))
    before = validator.append_stats()["pending_appends"]
    _replay_pieces(validator, oracle_mod, log, rs, [0] + cuts + [log.nrec])
    if validator.words > 4:
        assert validator.append_stats()["pending_appends"] == before


def test_tables_first_written_by_appends(validator, oracle_mod):
    """The first piece writes few of the tables: later tables (and their
    maxima, read by locked read sets) arrive through appends only."""
    log, rs = random_case(970, n_commits=200, n_txn=60, tables=("ta", "tb", "tc", "td", "te", "tf"),
                          value_range=40)
    cuts = list(range(8, log.nrec, 5))
    _replay_pieces(validator, oracle_mod, log, rs, [0] + cuts + [log.nrec])
