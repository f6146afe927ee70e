"""CPU: pin the oracle (C restatement of bdb_osql_serial_check) against the
reference's own known answers (tests/serialstep.test, restated in
tests/golden/serialstep.json) and against an independent set-formula model."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.workloads import config1_events, config2, random_case, replay
from helpers import model_check, scenario_events, serialstep


def oracle_checker(o):
    return lambda log, rs: o.check(log, rs)[0]


@pytest.mark.parametrize("name", sorted(serialstep()))
def test_serialstep_known_answers(oracle_mod, name):
    sc = serialstep()[name]
    rcs = replay(scenario_events(sc), oracle_checker(oracle_mod))
    failed = sorted(t for t, rc in rcs.items() if rc)
    assert failed == sorted(sc["expect_fail"])
    assert len(failed) == sc["reference_failures"]


def test_serialstep_model_agrees():
    for name, sc in serialstep().items():
        rcs = replay(scenario_events(sc), lambda log, rs: model_check(log, rs)[0])
        assert sorted(t for t, rc in rcs.items() if rc) == sorted(sc["expect_fail"]), name


@pytest.mark.parametrize("seed", range(12))
def test_oracle_vs_model_random(oracle_mod, seed):
    log, rs = random_case(seed, broken=(seed % 3 == 0))
    for regop_only in (0, 1):
        rc, post, _ = oracle_mod.check(log, rs, regop_only=regop_only)
        mrc, mpost = model_check(log, rs, regop_only=regop_only)
        np.testing.assert_array_equal(rc != 0, mrc != 0)
        np.testing.assert_array_equal(post, mpost)


def _one(oracle_mod, lb, ranges, snap, regop_only=0):
    log = lb.build()
    rs = ReadSets.from_lists([ranges], [snap], tbnames=lb.tbnames)
    rc, post, _ = oracle_mod.check(log, rs, regop_only=regop_only)
    return int(rc[0] != 0), int(post[0]), log


def test_min_length_memcmp_prefix(oracle_mod):
    lb = LogBuilder(["t"])
    s = lb.next_lsn()
    lb.begin(1)
    lb.write(1, F.REC_UNDO_UPD_IX, "t", 0, F.enc_int64(5) + F.enc_int64(7))
    lb.commit(1)
    pre = F.enc_int64(5)
    assert _one(oracle_mod, lb, [Range("t", 0, pre, pre)], s)[0] == 1        # prefix hit
    assert _one(oracle_mod, lb, [Range("t", 0, F.enc_int64(6), None, 0, 1)], s)[0] == 0
    long_lo = F.enc_int64(5) + F.enc_int64(7) + b"\xff"                        # longer than key
    assert _one(oracle_mod, lb, [Range("t", 0, long_lo, long_lo)], s)[0] == 1  # truncated compare
    assert _one(oracle_mod, lb, [Range("t", 0, b"", b"")], s)[0] == 1          # zero-length bounds
    assert _one(oracle_mod, lb, [Range("t", 1, pre, pre)], s)[0] == 0          # other index


def test_span_quirk_and_first_range_lock(oracle_mod):
    lb = LogBuilder(["a", "b"])
    s = lb.next_lsn()
    lb.begin(1)
    lb.write(1, F.REC_UNDO_ADD_IX_LK, "a", 0, F.enc_int64(10))
    lb.write(1, F.REC_UNDO_DEL_DTA, "a")
    lb.commit(1)
    k = F.enc_int64
    # a's ix0 span covers array slots 0..2, including b's range [10,10]
    unsorted = [Range("a", 0, k(5), k(5)), Range("b", 0, k(10), k(10)), Range("a", 0, k(7), k(7))]
    assert _one(oracle_mod, lb, unsorted, s)[0] == 1
    assert _one(oracle_mod, lb, [unsorted[0], unsorted[2], unsorted[1]], s)[0] == 0
    # islocked comes from the table's FIRST range: a later locked range is ignored
    assert _one(oracle_mod, lb, [Range("a", 1, k(0), k(0)), Range.locked("a")], s)[0] == 0
    assert _one(oracle_mod, lb, [Range.locked("a"), Range("a", 1, k(0), k(0))], s)[0] == 1


def test_window_rules(oracle_mod):
    lb = LogBuilder(["t"])
    s0 = lb.next_lsn()
    k = F.enc_int64(1)
    lb.begin(1)
    lb.write(1, F.REC_UNDO_UPD_IX, "t", 0, k)
    lb.commit(1, isabort=1)                       # aborted: ignored
    lb.commit(2, empty=True)                      # read-only logical txn: ignored
    st = lb.begin(3)
    lb.raw(F.REC_TXN_REGOP, prev=st)              # regop not pointing at a commit
    r = [Range("t", 0, k, k)]
    rc, post, log = _one(oracle_mod, lb, r, s0)
    assert rc == 0 and post == int(log.end_lsn)   # full mode moves the LSN to the end
    assert _one(oracle_mod, lb, r, s0, regop_only=1)[:2] == (0, s0)
    lb.begin(4)
    lb.write(4, F.REC_UNDO_UPD_IX, "t", 0, k)
    c4 = lb.commit(4)
    assert _one(oracle_mod, lb, r, s0)[0] == 1
    assert _one(oracle_mod, lb, r, c4)[0] == 0    # snapshot at the commit itself
    assert _one(oracle_mod, lb, [], s0)[0] == 0   # empty read set never conflicts
    assert _one(oracle_mod, lb, r, s0, regop_only=1)[0] == 1
    end = int(lb.build().end_lsn)
    assert _one(oracle_mod, lb, r, end)[0] == 0   # at end of log: DB_NOTFOUND -> 0
    assert _one(oracle_mod, lb, r, s0 + 1)[0] == 1  # not a record LSN: cursor error


def test_config1_replay_small(oracle_mod):
    ev = config1_events(n_txn=200)
    rcs = replay(ev, oracle_checker(oracle_mod))
    mrcs = replay(ev, lambda log, rs: model_check(log, rs)[0])
    assert rcs == mrcs
    assert 0 < sum(rcs.values()) < len(rcs)


def test_config2_small_oracle_vs_model(oracle_mod):
    c2 = config2(n_commits=300, n_txn=60, value_bits=16, width=1 << 8, snap_recent=0.5)
    rc, _, _ = oracle_mod.check(c2.log, c2.readsets)
    mrc, _ = model_check(c2.log, c2.readsets)
    np.testing.assert_array_equal(rc != 0, mrc != 0)
