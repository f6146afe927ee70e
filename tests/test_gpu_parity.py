"""GPU parity: the HIP join (through the C ABI) against the oracle, bit-exact on
verdicts and on the post-call (file, offset) side effect."""
import ctypes

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import CurRangeArrays, bdb_osql_serial_check
from comdb2_amd.workloads import config1_events, config2, random_case, replay
from helpers import scenario_events, serialstep

pytestmark = pytest.mark.gpu


def gpu_checker(v):
    def check(log, rs):
        v.ingest_log(log)
        return v.check_readsets(rs)
    return check


@pytest.mark.parametrize("seed", range(16))
def test_random_cases_flat(validator, oracle_mod, seed):
    log, rs = random_case(seed, broken=(seed % 4 == 0))
    want, _, _ = oracle_mod.check(log, rs)
    validator.ingest_log(log)
    got = validator.check_readsets(rs)
    np.testing.assert_array_equal(got != 0, want != 0)


@pytest.mark.parametrize("seed", range(8))
def test_random_cases_currangearr_batch(validator, oracle_mod, seed):
    log, rs = random_case(100 + seed, broken=(seed % 2 == 0), max_ranges=12)
    validator.ingest_log(log)
    sets, snaps = _to_lists(rs)
    for regop_only in (0, 1):
        want, want_post, _ = oracle_mod.check(log, rs, regop_only=regop_only)
        arrs = CurRangeArrays(sets, snaps)
        got = validator.check_batch(arrs, regop_only=regop_only)
        np.testing.assert_array_equal(got != 0, want != 0)
        post = np.array([(a.file << 32) | a.offset for a in arrs.arrs], dtype=np.uint64)
        np.testing.assert_array_equal(post, want_post)


def _to_lists(rs):
    sets = []
    for t in range(rs.ntxn):
        cur = []
        for r in range(int(rs.txn_off[t]), int(rs.txn_off[t + 1])):
            lk = bytes(rs.keys[int(rs.lkey_off[r]):int(rs.lkey_off[r]) + int(rs.lkeylen[r])])
            rk = bytes(rs.keys[int(rs.rkey_off[r]):int(rs.rkey_off[r]) + int(rs.rkeylen[r])])
            cur.append(Range(rs.tbnames[rs.table[r]], int(rs.idxnum[r]),
                             lk if rs.lkeylen[r] else None, rk if rs.rkeylen[r] else None,
                             int(rs.lflag[r]), int(rs.rflag[r]), int(rs.islocked[r])))
        sets.append(cur)
    return sets, [int(s) for s in rs.snap]


def test_single_call_entry(validator, oracle_mod):
    log, rs = random_case(7)
    validator.ingest_log(log)
    sets, snaps = _to_lists(rs)
    want, want_post, _ = oracle_mod.check(log, rs)
    arrs = CurRangeArrays(sets, snaps)
    for i, a in enumerate(arrs.arrs):
        assert (bdb_osql_serial_check(validator, a) != 0) == (want[i] != 0)
        assert ((a.file << 32) | a.offset) == int(want_post[i])
    assert bdb_osql_serial_check(validator, None) == 0


@pytest.mark.parametrize("name", sorted(serialstep()))
def test_serialstep_known_answers_gpu(validator, name):
    sc = serialstep()[name]
    rcs = replay(scenario_events(sc), gpu_checker(validator))
    assert sorted(t for t, rc in rcs.items() if rc) == sorted(sc["expect_fail"])


def test_config1_replay(validator, oracle_mod):
    ev = config1_events(n_txn=400)
    got = replay(ev, gpu_checker(validator))
    want = replay(ev, lambda log, rs: oracle_mod.check(log, rs)[0])
    assert got == want


@pytest.mark.parametrize("kw", [
    dict(n_commits=3000, n_txn=800, value_bits=20, width=1 << 10, snap_recent=0.5),
    dict(n_commits=20000, n_txn=2000, value_bits=24, width=1 << 12, snap_recent=0.2),
    dict(n_commits=5000, n_txn=1000, value_bits=8, width=4, snap_recent=1.0),  # heavy duplicates
])
def test_config2_scaled_bit_exact(validator, oracle_mod, kw):
    c2 = config2(**kw)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets, nthreads=8)
    validator.ingest_log(c2.log)
    got = validator.check_readsets(c2.readsets)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert int((got != 0).sum()) > 0


def test_long_keys_many_groups(validator, oracle_mod):
    # keys up to 64 bytes (8 words), 24 groups, ranges spanning many tiles
    rng = np.random.default_rng(5)
    lb = LogBuilder()
    snaps = [lb.next_lsn()]
    tabs = [f"t{i}" for i in range(8)]
    for c in range(3000):
        lb.begin(c)
        for _ in range(6):
            tb = tabs[int(rng.integers(0, 8))]
            ix = int(rng.integers(0, 3))
            kl = [9, 33, 64][ix]
            k = bytes([8]) + rng.integers(0, 3, size=kl - 1).astype(np.uint8).tobytes()
            lb.write(c, F.REC_UNDO_ADD_IX_LK, tb, ix, k)
        snaps.append(lb.commit(c))
    log = lb.build()
    sets, ss = [], []
    for t in range(500):
        rs = []
        for _ in range(int(rng.integers(1, 6))):
            tb = tabs[int(rng.integers(0, 8))]
            ix = int(rng.integers(0, 3))
            a = bytes([8]) + rng.integers(0, 3, size=int(rng.integers(0, 40))).astype(np.uint8).tobytes()
            b = bytes([8]) + rng.integers(0, 3, size=int(rng.integers(0, 40))).astype(np.uint8).tobytes()
            rs.append(Range(tb, ix, min(a, b), max(a, b)))
        sets.append(rs)
        ss.append(snaps[int(rng.integers(0, len(snaps)))])
    rs = ReadSets.from_lists(sets, ss, tbnames=lb.tbnames)
    want, _, _ = oracle_mod.check(log, rs)
    validator.ingest_log(log)
    assert validator.words == 8
    got = validator.check_readsets(rs)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_config2_full_size_sampled(validator, oracle_mod):
    """BASELINE config 2 at full size: GPU verdicts for all 100k read sets;
    the oracle re-checks a deterministic sample of 2000 of them, and the
    batch is invariant under read-set order (permutation property)."""
    c2 = config2()
    validator.ingest_log(c2.log)
    got = validator.check_readsets(c2.readsets)
    rate = float((got != 0).mean())
    assert 0.2 <= rate <= 0.6, rate
    sample = np.arange(0, c2.readsets.ntxn, 50)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets.subset(sample), nthreads=16)
    np.testing.assert_array_equal(got[sample] != 0, want != 0)
    perm = np.random.default_rng(1).permutation(c2.readsets.ntxn)
    got_p = validator.check_readsets(c2.readsets.subset(perm))
    np.testing.assert_array_equal(got_p, got[perm])


@pytest.mark.parametrize("kw", [dict(n_writes=30000, n_txn=2000),
                                dict(n_writes=200000, n_txn=5000, vmax=1 << 20)])
def test_config3_composite_keys(validator, oracle_mod, kw):
    from comdb2_amd.workloads import config3
    log, rs = config3(**kw)
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    validator.ingest_log(log)
    got = validator.check_readsets(rs)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_config5_zipf_hot_keys(validator, oracle_mod):
    from comdb2_amd.workloads import config5
    c5 = config5(n_commits=50000, n_txn=5000, snap_recent=0.002)
    want, _, _ = oracle_mod.check(c5.log, c5.readsets, nthreads=8)
    validator.ingest_log(c5.log)
    got = validator.check_readsets(c5.readsets)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_pipelined_batch_entry_matches_oracle(validator, oracle_mod):
    """A batch large enough for the chunked pipeline of the drop-in entry
    (>= 65536 read sets: chunks marshalled on the host threads while the
    previous chunk is on the GPU) equals the flat entry on every read set and
    the oracle on a sample; post-call (file, offset) = the end LSN."""
    from comdb2_amd.hsc import NativeCurRangeArrs
    c2 = config2(n_commits=20_000, n_txn=70_000, value_bits=24, width=1 << 6, snap_recent=0.2)
    validator.ingest_log(c2.log)
    flat = validator.check_readsets(c2.readsets)
    arrs = NativeCurRangeArrs(c2.readsets)
    try:
        snaps = np.asarray(c2.readsets.snap, np.uint64)
        f = np.ascontiguousarray(snaps >> np.uint64(32), np.uint32)
        o = np.ascontiguousarray(snaps & np.uint64(0xFFFFFFFF), np.uint32)
        for threads in (1, 0):
            validator.set_threads(threads)
            ff, oo = f.copy(), o.copy()
            got = validator.check_batch(arrs, file=ff, offset=oo)
            np.testing.assert_array_equal(got != 0, flat != 0)
            end = int(c2.log.end_lsn)
            assert (ff == end >> 32).all() and (oo == end & 0xFFFFFFFF).all()
    finally:
        arrs.close()
        validator.set_threads(0)
    sample = np.arange(0, c2.readsets.ntxn, 97)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets.subset(sample))
    np.testing.assert_array_equal(flat[sample] != 0, want != 0)
    assert 0.05 < (flat != 0).mean() < 0.95
