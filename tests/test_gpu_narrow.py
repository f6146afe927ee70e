"""GPU parity of the window layouts and probe paths.

The narrow layout (every key as one 62-bit code under a 16-ary index,
comdb2_amd/csrc/hsc_narrow.hip) answers a batch with the direct probe
kernel, with the tile pipeline on 8-byte rows (u32 key delta + commit rank,
where every tile fits) or with the tile pipeline over 16-byte code rows; the
wide layout keeps every key as its big-endian words.  All four must give
verdicts bit-identical to the oracle (oracle/serial_oracle.c, the
bdb_osql_serial_check restatement): every case runs four times on the same
context."""

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import (PATH_NO_COMP_NARROW, PATH_TILE_DIR, LAYOUT_AUTO, LAYOUT_NARROW, LAYOUT_NARROW_CODES,
                            LAYOUT_NARROW_DIRECT, LAYOUT_NARROW_TILES, LAYOUT_WIDE)
from comdb2_amd.workloads import config2, config5

pytestmark = pytest.mark.gpu


def both_layouts(v, oracle_mod, log, rs, expect_auto):
    """Direct probe, tile pipeline over codes (both on the narrow layout when
    the window fits it) and the wide layout, each against the oracle."""
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    got = {}
    # (layout, build knob): locate finds tiles through the LDS bucket table by
    # default and through the 16-ary directory with PATH_TILE_DIR set (the path
    # of windows with too many tiles for the table).  Rows carry lsn - oldest
    # commit + 1 when the window spans < 2^32 of log, else commit ranks
    # (test_multi_file_window_commit_ranks); the bucket table's mode (linear
    # or log) is picked per window by its fullest bucket (config 5's Zipf keys
    # take log mode)
    runs = [(LAYOUT_NARROW_DIRECT, None), (LAYOUT_NARROW_TILES, None),
            (LAYOUT_NARROW_TILES, PATH_TILE_DIR), (LAYOUT_NARROW_CODES, None), (LAYOUT_WIDE, None)]
    try:
        for layout, knob in runs:
            v.set_paths(knob or 0)
            v.set_layout(layout)
            v.ingest_log(log)
            assert v.layout == (LAYOUT_WIDE if layout == LAYOUT_WIDE else expect_auto)
            got[layout] = v.check_readsets(rs)
            np.testing.assert_array_equal(got[layout] != 0, want != 0,
                                          err_msg=f"layout {layout} knob {knob}")
    finally:
        v.set_paths(0)
        v.set_layout(LAYOUT_AUTO)
    return want


def keyed_case(seed, n_commits, per_commit, key_fn, range_fn, n_txn, ranges_per_txn=6,
               snap_recent=0.3, dta_table=False, step=64):
    """One index of keys key_fn(rng) written by n_commits txns; read sets of
    range_fn(rng) ranges with snapshots among the most recent commits."""
    rng = np.random.default_rng(seed)
    lb = LogBuilder(step=step)
    commits = [lb.next_lsn()]
    for c in range(n_commits):
        lb.begin(c)
        for _ in range(per_commit):
            lb.write(c, F.REC_UNDO_UPD_IX, "t1", 0, key_fn(rng))
        if dta_table and c % 7 == 0:
            lb.write(c, F.REC_UNDO_ADD_DTA, "t2")
        commits.append(lb.commit(c))
    log = lb.build()
    recent = max(1, int(len(commits) * snap_recent))
    sets, snaps = [], []
    for _ in range(n_txn):
        rs = [range_fn(rng) for _ in range(ranges_per_txn)]
        if dta_table and rng.random() < 0.1:
            rs.append(Range("t2", -1, None, None, 1, 1, 1))
        sets.append(rs)
        snaps.append(commits[len(commits) - 1 - int(rng.integers(0, recent))])
    return log, ReadSets.from_lists(sets, snaps, tbnames=lb.tbnames)


@pytest.mark.parametrize("kw,expect", [
    (dict(n_commits=3000, n_txn=800, value_bits=20, width=1 << 10, snap_recent=0.5), LAYOUT_NARROW),
    (dict(n_commits=20000, n_txn=3000, value_bits=36, width=1 << 28, snap_recent=0.05), LAYOUT_NARROW),
    (dict(n_commits=20000, n_txn=3000, value_bits=40, width=1 << 30, snap_recent=0.05), LAYOUT_NARROW),
    (dict(n_commits=20000, n_txn=3000, value_bits=16, width=1 << 14, snap_recent=0.02), LAYOUT_NARROW),
    (dict(n_commits=5000, n_txn=1000, value_bits=8, width=4, snap_recent=1.0), LAYOUT_NARROW),
])
def test_config2_layouts(validator, oracle_mod, kw, expect):
    c2 = config2(**kw)
    want = both_layouts(validator, oracle_mod, c2.log, c2.readsets, expect)
    assert int((want != 0).sum()) > 0


def test_config5_zipf_layouts(validator, oracle_mod):
    c5 = config5(n_commits=50000, n_txn=5000, snap_recent=0.002)
    both_layouts(validator, oracle_mod, c5.log, c5.readsets, LAYOUT_NARROW)


def test_full_range_int64_falls_back_to_wide(validator, oracle_mod):
    big = lambda rng: F.enc_int64(int(rng.integers(-(1 << 63), (1 << 63) - 1, dtype=np.int64)))

    def rng_range(rng):
        a = int(rng.integers(-(1 << 63), (1 << 63) - (1 << 60), dtype=np.int64))
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(a + int(rng.integers(0, 1 << 58))))
    log, rs = keyed_case(11, 3000, 4, big, rng_range, 600)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_WIDE)


def test_three_word_keys_prefix_ranges(validator, oracle_mod):
    # 18-byte keys enc(7) || enc(b): W = 3, tz = 48; ranges mix full keys and
    # prefixes of 9..17 bytes, some open on one side
    key = lambda rng: F.enc_int64(7) + F.enc_int64(int(rng.integers(0, 1 << 20)))

    def rng_range(rng):
        b = int(rng.integers(0, 1 << 20))
        lo = F.enc_int64(7) + F.enc_int64(b)
        hi = F.enc_int64(7) + F.enc_int64(b + int(rng.integers(0, 1 << 12)))
        lo = lo[: int(rng.integers(9, 19))]
        hi = hi[: int(rng.integers(9, 19))]
        u = rng.random()
        if u < 0.05:
            return Range("t1", 0, None, hi, 1, 0)
        if u < 0.1:
            return Range("t1", 0, lo, None, 0, 1)
        return Range("t1", 0, lo, hi)
    log, rs = keyed_case(12, 4000, 5, key, rng_range, 800)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)


@pytest.mark.parametrize("ids,accts", [(20, 5), (3000, 300), (1 << 20, 7)])
def test_composite_keys_compressed_codes(validator, oracle_mod, ids, accts):
    """Two-field keys enc(id) || enc(acct) (the config-1 / serial.c index):
    their varying bits sit ~64 bits apart, too far for one 62-bit span, but
    total <= 62, so the narrow index runs over compressed codes (NarrowView
    comp).  Bounds leave the rows' constant pattern anywhere: ids and accts
    past the written ones, negative values, 9-byte id prefixes and cut keys,
    open ends -- every narrow path (small kernel, direct, tiles, codes) vs
    the oracle, and the compact / wide layouts with the mode off."""
    key = lambda rng: F.enc_int64(int(rng.integers(0, ids))) + F.enc_int64(int(rng.integers(0, accts)))

    def rng_range(rng):
        i = int(rng.integers(-2, ids + 2))
        a = int(rng.integers(-2, accts + 2))
        u = rng.random()
        if u < 0.3:  # the point read of one account
            k = F.enc_int64(i) + F.enc_int64(a)
            return Range("t1", 0, k, k)
        if u < 0.5:  # sum(bal) where id = ?: a 9-byte prefix range
            return Range("t1", 0, F.enc_int64(i), F.enc_int64(i))
        if u < 0.6:
            return Range("t1", 0, None, F.enc_int64(i) + F.enc_int64(a), 1, 0)
        if u < 0.7:
            return Range("t1", 0, F.enc_int64(i) + F.enc_int64(a), None, 0, 1)
        lo = F.enc_int64(i) + F.enc_int64(a)
        hi = F.enc_int64(i + int(rng.integers(0, 3))) + F.enc_int64(int(rng.integers(-1, accts + 1)))
        return Range("t1", 0, lo[: int(rng.integers(1, 19))], hi[: int(rng.integers(1, 19))])
    log, rs = keyed_case(21 + ids, 3000, 3, key, rng_range, 700)
    want = both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)
    assert int((want != 0).sum()) > 0
    validator.set_paths(PATH_NO_COMP_NARROW)
    try:
        validator.ingest_log(log)
        assert validator.layout != LAYOUT_NARROW
        np.testing.assert_array_equal(validator.check_readsets(rs) != 0, want != 0)
    finally:
        validator.set_paths(0)


def test_low_bits_vary_tz0(validator, oracle_mod):
    # 16-byte keys whose last 4 bytes vary (tz = 0), ranges with bounds of
    # 12..16 bytes (prefix compares pad inside word 1)
    head = bytes([8]) + bytes(range(1, 12))

    def key(rng):
        return head + int(rng.integers(0, 1 << 26)).to_bytes(4, "big")

    def rng_range(rng):
        a = int(rng.integers(0, 1 << 26))
        lo = (head + a.to_bytes(4, "big"))[: int(rng.integers(12, 17))]
        hi = (head + min(a + int(rng.integers(0, 1 << 16)), (1 << 32) - 1).to_bytes(4, "big"))
        return Range("t1", 0, lo, hi[: int(rng.integers(12, 17))])
    log, rs = keyed_case(13, 5000, 4, key, rng_range, 800)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)


def test_locked_dta_table_and_spans(validator, oracle_mod):
    # second table with data writes only (no key group): table locks go
    # through the lock probes, the index stays one narrow group
    key = lambda rng: F.enc_int64(int(rng.integers(0, 1 << 18)))

    def rng_range(rng):
        a = int(rng.integers(0, 1 << 18))
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(a + int(rng.integers(0, 1 << 13))))
    log, rs = keyed_case(14, 6000, 6, key, rng_range, 1000, dta_table=True, snap_recent=0.01)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)


def test_empty_and_reversed_ranges(validator, oracle_mod):
    key = lambda rng: F.enc_int64(int(rng.integers(0, 1 << 16)))

    def rng_range(rng):
        a = int(rng.integers(0, 1 << 16))
        b = a - int(rng.integers(0, 100)) if rng.random() < 0.5 else a
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(b))
    log, rs = keyed_case(15, 3000, 8, key, rng_range, 600)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)


def test_multi_file_window_commit_ranks(validator, oracle_mod):
    """A window over many log files (records 2^28 bytes apart: a new file every
    16 records) spans more than 2^32 of LSN space, so the narrow tiles carry
    commit ranks and snapshots go through the commit directory."""
    key = lambda rng: F.enc_int64(int(rng.integers(0, 1 << 22)))

    def rng_range(rng):
        a = int(rng.integers(0, 1 << 22))
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(a + int(rng.integers(0, 1 << 14))))
    log, rs = keyed_case(16, 4000, 6, key, rng_range, 900, step=1 << 28, snap_recent=0.05)
    assert int(log.lsn[-1] >> 32) - int(log.lsn[0] >> 32) > 100
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)


def test_hot_tile_bucket_overflow(validator, oracle_mod):
    """Most ranges of a dense batch land in one 4096-row tile: its fixed
    bucket (1024 records) spills, and the join covers the tile's further
    records with extra items (hsc_narrow.hip k_plan_s)."""
    key = lambda rng: F.enc_int64(int(rng.integers(0, 1 << 24)))

    def rng_range(rng):
        if rng.random() < 0.8:  # a narrow hot band: a handful of tiles
            a = int(rng.integers(1 << 23, (1 << 23) + (1 << 12)))
        else:
            a = int(rng.integers(0, 1 << 24))
        return Range("t1", 0, F.enc_int64(a), F.enc_int64(a + int(rng.integers(0, 64))))
    log, rs = keyed_case(17, 8000, 8, key, rng_range, 4000, ranges_per_txn=8, snap_recent=0.02)
    both_layouts(validator, oracle_mod, log, rs, LAYOUT_NARROW)
