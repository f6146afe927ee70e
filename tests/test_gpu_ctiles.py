"""Compact tiles (hsc_ctiles.hip): compact windows whose gid || code keys fit
<= 3 words are probed as one sorted array of wide keys with 32-bit commit
times -- bucket-table locate, fixed-capacity tile buckets, 4-byte bucket
entries, full-key Eytzinger joins.  Verdicts must equal the oracle's and the
wide compact pipeline's (LAYOUT_COMPACT_WIDE) on the same windows: config 3,
short composite keys with ties at every word, hot tiles that overflow their
bucket, sparse batches and appended rows."""
import os

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import (LAYOUT_AUTO, LAYOUT_COMPACT, LAYOUT_COMPACT_WIDE, LAYOUT_NARROW,
                            PATH_NO_COMP_NARROW, PATH_NO_CT_POINTS, Validator)

pytestmark = pytest.mark.gpu
# torch (device arrays for hsc_window_ingest_device) is imported before any
# test initialises HIP in this process
torch = pytest.importorskip("torch")

ROWS = [0x00, 0x08, 0x61, 0x62]
PROBE = [0x00, 0x07, 0x08, 0x09, 0x60, 0x61, 0x62, 0x63, 0xFF]


def _short_case(seed, n_commits=3000, n_txn=900, lens=(9, 17, 23), n_tabs=4, hot=0.0, var=None,
                ends=False, rows=None, probe=None):
    """Keys of few varying bits per byte (codes + group id fit 3 words), probes
    equal to rows, prefixes, one-byte edits, inverted and open ranges; hot > 0:
    that share of ranges are points on a handful of keys (overflowing tiles)."""
    rng = np.random.default_rng(seed)
    ROWS_, PROBE_ = rows or ROWS, probe or PROBE
    lb = LogBuilder()
    snaps = [lb.next_lsn()]
    tabs = [f"t{i}" for i in range(n_tabs)]
    keys = {}
    for c in range(n_commits):
        lb.begin(c)
        for _ in range(int(rng.integers(1, 9))):
            tb = tabs[int(rng.integers(0, n_tabs - 1))]  # the last table is never written
            ix = int(rng.integers(0, len(lens)))
            nv = lens[ix] - 1 if var is None else min(var, lens[ix] - 1)  # varying bytes, then 0x01s
            k = bytes([8]) + rng.choice(ROWS_, size=nv).astype(np.uint8).tobytes()
            k += b"\x01" * (lens[ix] - len(k))
            if ends:  # ... and two more varying bytes at the key's end
                k = k[:-2] + rng.choice(ROWS_, size=2).astype(np.uint8).tobytes()
            keys.setdefault((tb, ix), []).append(k)
            lb.write(c, F.REC_UNDO_ADD_IX_LK, tb, ix, k)
        snaps.append(lb.commit(c))
    log = lb.build()
    hot_keys = [(tb, ix, ks[int(rng.integers(0, len(ks)))]) for (tb, ix), ks in
                sorted(keys.items())[:3]]

    def key(tb, ix):
        kl = lens[ix]
        ks = keys.get((tb, ix))
        if ks and rng.random() < 0.6:
            k = bytearray(ks[int(rng.integers(0, len(ks)))])
            if rng.random() < 0.3:
                k[int(rng.integers(0, kl))] = int(rng.choice(PROBE_))
            cut = int(rng.integers(1, kl + 1)) if rng.random() < 0.25 else kl
            return bytes(k[:cut])
        return bytes(rng.choice(PROBE_, size=int(rng.integers(1, kl + 1))).astype(np.uint8))

    sets, ss = [], []
    for t in range(n_txn):
        rs = []
        for _ in range(int(rng.integers(1, 9))):
            if rng.random() < hot:
                tb, ix, k = hot_keys[int(rng.integers(0, len(hot_keys)))]
                rs.append(Range(tb, ix, k, k))
                continue
            tb = tabs[int(rng.integers(0, n_tabs))]
            ix = int(rng.integers(0, len(lens)))
            a, b = key(tb, ix), key(tb, ix)
            u = rng.random()
            if u < 0.4:
                rs.append(Range(tb, ix, a, a))
            elif u < 0.85:
                rs.append(Range(tb, ix, min(a, b), max(a, b)))
            elif u < 0.9:
                rs.append(Range(tb, ix, max(a, b), min(a, b)))
            elif u < 0.95:
                rs.append(Range(tb, ix, None, a, lflag=1))
            else:
                rs.append(Range(tb, ix, a, None, rflag=1))
        if rng.random() < 0.02:
            rs.append(Range.locked(tabs[int(rng.integers(0, n_tabs))]))
        rs.sort(key=lambda r: (r.tbname, -r.islocked, r.idxnum, r.lkey or b""))
        sets.append(rs)
        ss.append(snaps[int(rng.integers(max(0, len(snaps) - 300), len(snaps)))])
    return log, ReadSets.from_lists(sets, ss, tbnames=lb.tbnames)


def _both(v, log, rs):
    """Verdicts through the compact tiles and through the wide compact
    pipeline (which must agree)."""
    v.set_layout(LAYOUT_AUTO)
    v.ingest_log(log)
    assert v.layout == LAYOUT_COMPACT
    assert 1 <= v.tile_key_words <= 3
    got = v.check_readsets(rs) != 0
    v.ingest_log(log)
    v.set_layout(LAYOUT_COMPACT_WIDE)
    ref = v.check_readsets(rs) != 0
    v.set_layout(LAYOUT_AUTO)
    return got, ref


@pytest.mark.parametrize("seed", range(5))
def test_short_keys_match_oracle(oracle_mod, seed):
    log, rs = _short_case(seed)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, ref = _both(v, log, rs)
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)
    assert 0.05 < want.mean() < 0.95


def test_hot_tiles_overflow_match_oracle(oracle_mod):
    """Half the ranges are points on three keys: their tiles take far more than
    a bucket's 1024 records (overflow runs, extra join items)."""
    log, rs = _short_case(21, n_commits=4000, n_txn=6000, hot=0.5)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, ref = _both(v, log, rs)
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)


def test_sparse_batch_matches_oracle(oracle_mod):
    """A sparse batch (fewer ranges than 8 per tile) on a compact-tile window
    takes the wide pipeline, which stages only the tiles its ranges reach."""
    log, rs = _short_case(5, n_commits=6000, n_txn=20)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, _ = _both(v, log, rs)
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("kw", [dict(n_writes=40000, n_txn=2000),
                                dict(seed=5, n_writes=80000, n_txn=3000, keys_per_commit=3)])
def test_config3_matches_oracle(oracle_mod, kw):
    from comdb2_amd.workloads import config3
    log, rs = config3(**kw)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, ref = _both(v, log, rs)
        assert v.tile_key_words == 3 and v.code_words == 3
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)


def test_appended_rows_match_oracle(oracle_mod):
    """Rows appended after the build sit in the delta run, probed beside the
    compact tiles into the same flags."""
    from test_incremental import log_slice
    log, rs = _short_case(9, n_commits=3000, n_txn=800)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    cut = log.nrec * 3 // 4
    v = Validator(0)
    try:
        v.ingest_log(log_slice(log, 0, cut))
        v.check_readsets(rs)  # built: the rest goes to the delta run
        assert v.layout == LAYOUT_COMPACT and v.tile_key_words >= 1
        v.append_log(log_slice(log, cut, log.nrec))
        assert v.delta_rows > 0
        got = v.check_readsets(rs) != 0
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)


def test_long_keys_unfused_locate_match_oracle(oracle_mod):
    """72-byte keys (W = 9 words) whose varying bytes fit 3-word keys: the
    bounds go through the generic bound kernel and the unfused locate."""
    log, rs = _short_case(13, n_commits=2500, n_txn=800, lens=(9, 72), var=20)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, ref = _both(v, log, rs)
        assert v.words == 9
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)


def test_one_word_keys_match_oracle(oracle_mod):
    """Varying bytes at both ends of 17-byte keys: too far apart for the
    narrow 62-bit codes, but the compact codes plus the group id fit one word
    (WG = 1)."""
    log, rs = _short_case(17, n_commits=2500, n_txn=800, lens=(9, 17), var=2, ends=True)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        # (by default such a window takes the narrow index over compressed
        # codes: its varying bits total <= 62 -- checked there too)
        v.ingest_log(log)
        assert v.layout == LAYOUT_NARROW
        np.testing.assert_array_equal(v.check_readsets(rs) != 0, want)
        v.set_paths(PATH_NO_COMP_NARROW)
        got, ref = _both(v, log, rs)
        assert v.tile_key_words == 1
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)
    assert 0.02 < want.mean() < 0.98


@pytest.mark.parametrize("case", ["short", "hot", "one_word", "config3"])
def test_point_index_matches_join_records(oracle_mod, case):
    """Point probes (lo == hi) answered by the compact tiles' point index in
    the bound kernel (no join record) give the verdicts of the join-record
    path (HSC_PATH_NO_CT_POINTS) and of the oracle, and the join gets fewer
    records: random short keys, three hot keys taking half the ranges, one-word
    keys (WG = 1) and config 3."""
    paths = 0
    if case == "short":
        log, rs = _short_case(31, n_commits=3000, n_txn=900)
    elif case == "hot":
        log, rs = _short_case(32, n_commits=4000, n_txn=3000, hot=0.5)
    elif case == "one_word":
        log, rs = _short_case(33, n_commits=2500, n_txn=800, lens=(9, 17), var=2, ends=True)
        paths = PATH_NO_COMP_NARROW
    else:
        from comdb2_amd.workloads import config3
        log, rs = config3(n_writes=60000, n_txn=3000, seed=7)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        recs = []
        got = []
        for p in (paths, paths | PATH_NO_CT_POINTS):
            v.set_paths(p)
            v.ingest_log(log)
            assert v.layout == LAYOUT_COMPACT and 1 <= v.tile_key_words <= 3
            v.enable_timing(True)
            got.append(v.check_readsets(rs) != 0)
            recs.append(v.timing()["records"])
            v.enable_timing(False)
    finally:
        v.close()
    np.testing.assert_array_equal(got[0], want)
    np.testing.assert_array_equal(got[1], want)
    assert recs[0] < recs[1], recs  # the points took no join records


def test_config3_full_size_matches_sortjoin():
    """BASELINE config 3 at full size (4M index writes, 100k read sets) through
    the compact tiles: equal to the CPU sort-join over the same window
    (oracle/sortjoin.c) and to the wide compact pipeline."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import oracle
    from comdb2_amd.workloads import config3_arrays
    a = config3_arrays(n_writes=4_000_000, n_txn=100_000)
    v = Validator(0)
    try:
        for g, (tb, ix, L) in enumerate(a.groups):
            assert v.register_group(tb, ix, L) == g
        gid, words, lsn = a.window()
        dev = torch.device("cuda", 0)
        tg = torch.from_numpy(gid).to(dev)
        tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
        tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
        v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                        a.end_lsn)
        torch.cuda.synchronize()
        v.merge_table_max(a.table_max)
        assert v.tile_key_words == 3
        m = v.marshal(a.readsets)
        got = v.check_readsets(a.readsets) != 0
        v.set_layout(LAYOUT_COMPACT_WIDE)
        ref = v.check_readsets(a.readsets) != 0
        sj = oracle.SortJoin(gid, words, lsn, len(a.groups))
        want, _ = sj.probe(m, v.table_max(), nthreads=8)
        sj.close()
    finally:
        v.close()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got, want != 0)
    assert 0.05 < got.mean() < 0.99


def test_keys_in_the_top_bucket_match_oracle(oracle_mod):
    """32 groups (5 group bits) whose keys' varying bytes are 0x00 / 0xFF: the
    last group's keys reach the top of the key space, so the locate's bucket
    table spans 2^64 (its last bucket boundary overflows)."""
    log, rs = _short_case(23, n_commits=3000, n_txn=900, lens=(9, 12, 17, 20), n_tabs=9, var=10,
                          rows=[0x00, 0xFF], probe=[0x00, 0x01, 0xFE, 0xFF])
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    v = Validator(0)
    try:
        got, ref = _both(v, log, rs)
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(ref, want)
    assert 0.02 < want.mean() < 0.98
