"""Compact codes of wide windows (hsc_compact.hip): each (table, index, key
length) group's keys keep only the bits that vary inside the group, and probe
bounds map onto the codes exactly (mismatches at constant bits above / below
the group's pattern, prefix ranges padded 0x00 / 0xFF, open ends, ranges that
miss every row).  Verdicts must equal the oracle's and the plain wide
layout's."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import LAYOUT_AUTO, LAYOUT_COMPACT, LAYOUT_WIDE

pytestmark = pytest.mark.gpu

ALPHA_ROWS = [0x08, 0x61, 0x62, 0x63]              # window key bytes (few varying bits)
ALPHA_PROBE = [0x00, 0x08, 0x09, 0x60, 0x61, 0x62, 0x63, 0x64, 0x7F, 0x80, 0xE1, 0xFF]


def _case(seed, n_commits=2500, n_txn=700, lens=(9, 24, 41, 64), n_tabs=5):
    rng = np.random.default_rng(seed)
    lb = LogBuilder()
    snaps = [lb.next_lsn()]
    tabs = [f"t{i}" for i in range(n_tabs)]
    head = {}  # per group: a fixed random prefix (constant bytes)
    for tb in tabs:
        for ix, kl in enumerate(lens):
            head[(tb, ix)] = bytes([8]) + rng.choice(ALPHA_ROWS, size=int(rng.integers(0, 6))).astype(np.uint8).tobytes()
    keys = {}
    for c in range(n_commits):
        lb.begin(c)
        for _ in range(int(rng.integers(1, 7))):
            tb = tabs[int(rng.integers(0, n_tabs - 1))]  # the last table is never written: its probes miss every row
            ix = int(rng.integers(0, len(lens)))
            kl = lens[ix]
            h = head[(tb, ix)]
            body = rng.choice(ALPHA_ROWS, size=kl - len(h)).astype(np.uint8)
            if rng.random() < 0.5:  # a run of constant zero bytes inside the key
                z = int(rng.integers(0, len(body)))
                body[z:z + 5] = 0
            k = (h + body.tobytes())[:kl]
            keys.setdefault((tb, ix), []).append(k)
            lb.write(c, F.REC_UNDO_ADD_IX_LK, tb, ix, k)
        snaps.append(lb.commit(c))
    log = lb.build()

    def probe_key(tb, ix):
        kl = lens[ix]
        u = rng.random()
        ks = keys.get((tb, ix))
        if ks and u < 0.45:
            k = bytearray(ks[int(rng.integers(0, len(ks)))])
            if rng.random() < 0.5:  # flip one byte to a probe-alphabet byte
                k[int(rng.integers(0, kl))] = int(rng.choice(ALPHA_PROBE))
            cut = int(rng.integers(1, kl + 1)) if rng.random() < 0.3 else kl
            return bytes(k[:cut])
        n = int(rng.integers(1, kl + 1))
        return bytes(rng.choice(ALPHA_PROBE, size=n).astype(np.uint8))

    sets, ss = [], []
    for t in range(n_txn):
        rs = []
        for _ in range(int(rng.integers(1, 8))):
            tb = tabs[int(rng.integers(0, n_tabs))]
            ix = int(rng.integers(0, len(lens)))
            a, b = probe_key(tb, ix), probe_key(tb, ix)
            u = rng.random()
            if u < 0.35:
                rs.append(Range(tb, ix, a, a))
            elif u < 0.85:
                rs.append(Range(tb, ix, min(a, b), max(a, b)))
            elif u < 0.9:
                rs.append(Range(tb, ix, max(a, b), min(a, b)))  # inverted: matches nothing
            elif u < 0.95:
                rs.append(Range(tb, ix, None, a, lflag=1))
            else:
                rs.append(Range(tb, ix, a, None, rflag=1))
        rs.sort(key=lambda r: (r.tbname, -r.islocked, r.idxnum, r.lkey or b""))
        sets.append(rs)
        ss.append(snaps[int(rng.integers(max(0, len(snaps) - 400), len(snaps)))])
    return log, ReadSets.from_lists(sets, ss, tbnames=lb.tbnames)


@pytest.mark.parametrize("seed", range(6))
def test_compact_matches_oracle_and_wide(validator, oracle_mod, seed):
    log, rs = _case(seed)
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    validator.set_layout(LAYOUT_AUTO)
    validator.ingest_log(log)
    assert validator.layout == LAYOUT_COMPACT
    assert validator.code_words < validator.words == 8
    got = validator.check_readsets(rs)
    np.testing.assert_array_equal(got != 0, want != 0)
    validator.set_layout(LAYOUT_WIDE)
    validator.ingest_log(log)
    assert validator.layout == LAYOUT_WIDE
    np.testing.assert_array_equal(validator.check_readsets(rs) != 0, want != 0)
    validator.set_layout(LAYOUT_AUTO)
    assert 0.05 < float((want != 0).mean()) < 0.95


def test_config3_window_is_compact(validator, oracle_mod):
    from comdb2_amd.workloads import config3
    log, rs = config3(n_writes=60000, n_txn=3000)
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    validator.set_layout(LAYOUT_AUTO)
    validator.ingest_log(log)
    assert validator.layout == LAYOUT_COMPACT and validator.code_words <= 3
    np.testing.assert_array_equal(validator.check_readsets(rs) != 0, want != 0)


@pytest.mark.parametrize("seed", range(2))
def test_compact_long_keys_match_oracle(oracle_mod, seed):
    """Keys over 64 bytes (W > 8 words) take the generic bound kernel; the
    register-resident one covers W <= 8 (the tests above)."""
    from comdb2_amd.hsc import Validator
    log, rs = _case(100 + seed, n_commits=1200, n_txn=400, lens=(9, 72))
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    v = Validator(0)  # own context: its group dictionary keeps the 9-word key length
    try:
        v.ingest_log(log)
        assert v.layout == LAYOUT_COMPACT and v.words > 8
        np.testing.assert_array_equal(v.check_readsets(rs) != 0, want != 0)
    finally:
        v.close()


def test_compact_many_groups_match_oracle(oracle_mod):
    """120 groups of 8-word keys: the per-group tables exceed the bound
    kernel's LDS budget, so it reads them from global memory."""
    from comdb2_amd.hsc import Validator
    log, rs = _case(7, n_commits=3000, n_txn=600, n_tabs=30)
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    v = Validator(0)  # own context: the shared one's group dictionary holds longer keys
    try:
        v.ingest_log(log)
        assert v.layout == LAYOUT_COMPACT and v.words == 8
        np.testing.assert_array_equal(v.check_readsets(rs) != 0, want != 0)
    finally:
        v.close()
