"""Key groups first seen after a window build.  A write appended to a built
window under a (table, index, key length) group the build did not have must
rebuild the window before the next probe: the per-group device tables (group
spans, compact-code masks) are sized at the build, and the marshal emits
probes with the new gid.  Verdicts equal the oracle (oracle/serial_oracle.c)
on the whole log, for appends as log records and as decoded writes, on the
AUTO (narrow / compact) and WIDE layouts; the device-ingested window takes a
group registered after its build the same way."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import LAYOUT_AUTO, LAYOUT_WIDE

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _key(rng, klen):
    k = F.enc_int64(int(rng.integers(0, 40))) + F.enc_int64(int(rng.integers(0, 3)))
    return (k + bytes(64))[:klen]


def _commit(lb, rng, name, writes):
    lb.begin(name)
    for tb, ix, klen in writes:
        lb.write(name, F.REC_UNDO_UPD_IX, tb, ix, _key(rng, klen))
    return lb.commit(name)


def _case(seed):
    """First part: t1 index 0 only (9-byte keys).  Second part: t2 (a new
    table), t1 index 1 (a new index) and t1 index 0 with 18-byte keys (a new
    key length of a known index)."""
    rng = np.random.default_rng(seed)
    lb = LogBuilder(["t1", "t2"])
    snaps = [lb.next_lsn()]
    for c in range(40):
        _commit(lb, rng, ("a", c), [("t1", 0, 9)] * 3)
        snaps.append(lb.next_lsn())
    n_first = len(lb.rows)
    new_groups = [("t2", 0, 9), ("t2", 3, 27), ("t1", 1, 9), ("t1", 0, 18)]
    for c in range(40):
        w = [new_groups[int(rng.integers(0, len(new_groups)))] for _ in range(2)]
        w.append(("t1", 0, 9))
        _commit(lb, rng, ("b", c), w)
        snaps.append(lb.next_lsn())
    log = lb.build()
    sets, ss = [], []
    for i in range(300):
        rs = []
        for _ in range(int(rng.integers(1, 5))):
            tb, ix, klen = ([("t1", 0, 9)] + new_groups)[int(rng.integers(0, 5))]
            lo, hi = _key(rng, klen), _key(rng, klen)
            if lo > hi:
                lo, hi = hi, lo
            m = int(rng.integers(1, klen + 1))
            rs.append(Range(tb, ix, lo[:m], hi[:m]))
        sets.append(rs)
        ss.append(snaps[int(rng.integers(0, len(snaps)))])
    return log, n_first, ReadSets.from_lists(sets, ss, tbnames=lb.tbnames)


@pytest.mark.parametrize("layout", [LAYOUT_AUTO, LAYOUT_WIDE])
@pytest.mark.parametrize("mode", ["log", "writes"])
def test_groups_first_seen_after_the_build(validator, oracle_mod, layout, mode):
    from test_incremental import log_slice
    for seed in range(3):
        log, n_first, rs = _case(seed)
        want, _, _ = oracle_mod.check(log, rs)
        assert 0 < int((want != 0).sum()) < len(want)
        validator.set_layout(layout)
        first = log_slice(log, 0, n_first)
        validator.ingest_log(first)
        validator.check_readsets(rs.with_snaps(np.minimum(rs.snap, first.end_lsn)))  # built
        if mode == "log":
            validator.append_log(log_slice(log, n_first, log.nrec))
        else:
            writes, commit = [], {}
            # decoded writes of the second part: walk each committed txn's records
            rows = list(zip(log.lsn[n_first:], log.rectype[n_first:], log.table[n_first:],
                            log.ix[n_first:], log.key_off[n_first:], log.keylen[n_first:]))
            pending = []
            for l, rt, tb, ix, ko, kl in rows:
                if rt == F.REC_UNDO_UPD_IX:
                    pending.append((log.tbnames[int(tb)], int(ix), bytes(log.keys[int(ko):int(ko) + int(kl)])))
                elif rt == F.REC_TXN_REGOP:
                    writes += [(tb_, ix_, k_, int(l)) for tb_, ix_, k_ in pending]
                    pending = []
            validator.append_writes(writes, end_lsn=int(log.end_lsn))
        got = validator.check_readsets(rs)
        np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"seed {seed} {mode} {layout}")
    validator.set_layout(LAYOUT_AUTO)


def test_group_registered_after_device_ingest():
    """A device-ingested window (one group) takes a second group registered
    after the build: the next check folds it in (no out-of-range gid)."""
    from comdb2_amd.hsc import Validator
    from comdb2_amd.workloads import int64_words
    v = Validator(0)  # its own dictionaries: 9-byte keys only
    try:
        g0 = v.register_group("dev_t", 0, 9)
        vals = np.arange(0, 4000, 4, dtype=np.int64)
        words = torch.tensor(int64_words(vals).astype(np.uint64).view(np.int64), device="cuda")
        gid = torch.full((len(vals),), g0, dtype=torch.int32, device="cuda")
        lsn = torch.tensor(np.arange(1, len(vals) + 1, dtype=np.int64) * 64 + (1 << 32), device="cuda")
        end = int((len(vals) + 1) * 64 + (1 << 32))
        torch.cuda.synchronize()
        v.ingest_device(len(vals), 2, gid.data_ptr(), words.data_ptr(), lsn.data_ptr(), end)
        g1 = v.register_group("dev_t2", 1, 9)
        assert g1 != g0
        k = F.enc_int64(8)
        rs = ReadSets.from_lists([[Range("dev_t", 0, k, k)], [Range("dev_t2", 1, k, k)]],
                                 [1 << 32, 1 << 32], tbnames=["dev_t", "dev_t2"])
        assert v.check_readsets(rs).tolist() == [1, 0]
        v.append_writes([("dev_t2", 1, k, end + 64)], end_lsn=end + 128)
        assert v.check_readsets(rs).tolist() == [1, 1]
    finally:
        v.close()
