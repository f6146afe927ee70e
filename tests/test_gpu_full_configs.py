"""GPU: BASELINE configs 3 and 5 at their bench sizes (one GPU), checked
against the log-based oracle (oracle/serial_oracle.c: the reference's per
read set log rescan, chain walks and range scans) on an every-50th sample of
the 100k read sets, not only against the CPU sort-join.  The oracle reads a
tail of the log from the oldest sampled snapshot on (workloads.config3_log /
config5_log: each check only reads records after its snapshot).  The read
sets are narrow, as config 2's, so the sample discriminates:
the conflict rate is asserted in the 20-60 % band."""
import numpy as np
import pytest

from comdb2_amd.hsc import Validator

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _ingest(v, gid, words, lsn, end_lsn):
    dev = torch.device("cuda", 0)
    tg = torch.from_numpy(np.ascontiguousarray(gid)).to(dev)
    tw = torch.from_numpy(np.ascontiguousarray(words).reshape(-1).view(np.int64)).to(dev)
    tl = torch.from_numpy(np.ascontiguousarray(lsn).view(np.int64)).to(dev)
    v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), end_lsn)
    torch.cuda.synchronize()


def _first_commit(commit_lsn, snaps):
    """Index of the commit whose regop is the oldest snapshot (or the commit
    before it): the tail of the log from there holds every record a check of
    these snapshots reads."""
    s = int(snaps.min())
    c0 = int(np.searchsorted(commit_lsn, s))
    if c0 >= len(commit_lsn) or int(commit_lsn[c0]) != s:
        c0 = max(0, c0 - 1)
    return c0


def test_config3_full_size_sampled_vs_log_oracle(oracle_mod):
    from comdb2_amd.workloads import config3_arrays, config3_log
    a = config3_arrays(n_writes=4_000_000, n_txn=100_000)
    v = Validator(0)
    try:
        for g, (tb, ix, L) in enumerate(a.groups):
            assert v.register_group(tb, ix, L) == g
        gid, words, lsn = a.window()
        _ingest(v, gid, words, lsn, a.end_lsn)
        v.merge_table_max(a.table_max)
        assert v.tile_key_words == 3  # the compact tiles path of the bench
        got = v.check_readsets(a.readsets) != 0
    finally:
        v.close()
    rate = float(got.mean())
    assert 0.2 < rate < 0.6, rate
    sample = np.arange(0, a.readsets.ntxn, 50)
    sub = a.readsets.subset(sample)
    tail = config3_log(a, from_commit=_first_commit(a.commit_lsn, sub.snap))
    want, _, _ = oracle_mod.check(tail, sub, nthreads=16)
    np.testing.assert_array_equal(got[sample], want != 0)


def test_config5_full_size_sampled_vs_log_oracle(oracle_mod):
    from comdb2_amd.workloads import config5_log, config5_scaled
    c5 = config5_scaled(keys_per_gpu=125_000_000, n_txn=100_000)
    v = Validator(0)
    try:
        assert v.register_group("t1", 0, 9) == 0
        _ingest(v, c5.gid, c5.words, c5.lsn, c5.end_lsn)
        v.merge_table_max(np.array([c5.lsn.max()], np.uint64))
        got = v.check_readsets(c5.readsets) != 0
    finally:
        v.close()
    rate = float(got.mean())
    assert 0.2 < rate < 0.6, rate
    sample = np.arange(0, c5.readsets.ntxn, 50)
    sub = c5.readsets.subset(sample)
    K, R = 10, 13
    regops = c5.lsn[K - 1::K]  # one row per key: every K-th row is a new commit
    tail = config5_log([c5.keys], keys_per_commit=K,
                       from_commit=_first_commit(regops, sub.snap))
    assert tail.nrec < len(c5.keys) // 10 * R // 4
    want, _, _ = oracle_mod.check(tail, sub, nthreads=16)
    np.testing.assert_array_equal(got[sample], want != 0)
