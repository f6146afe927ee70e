"""GPU: the small-batch path of the drop-in entry (k_small_narrow: one launch
for ranges, delta run and table locks, probe columns and verdicts in
fine-grained host memory, completion by a polled done word) against the
staged path (hsc_set_paths(PATH_NO_SMALL)) and the oracle
(oracle/serial_oracle.c): lone calls, collector-sized batches, batches with a
delta run pending and with table locks."""

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import Range, ReadSets
from comdb2_amd.hsc import LAYOUT_NARROW, PATH_NO_SMALL, NativeCurRangeArrs, Validator
from comdb2_amd.workloads import config2
from test_incremental import log_slice

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def staged():
    v = Validator(0)
    v.set_paths(PATH_NO_SMALL)
    yield v
    v.close()


@pytest.mark.parametrize("seed", range(4))
def test_small_batches_equal_staged_and_oracle(validator, staged, oracle_mod, seed):
    c2 = config2(seed=4100 + seed, n_commits=4000, n_txn=600, value_bits=24, width=1 << 8,
                 snap_recent=0.05)
    log, rs = c2.log, c2.readsets
    want, _, _ = oracle_mod.check(log, rs)
    for v in (validator, staged):
        v.ingest_log(log)
        assert v.layout == LAYOUT_NARROW  # the small path's window
    for lo, hi in ((0, 1), (1, 9), (9, 300), (300, 600)):
        sub = rs.subset(np.arange(lo, hi))
        a = validator.check_readsets(sub)
        b = staged.check_readsets(sub)
        np.testing.assert_array_equal(a != 0, b != 0)
        np.testing.assert_array_equal(a != 0, want[lo:hi] != 0)
    # table locks (a full scan of t1) at snapshots before, inside and after the log
    k = F.enc_int64(int(c2.key_values[5]))
    snaps = [int(log.lsn[0]), int(log.lsn[log.nrec // 2]), int(log.lsn[-1]), int(log.end_lsn)]
    sets = [[Range.locked("t1")], [Range("t1", 0, k, k), Range.locked("t1")]] * 2
    lk = ReadSets.from_lists(sets, snaps, tbnames=["t1"])
    want_l, _, _ = oracle_mod.check(log, lk)
    np.testing.assert_array_equal(validator.check_readsets(lk) != 0, want_l != 0)
    np.testing.assert_array_equal(staged.check_readsets(lk) != 0, want_l != 0)
    assert 0 < int((want_l != 0).sum()) < len(want_l)


def test_lone_calls_with_a_delta_run(validator, staged, oracle_mod):
    """A config-2-shaped window built from a prefix, the rest appended (delta
    run pending), then hip_serial_check_batch calls of 1 and 37 read sets
    (CurRangeArr*, as a master holds them) on both paths."""
    c2 = config2(n_commits=3000, n_txn=400, value_bits=24, width=1 << 8, snap_recent=0.05)
    log = c2.log
    R = 13
    for v in (validator, staged):
        v.ingest_log(log_slice(log, 0, 2000 * R))
        v.check_readsets(c2.readsets.subset([0]))  # built: the rest goes to the delta run
        v.append_log(log_slice(log, 2000 * R, log.nrec))
        assert v.delta_rows > 0
    want, post, _ = oracle_mod.check(log, c2.readsets)
    arrs = NativeCurRangeArrs(c2.readsets)
    try:
        ptrs = arrs.pointers()
        for step in (1, 37):
            for t0 in range(0, c2.readsets.ntxn, step * 5):
                n = min(step, c2.readsets.ntxn - t0)
                snaps = c2.readsets.snap[t0:t0 + n]
                for v in (validator, staged):
                    f = np.ascontiguousarray(snaps >> np.uint64(32), np.uint32)
                    o = np.ascontiguousarray(snaps & np.uint64(0xFFFFFFFF), np.uint32)
                    sub = _Sub(ptrs, t0, n)
                    got = v.check_batch(sub, file=f, offset=o)
                    np.testing.assert_array_equal(got != 0, want[t0:t0 + n] != 0)
                    assert (((f.astype(np.uint64) << np.uint64(32)) | o) == post[t0:t0 + n]).all()
    finally:
        arrs.close()
    assert 0 < int((want != 0).sum()) < len(want)


class _Sub:
    """n CurRangeArr* starting at element t0 of a native array."""

    def __init__(self, ptrs, t0, n):
        import ctypes as C
        self.n = n
        self._p = C.cast(C.addressof(ptrs.contents) + 8 * t0, C.POINTER(C.c_void_p))

    def pointers(self):
        return self._p


def test_small_batches_race_stream_switches_and_appends(oracle_mod):
    """One thread runs small batches (k_small_narrow, verdicts read without
    the context lock) while another switches the context's stream and
    appends commits: a stream switch or a delta merge waits for the small
    kernels in flight (wait_small), so no probe reads a run being rewritten;
    every call succeeds and the final verdicts equal the oracle's."""
    import threading
    c2 = config2(seed=4242, n_commits=3000, n_txn=300, value_bits=22, width=1 << 8,
                 snap_recent=0.05)
    log, rs = c2.log, c2.readsets
    R = 13
    want, _, _ = oracle_mod.check(log, rs)
    v = Validator(0)
    errors = []
    stop = threading.Event()
    try:
        v.ingest_log(log_slice(log, 0, 1500 * R))
        v.check_readsets(rs.subset([0]))  # built: appends go to the delta run
        side = torch.cuda.Stream(device=0)

        def checker():
            k = 0
            while not stop.is_set():
                try:
                    v.check_readsets(rs.subset(np.arange(k % 290, k % 290 + 1 + k % 7)))
                except Exception as e:  # noqa: BLE001
                    errors.append(e)
                    return
                k += 1

        th = threading.Thread(target=checker)
        th.start()
        try:
            for i, c in enumerate(range(1500, 3000, 100)):
                v.set_stream(side.cuda_stream if i % 2 else 0)
                v.append_log(log_slice(log, c * R, min(c + 100, 3000) * R))
        finally:
            stop.set()
            th.join()
        v.set_stream(0)
        assert not errors, errors
        np.testing.assert_array_equal(v.check_readsets(rs) != 0, want != 0)
    finally:
        v.close()
