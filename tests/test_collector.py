"""Batching collector (hsc_collector_check): many native caller threads, one
read set per call, as comdb2's block processors call bdb_osql_serial_check
(db/toblock.c:4779-4836 -> bdb/serializable.c:571).  Verdicts and the
(file, offset) side effect must be exactly the single call's.  regop_only
probes are answered from the context's published snapshot in the caller's
thread and never queue (no collector pass runs for them); the host-only
tests drive them against the oracle, and the batching itself with full
checks, which a host-only context fails closed (every verdict 1); the GPU
tests run the full check against the oracle."""
import numpy as np
import pytest

from comdb2_amd.hsc import NativeCurRangeArrs, Validator
from comdb2_amd.workloads import config2, random_case


@pytest.fixture(scope="module")
def host():
    v = Validator(-1)
    yield v
    v.close()


@pytest.mark.parametrize("nthreads,inflight", [(1, 0), (4, 0), (16, 0), (16, 1), (16, 4), (32, 3)])
def test_regop_only_through_collector(host, oracle_mod, nthreads, inflight):
    # inflight: batches the collector lets run at once (0 = its default, 2)
    log, rs = random_case(321 + nthreads, broken=True, n_txn=400)
    host.ingest_log(log)
    want, _, _ = oracle_mod.check(log, rs, regop_only=1)
    arrs = NativeCurRangeArrs(rs)
    got, st = host.concurrent_check(arrs, nthreads, rounds=3, regop_only=1, inflight=inflight)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert st["calls"] == 3 * rs.ntxn and st["batches"] == 0  # never queued
    direct, _ = host.concurrent_check(arrs, nthreads, regop_only=1, collect=False)
    np.testing.assert_array_equal(direct, got)
    # the batching: full checks (failed closed on a host-only context)
    full, st = host.concurrent_check(arrs, nthreads, rounds=3, regop_only=0, inflight=inflight)
    assert (full == 1).all() and st["calls"] == 3 * rs.ntxn
    assert 1 <= st["batches"] <= st["calls"] and st["max_batch"] <= nthreads
    arrs.close()


def test_collector_bounds_batches(host, oracle_mod):
    log, rs = random_case(99, n_txn=300)
    host.ingest_log(log)
    want, _, _ = oracle_mod.check(log, rs, regop_only=1)
    arrs = NativeCurRangeArrs(rs)
    got, st = host.concurrent_check(arrs, 16, rounds=2, regop_only=1, max_batch=3,
                                    max_wait_us=200)
    np.testing.assert_array_equal(got != 0, want != 0)
    got, st = host.concurrent_check(arrs, 16, rounds=2, regop_only=0, max_batch=3,
                                    max_wait_us=200)
    assert (got == 1).all()
    assert st["max_batch"] <= 3 and st["batches"] >= st["calls"] / 3
    arrs.close()


@pytest.mark.parametrize("max_batch,inflight", [(5, 3), (1, 1), (64, 4)])
def test_collector_many_threads_cut_batches(host, oracle_mod, max_batch, inflight):
    # 128 callers on the container's few CPUs, batches cut by max_batch
    # without a gather window: the requests left queued move to the next
    # batch's wait word and elect its leader
    log, rs = random_case(77, n_txn=500)
    host.ingest_log(log)
    want, _, _ = oracle_mod.check(log, rs, regop_only=1)
    arrs = NativeCurRangeArrs(rs)
    got, st = host.concurrent_check(arrs, 128, rounds=4, regop_only=1, max_batch=max_batch,
                                    inflight=inflight)
    np.testing.assert_array_equal(got != 0, want != 0)
    got, st = host.concurrent_check(arrs, 128, rounds=4, regop_only=0, max_batch=max_batch,
                                    inflight=inflight)
    assert (got == 1).all()
    assert st["calls"] == 4 * rs.ntxn and st["max_batch"] <= max_batch
    arrs.close()


def test_full_checks_fail_closed_without_device(host):
    # a host-only context cannot run the join: every full check answers 1
    # (errors are "not serializable"), through the collector as directly
    log, rs = random_case(5, n_txn=64)
    host.ingest_log(log)
    arrs = NativeCurRangeArrs(rs)
    got, st = host.concurrent_check(arrs, 8, regop_only=0)
    assert (got == 1).all() and st["calls"] == rs.ntxn
    arrs.close()


def test_collector_inflight_bounds():
    from comdb2_amd.hsc import load
    import ctypes as C
    lib = load()
    assert lib.hsc_collector_set_inflight(None, 2) != 0
    host = Validator(-1)
    col = C.c_void_p()
    assert lib.hsc_collector_create(host.ctx, 0, 0, C.byref(col)) == 0
    try:
        for bad in (0, 9, -1):
            assert lib.hsc_collector_set_inflight(col, bad) != 0
        for ok in (1, 4, 8):
            assert lib.hsc_collector_set_inflight(col, ok) == 0
    finally:
        lib.hsc_collector_destroy(col)
        host.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nthreads,inflight", [(2, 0), (16, 0), (64, 0), (64, 1), (64, 4)])
def test_gpu_full_checks_through_collector(validator, oracle_mod, nthreads, inflight):
    # the small-batch kernels of up to `inflight` batches queue on the stream
    # while their callers wait without the context lock
    log, rs = random_case(700 + nthreads, broken=(nthreads == 16), n_txn=600, max_ranges=12)
    validator.ingest_log(log)
    want, _, _ = oracle_mod.check(log, rs)
    arrs = NativeCurRangeArrs(rs)
    got, st = validator.concurrent_check(arrs, nthreads, rounds=2, inflight=inflight)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert st["calls"] == 2 * rs.ntxn and st["max_batch"] <= nthreads
    arrs.close()


@pytest.mark.gpu
@pytest.mark.parametrize("autocollect", [False, True])
def test_gpu_uncollected_callers_share_small_slots(oracle_mod, autocollect):
    # 32 threads calling hip_bdb_osql_serial_check on a narrow window (the
    # small-batch path).  autocollect off: one pass per call, each releasing
    # the context lock while its kernel runs (up to 8 slots in flight); on
    # (the default): the calls join the context's own collector
    v = Validator(0)
    try:
        v.set_autocollect(autocollect)
        wl = config2(n_commits=20_000, n_txn=2_000, seed=13)
        v.ingest_log(wl.log)
        want, _, _ = oracle_mod.check(wl.log, wl.readsets)
        arrs = NativeCurRangeArrs(wl.readsets)
        got, st = v.concurrent_check(arrs, 32, rounds=2, collect=False)
        np.testing.assert_array_equal(got != 0, want != 0)
        if autocollect:
            assert 0 < st["small_path"]["passes"] <= 2 * wl.readsets.ntxn
        else:
            assert st["small_path"]["passes"] == 2 * wl.readsets.ntxn
        arrs.close()
    finally:
        v.close()


@pytest.mark.gpu
def test_gpu_collector_config2_sample(oracle_mod):
    v = Validator(0)
    try:
        wl = config2(n_commits=20_000, n_txn=4_000, seed=11)
        v.ingest_log(wl.log)
        want, _, _ = oracle_mod.check(wl.log, wl.readsets)
        arrs = NativeCurRangeArrs(wl.readsets)
        got, st = v.concurrent_check(arrs, 32)
        np.testing.assert_array_equal(got != 0, want != 0)
        assert st["batches"] < st["calls"]  # calls really were batched
        arrs.close()
    finally:
        v.close()


@pytest.mark.parametrize("autocollect", [True, False])
def test_dropin_entry_autocollect_regop(host, oracle_mod, autocollect):
    """hip_bdb_osql_serial_check through the context's own collector (the
    default) and one pass per call give the same verdicts; bad switch
    values are refused."""
    import ctypes as C
    from comdb2_amd.hsc import load
    lib = load()
    assert lib.hsc_set_autocollect(host.ctx, 2) != 0
    assert lib.hsc_set_autocollect(None, 1) != 0
    host.set_autocollect(autocollect)
    try:
        log, rs = random_case(4242, broken=True, n_txn=300)
        host.ingest_log(log)
        want, _, _ = oracle_mod.check(log, rs, regop_only=1)
        arrs = NativeCurRangeArrs(rs)
        got, _ = host.concurrent_check(arrs, 8, rounds=2, regop_only=1, collect=False)
        np.testing.assert_array_equal(got != 0, want != 0)
        arrs.close()
    finally:
        host.set_autocollect(True)
