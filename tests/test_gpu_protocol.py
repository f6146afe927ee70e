"""GPU: the regop_only probe and the master's commit protocol
(db/toblock.c:4757-4836).

* regop_only is answered from the context's published snapshot without the
  context lock or the collector; on a window with appends not yet built, on
  log windows with non-record snapshots (the locked path) and through every
  entry (single call, batch, collector), its verdicts equal the oracle's
  regop_only verdicts on the whole log.
* The protocol harness (hsc_harness_commit_protocol): one thread over the
  config-1 stream reproduces the oracle replay's golden
  (tests/golden/config1_replay.json); 16 and 64 threads produce verdicts that
  workloads.protocol_replay_check confirms against the oracle on the log as
  it stood at every verdict."""
import json
import os

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.hsc import CurRangeArrays, Validator, bdb_osql_serial_check
from comdb2_amd.workloads import (SEED_CONFIG1, config1_events, protocol_replay_check,
                                  random_case)
from test_incremental import log_slice

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "config1_replay.json")


def _arrs(rs):
    sets = []
    for t in range(rs.ntxn):
        a, b = int(rs.txn_off[t]), int(rs.txn_off[t + 1])
        rr = []
        for r in range(a, b):
            key = lambda off, ln: None if int(off) == F.KEY_NULL else bytes(rs.keys[int(off):int(off) + int(ln)])
            rr.append(F.Range(rs.tbnames[rs.table[r]], int(rs.idxnum[r]), key(rs.lkey_off[r], rs.lkeylen[r]),
                              key(rs.rkey_off[r], rs.rkeylen[r]), int(rs.lflag[r]), int(rs.rflag[r]),
                              int(rs.islocked[r])))
        sets.append(rr)
    return CurRangeArrays(sets, [int(s) for s in rs.snap])


@pytest.mark.parametrize("seed", range(6))
def test_regop_probe_on_a_dirty_window_matches_the_oracle(oracle_mod, seed):
    log, rs = random_case(700 + seed, n_commits=150, broken=(seed % 3 == 0))
    want, _, _ = oracle_mod.check(log, rs, regop_only=1)
    v = Validator(0)
    try:
        cut = log.nrec // 3
        v.ingest_log(log_slice(log, 0, cut))
        v.check_readsets(rs)  # built: the rest lands in the delta run / pending tail
        rng = np.random.default_rng(seed)
        pieces = sorted(set(rng.integers(cut + 1, log.nrec, size=3).tolist()))
        for a, b in zip([cut] + pieces, pieces + [log.nrec]):
            v.append_log(log_slice(log, a, b))
        # no full check since the appends: the window is not rebuilt or merged
        for collect in (True, False):
            v.set_autocollect(collect)
            arrs = _arrs(rs)
            got = np.array([bdb_osql_serial_check(v, a, regop_only=1) for a in arrs.arrs])
            np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"single, collect={collect}")
            # regop_only leaves the snapshots alone
            np.testing.assert_array_equal([(a.file << 32) | a.offset for a in arrs.arrs], rs.snap)
        got = v.check_batch(_arrs(rs), regop_only=1)
        np.testing.assert_array_equal(got != 0, want != 0, err_msg="batch")
        st = v.regop_stats()
        assert st["fast"] > 0
        # the full check afterwards still agrees (the probes changed nothing)
        full, _, _ = oracle_mod.check(log, rs)
        np.testing.assert_array_equal(v.check_readsets(rs) != 0, full != 0)
    finally:
        v.close()


def test_regop_probe_through_a_collector(oracle_mod):
    log, rs = random_case(777, n_commits=200)
    want, _, _ = oracle_mod.check(log, rs, regop_only=1)
    v = Validator(0)
    try:
        v.ingest_log(log)
        got, st = v.concurrent_check(_arrs(rs), 8, regop_only=1)
        np.testing.assert_array_equal(got[:rs.ntxn] != 0, want != 0)
        assert st["batches"] == 0  # never queued: no collector pass ran
    finally:
        v.close()


def _txns(events):
    return [t for e, t in events if e == "begin"]


def test_one_thread_protocol_equals_the_golden():
    events = config1_events(seed=SEED_CONFIG1, n_txn=10_000)
    txns = _txns(events)
    v = Validator(0)
    try:
        v.ingest_log(F.LogBuilder().build())
        rc, seq, snap, cend, st = v.commit_protocol(txns, events, 1)
    finally:
        v.close()
    golden = json.load(open(GOLDEN))["rc"]
    got = {t.name: int(rc[i]) for i, t in enumerate(txns) if t.writes}
    assert got == golden
    assert st["commits"] + st["aborts"] == len(golden)
    assert st["regop_locked"] == 0 and st["regop_fast"] == st["regop_probes"] > 0


@pytest.mark.parametrize("threads", [16, 64])
def test_concurrent_protocol_verdicts_match_the_oracle(oracle_mod, threads):
    events = config1_events(seed=SEED_CONFIG1 + threads, n_txn=4000)
    txns = _txns(events)
    v = Validator(0)
    try:
        v.ingest_log(F.LogBuilder().build())
        e0 = v.end_lsn
        rc, seq, snap, cend, st = v.commit_protocol(txns, events, threads)
    finally:
        v.close()
    assert st["aborts"] > 0 and st["commits"] > 0
    out = protocol_replay_check(txns, rc, seq, snap, cend, e0,
                                lambda log, rs: oracle_mod.check(log, rs)[0])
    assert out["mismatches"] == 0, out
    assert out["checked"] == len(txns)
    assert st["regop_locked"] == 0
