"""GPU incremental window: writes committed after a build go to the device
delta run (hsc_delta.hip) and every probe checks it beside the main window;
past its cap the delta folds into the main window with one rebuild.  Verdicts
stay bit-exact against the oracle run on the whole log (oracle/serial_oracle.c):
random logs taken in pieces, a config-2 window with decoded appends, and
BASELINE config 1's full 10k-txn commit stream replayed with an append after
every passing commit (golden: tests/golden/config1_replay.json, the oracle
replay of the same stream)."""
import json
import os

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.hsc import LAYOUT_AUTO, LAYOUT_WIDE
from comdb2_amd.workloads import config1_events, config2, random_case, replay_incremental
from test_incremental import log_slice

pytestmark = pytest.mark.gpu
# torch (device arrays for hsc_window_ingest_device) is imported before the
# validator fixture initialises HIP in this process
torch = pytest.importorskip("torch")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "config1_replay.json")


@pytest.mark.parametrize("seed", range(8))
def test_random_logs_appended_in_pieces(validator, oracle_mod, seed):
    log, rs = random_case(400 + seed, n_commits=120, broken=(seed % 4 == 0))
    want, _, _ = oracle_mod.check(log, rs)
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(1, log.nrec, size=5).tolist()))
    pieces = [0] + cuts + [log.nrec]
    for layout in (LAYOUT_AUTO, LAYOUT_WIDE):
        validator.set_layout(layout)
        validator.ingest_log(log_slice(log, 0, pieces[1]))
        validator.check_readsets(rs)  # built: later pieces go to the delta run
        for a, b in zip(pieces[1:], pieces[2:]):
            validator.append_log(log_slice(log, a, b))
        got = validator.check_readsets(rs)
        np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"layout {layout}")
    validator.set_layout(LAYOUT_AUTO)


def test_config2_window_with_decoded_appends_and_merge(validator, oracle_mod):
    """A config-2 window built from the first 60% of the commits, the rest
    appended as decoded writes in batches of 50 commits: the delta run grows
    past its cap (65536 rows) once, so one append batch is folded into the main
    window by a rebuild; every checkpoint equals the oracle on the log so far."""
    c2 = config2(n_commits=20_000, n_txn=3000, value_bits=28, width=1 << 10, snap_recent=0.3)
    log = c2.log
    R = 13  # records per commit (ltran_start, 10 undo, ltran_commit, regop)
    n0 = 12_000
    validator.set_fold(65536, background=False)  # the inline merge at the run's cap
    try:
        _config2_appends(validator, oracle_mod, c2, log, R, n0)
    finally:
        validator.set_fold(0, background=True)


def _config2_appends(validator, oracle_mod, c2, log, R, n0):
    validator.ingest_log(log_slice(log, 0, n0 * R))
    validator.check_readsets(c2.readsets.with_snaps(np.minimum(c2.readsets.snap, log.lsn[n0 * R - 1])))
    keys = F.enc_int64_array(c2.key_values)
    merged = False
    for c0 in range(n0, 20_000, 50):
        writes = []
        for cc in range(c0, min(c0 + 50, 20_000)):
            for j in range(10):
                writes.append(("t1", 0, bytes(keys[cc * 10 + j]), int(c2.commit_lsn[cc])))
        c1 = min(c0 + 50, 20_000)
        end = int(log.lsn[c1 * R]) if c1 * R < log.nrec else int(log.end_lsn)
        before = validator.delta_rows
        validator.append_writes(writes, end_lsn=end)
        if (c0 // 50) % 40 == 0 or c1 == 20_000:
            sub = log_slice(log, 0, c1 * R)
            rs = c2.readsets.with_snaps(np.minimum(c2.readsets.snap, sub.lsn[-1]))
            want, _, _ = oracle_mod.check(sub, rs, nthreads=8)
            got = validator.check_readsets(rs)
            np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"after commit {c1}")
            merged |= before > 0 and validator.delta_rows == 0  # this check folded the run in
    assert merged


@pytest.mark.parametrize("mode", ["log", "writes"])
def test_config1_full_replay_incremental(validator, mode):
    g = json.load(open(GOLDEN))
    ev = config1_events(n_txn=g["n_txn"])
    got = replay_incremental(ev, validator, mode=mode)
    assert got == g["rc"]
    assert sum(v != 0 for v in got.values()) == g["not_serializable"]


def test_device_ingested_window_appends_and_device_merge(oracle_mod):
    """A window ingested from device arrays (no host copy of its rows) takes
    appends too: they go to the delta run, and past its cap the next check
    folds every version of the window plus the delta into one device rebuild
    (merge_delta) -- verdicts equal the oracle on the whole log."""
    from comdb2_amd.hsc import Validator
    from comdb2_amd.workloads import config2_device_window
    validator = Validator(0)  # own dictionaries: one 9-byte group, 2 key words
    validator.set_fold(65536, background=False)  # the inline merge at the run's cap
    c2 = config2(n_commits=12_000, n_txn=2000, value_bits=26, width=1 << 9, snap_recent=0.5)
    gid, words, lsn = config2_device_window(c2)
    n0 = 4000 * 10  # rows of the first 4000 commits
    dev = torch.device("cuda", 0)
    tg = torch.from_numpy(gid[:n0].copy()).to(dev)
    tw = torch.from_numpy(np.ascontiguousarray(words[:, :n0]).reshape(-1).view(np.int64)).to(dev)
    tl = torch.from_numpy(lsn[:n0].view(np.int64).copy()).to(dev)
    validator.register_group("t1", 0, 9)
    validator.ingest_device(n0, 2, tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), int(c2.log.end_lsn))
    torch.cuda.synchronize()
    keys = F.enc_int64_array(c2.key_values)
    R = 13
    append = lambda c0, c1: validator.append_writes(
        [("t1", 0, bytes(keys[i]), int(lsn[i])) for i in range(c0 * 10, c1 * 10)])
    for c0 in range(4000, 11_000, 1000):  # 7 x 10k rows: past the 65536-row delta cap once
        append(c0, c0 + 1000)
    assert validator.delta_rows == 60_000  # the 7th batch waits for the fold
    sub = log_slice(c2.log, 0, 11_000 * R)
    rs = c2.readsets.with_snaps(np.minimum(c2.readsets.snap, sub.lsn[-1]))
    want, _, _ = oracle_mod.check(sub, rs, nthreads=8)
    np.testing.assert_array_equal(validator.check_readsets(rs) != 0, want != 0)
    assert validator.delta_rows == 0  # folded into the main window by a device rebuild
    append(11_000, 12_000)
    assert validator.delta_rows == 10_000
    want, _, _ = oracle_mod.check(c2.log, c2.readsets, nthreads=8)
    got = validator.check_readsets(c2.readsets)
    np.testing.assert_array_equal(got != 0, want != 0)
    assert 0.05 < (want != 0).mean() < 0.95
    validator.close()


def _device_c2(rows_per_fold, background):
    from comdb2_amd.hsc import Validator
    from comdb2_amd.workloads import config2_device_window
    v = Validator(0)
    v.set_fold(rows_per_fold, background=background)
    c2 = config2(n_commits=12_000, n_txn=2000, value_bits=26, width=1 << 9, snap_recent=0.5)
    gid, words, lsn = config2_device_window(c2)
    n0 = 4000 * 10
    dev = torch.device("cuda", 0)
    tg = torch.from_numpy(gid[:n0].copy()).to(dev)
    tw = torch.from_numpy(np.ascontiguousarray(words[:, :n0]).reshape(-1).view(np.int64)).to(dev)
    tl = torch.from_numpy(lsn[:n0].view(np.int64).copy()).to(dev)
    v.register_group("t1", 0, 9)
    v.ingest_device(n0, 2, tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), int(c2.log.end_lsn))
    torch.cuda.synchronize()
    return v, c2, lsn


def test_background_folds_keep_verdicts(oracle_mod):
    """Background folds (hsc_set_fold: every 3000 delta rows, rebuilt on a
    second stream while checks go on against main + frozen + live runs):
    after every batch of appends the verdicts equal the inline-fold context's
    and, at checkpoints, the oracle's on the log so far."""
    bg, c2, lsn = _device_c2(3000, True)
    il, _, _ = _device_c2(3000, False)
    keys = F.enc_int64_array(c2.key_values)
    R = 13
    try:
        for c0 in range(4000, 12_000, 400):
            writes = [("t1", 0, bytes(keys[i]), int(lsn[i])) for i in range(c0 * 10, (c0 + 400) * 10)]
            bg.append_writes(writes)
            il.append_writes(writes)
            sub_end = (c0 + 400) * R
            rs = c2.readsets.with_snaps(np.minimum(c2.readsets.snap, c2.log.lsn[sub_end - 1]))
            got = bg.check_readsets(rs)
            np.testing.assert_array_equal(got != 0, il.check_readsets(rs) != 0, err_msg=f"commit {c0}")
            if c0 % 2000 == 0:
                want, _, _ = oracle_mod.check(log_slice(c2.log, 0, sub_end), rs, nthreads=8)
                np.testing.assert_array_equal(got != 0, want != 0, err_msg=f"commit {c0}")
        st = bg.fold_stats()
        assert st["started"] >= 10 and st["swapped"] >= 5, st
        assert il.fold_stats()["inline"] >= 10
        # every row is in the window + runs: a full fold gives the oracle's verdicts
        want, _, _ = oracle_mod.check(c2.log, c2.readsets, nthreads=8)
        np.testing.assert_array_equal(bg.check_readsets(c2.readsets) != 0, want != 0)
        g_all = bg.export_window(all_versions=True)
        assert len(g_all[0]) == 12_000 * 10
    finally:
        bg.close()
        il.close()


def test_config1_replay_with_background_folds():
    """The 10k-txn config-1 stream with a fold every ~1000 commits, background
    and inline: both equal the golden verdicts; the background run's slowest
    checks are reported beside the inline run's (the inline fold sits on the
    check path)."""
    import time

    from comdb2_amd.hsc import Validator
    g = json.load(open(GOLDEN))
    ev = config1_events(n_txn=g["n_txn"])
    lat = {}
    for bgmode in (True, False):
        v = Validator(0)
        v.set_fold(2000, background=bgmode)
        t = []
        got = replay_incremental(ev, v, mode="log", check_times=t)
        st = v.fold_stats()
        v.close()
        assert got == g["rc"]
        assert (st["swapped"] if bgmode else st["inline"]) >= 3, st
        lat[bgmode] = np.array(t) * 1e6
    print({k: {"p50": float(np.median(x)), "p99": float(np.percentile(x, 99)), "max": float(x.max())}
           for k, x in lat.items()})
