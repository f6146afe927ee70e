"""GPU: the multi-GPU context behind the C ABI (hsc_multi.cpp, hsc_route.hip;
SURVEY.md §8(e)).  On the one GPU of a test box, 2 and 4 member contexts
share cuda:0:
- the drop-in entries route each batch on the host while marshalling, and
  every member holding a probe checks its share (its small kernel for a
  lone call);
- device-resident batches routed on the device: direct stores into the
  other members' probe columns (the in-process path over xGMI), or the
  loopback transport -- the per-rank form (send blocks, k_route_unpack,
  owner slices gathered and OR-ed) with peer copies in place of RCCL;
- batches routed at marshal time (hsc_multi_probe_routed), both merges;
- a per-rank context of world 1 (RCCL loaded; one piece: no routing);
- replicated windows (HSC_MULTI_REPLICAS, the AUTO choice for a window that
  fits): every member holds the whole window, a lone call runs one member's
  kernel, a large batch is cut into per-member slices of read sets.
Verdicts are checked against the oracle (oracle/serial_oracle.c on the whole
log) and against one context holding the whole window."""
import json
import os

import numpy as np
import pytest

from comdb2_amd import hsc
from comdb2_amd.hsc import MultiValidator, Validator
from comdb2_amd.workloads import (config1_events, config3_arrays, config3_log, config5_log,
                                  config5_scaled, random_case, replay_incremental)
from test_incremental import log_slice

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "config1_replay.json")


@pytest.fixture(scope="module", params=[(2, hsc.MULTI_PIECES), (4, hsc.MULTI_PIECES),
                                        (2, hsc.MULTI_REPLICAS), (3, hsc.MULTI_REPLICAS)],
                ids=["pieces2", "pieces4", "replicas2", "replicas3"])
def multi(request):
    n, mode = request.param
    m = MultiValidator([0] * n)
    m.set_mode(mode)
    m.want_mode = mode
    yield m
    m.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_logs_vs_oracle(multi, oracle_mod, seed):
    log, rs = random_case(700 + seed, n_commits=150, n_txn=60, broken=(seed % 3 == 0))
    want, _, _ = oracle_mod.check(log, rs)
    multi.ingest_log(log)
    got = multi.check_readsets(rs)
    np.testing.assert_array_equal(got != 0, want != 0)
    # the same read sets through the drop-in entry (CurRangeArr*, file/offset in place)
    arrs = hsc.NativeCurRangeArrs(rs)
    try:
        got2 = multi.check_batch(arrs)
    finally:
        arrs.close()
    np.testing.assert_array_equal(got2 != 0, want != 0)
    assert multi.mode == multi.want_mode


@pytest.mark.parametrize("seed", range(4))
def test_random_logs_appended_in_pieces(multi, oracle_mod, seed):
    """Appended records are decoded by the front context and their rows go to
    their owners' delta runs."""
    log, rs = random_case(800 + seed, n_commits=150, n_txn=50)
    want, _, _ = oracle_mod.check(log, rs)
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(1, log.nrec, size=5).tolist()))
    pieces = [0] + cuts + [log.nrec]
    multi.ingest_log(log_slice(log, 0, pieces[1]))
    multi.check_readsets(rs)  # built: the rest goes to the members' delta runs
    for a, b in zip(pieces[1:], pieces[2:]):
        multi.append_log(log_slice(log, a, b))
    np.testing.assert_array_equal(multi.check_readsets(rs) != 0, want != 0)


def _sample_vs_oracle(oracle_mod, got, rs, tail_log, step):
    sample = np.arange(0, rs.ntxn, step)
    want, _, _ = oracle_mod.check(tail_log, rs.subset(sample), nthreads=16)
    np.testing.assert_array_equal(got[sample], want != 0)


def test_config3_vs_oracle_and_one_context(multi, oracle_mod):
    """Config 3 (32 composite-key groups): the pieces cut across groups and
    inside the big ones; table-lock probes go to member 0."""
    a = config3_arrays(n_writes=300_000, n_txn=6000)
    log = config3_log(a)
    multi.ingest_log(log)
    got = multi.check_readsets(a.readsets) != 0
    one = Validator(0)
    try:
        one.ingest_log(log)
        ref = one.check_readsets(a.readsets) != 0
    finally:
        one.close()
    np.testing.assert_array_equal(got, ref)
    assert 0.1 < got.mean() < 0.9
    _sample_vs_oracle(oracle_mod, got, a.readsets, log, 20)
    st = multi.route_stats()
    assert st["member_checks"] >= multi.world  # every member checked a share of the batch
    if multi.want_mode == hsc.MULTI_PIECES:
        assert st["rows"] >= st["probes"] > 0


def test_config5_vs_oracle_and_one_context(multi, oracle_mod):
    """Config 5 (Zipf(1.2) hot keys): equal-row splitters put the hot low keys
    on member 0's piece; verdicts are unaffected."""
    c5 = config5_scaled(keys_per_gpu=400_000, n_txn=5000)
    log = config5_log([c5.keys], keys_per_commit=10)
    multi.ingest_log(log)
    got = multi.check_readsets(c5.readsets) != 0
    one = Validator(0)
    try:
        one.ingest_log(log)
        ref = one.check_readsets(c5.readsets) != 0
    finally:
        one.close()
    np.testing.assert_array_equal(got, ref)
    assert 0.1 < got.mean() < 0.9
    _sample_vs_oracle(oracle_mod, got, c5.readsets, log, 25)


def test_explicit_splitters_and_straddling_ranges(oracle_mod):
    """Splitters inside dense key runs: many ranges straddle two pieces and are
    probed on both members (routed > probes); verdicts still equal."""
    log, rs = random_case(901, n_commits=300, n_txn=120, value_range=16)
    want, _, _ = oracle_mod.check(log, rs)
    m = MultiValidator([0, 0, 0])
    try:
        m.ingest_log(log)
        m.check_readsets(rs)
        # splitters at two existing keys of the window's first group
        one = Validator(0)
        one.ingest_log(log)
        gid, words, _ = one.export_window()
        one.close()
        sel = np.nonzero(gid == gid[len(gid) // 2])[0]
        k = sel[[len(sel) // 3, 2 * len(sel) // 3]]
        m.set_splitters(gid[k], words[:, k])
        got = m.check_readsets(rs)
        np.testing.assert_array_equal(got != 0, want != 0)
        st = m.route_stats()
        assert st["rows"] > st["probes"] > 0  # straddling ranges went to both members
    finally:
        m.close()


@pytest.mark.parametrize("mode", [hsc.MULTI_PIECES, hsc.MULTI_REPLICAS])
def test_config1_commit_stream_golden(mode):
    """BASELINE config 1's 10k-txn stream through a 2-member context: one
    check per commit, every passing txn's log records appended (routed to the
    owners' delta runs, or to every replica); verdicts equal the oracle
    replay's golden."""
    gold = json.load(open(GOLDEN))
    m = MultiValidator([0, 0])
    try:
        m.set_mode(mode)
        rc = replay_incremental(config1_events(n_txn=gold["n_txn"]), m, mode="log")
        assert m.mode == mode
    finally:
        m.close()
    assert rc == gold["rc"]


def _device_batch(v, rs, dev):
    mm = v.marshal(rs)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    b = dict(lo=t(mm["lo"]), hi=t(mm["hi"]), gid=t(mm["gid"]), snap=t(mm["snap"]), txn=t(mm["txn"]),
             lock_table=t(mm["lock_table"]), lock_snap=t(mm["lock_snap"]),
             lock_txn=t(mm["lock_txn"]), n=mm["n"], n_lock=mm["n_lock"], forced=mm["forced"])
    T = rs.ntxn
    b["bits"] = torch.zeros((T + 63) // 64, dtype=torch.int64, device=dev)
    b["verdict"] = torch.zeros(max(T, 1), dtype=torch.uint8, device=dev)
    b["struct"] = hsc.ProbeBatch(b["n"], b["lo"].data_ptr(), b["hi"].data_ptr(), b["gid"].data_ptr(),
                                 b["snap"].data_ptr(), b["txn"].data_ptr(), b["n_lock"],
                                 b["lock_table"].data_ptr(), b["lock_snap"].data_ptr(),
                                 b["lock_txn"].data_ptr(), T, b["verdict"].data_ptr(),
                                 b["bits"].data_ptr())
    return b


def _bits(b, T):
    x = b["bits"].cpu().numpy().view(np.uint8)
    return np.maximum(np.unpackbits(x, bitorder="little")[:T], b["forced"]).astype(bool)


@pytest.mark.parametrize("n", [2, 4])
def test_probe_device_per_member_batches(oracle_mod, n):
    """hsc_multi_probe_device: each member holds its own resident batch (read
    sets numbered from 0), routes it, and receives the merged verdicts of its
    own read sets -- the bench's per-GPU step; both lanes."""
    a = config3_arrays(n_writes=200_000, n_txn=4000 * n)
    log = config3_log(a)
    one = Validator(0)
    m = MultiValidator([0] * n)
    try:
        m.set_mode(hsc.MULTI_PIECES)
        one.ingest_log(log)
        m.ingest_log(log)
        dev = torch.device("cuda", 0)
        T = 4000
        parts = [a.readsets.subset(np.arange(i * T, (i + 1) * T)) for i in range(n)]
        want = [one.check_readsets(p) != 0 for p in parts]
        batches = [_device_batch(m, p, dev) for p in parts]
        torch.cuda.synchronize()
        for lane in (0, 1, 0):
            for b in batches:
                b["bits"].zero_()
            torch.cuda.synchronize()
            m.probe_device_multi([b["struct"] for b in batches], lane=lane)
            torch.cuda.synchronize()
            for i, b in enumerate(batches):
                np.testing.assert_array_equal(_bits(b, T), want[i], err_msg=f"member {i} lane {lane}")
    finally:
        m.close()
        one.close()


@pytest.mark.parametrize("n", [2, 4])
def test_loopback_transport_per_member_batches(oracle_mod, n):
    """The per-rank pipeline's data paths on one process: send blocks laid out
    per destination (block_target), moved by peer copies in place of
    ncclSend / ncclRecv, k_route_unpack's row and lock offsets, and the owner
    slices gathered and OR-ed -- every step a per-rank context runs between
    ranks, against one context's verdicts; both lanes."""
    a = config3_arrays(n_writes=200_000, n_txn=3000 * n)
    log = config3_log(a)
    one = Validator(0)
    m = MultiValidator([0] * n)
    try:
        m.set_mode(hsc.MULTI_PIECES)
        one.ingest_log(log)
        m.ingest_log(log)
        m.set_transport(True)
        dev = torch.device("cuda", 0)
        T = 3000
        parts = [a.readsets.subset(np.arange(i * T, (i + 1) * T)) for i in range(n)]
        want = [one.check_readsets(p) != 0 for p in parts]
        batches = [_device_batch(m, p, dev) for p in parts]
        torch.cuda.synchronize()
        for lane in (0, 1, 1):
            for b in batches:
                b["bits"].zero_()
            torch.cuda.synchronize()
            m.probe_device_multi([b["struct"] for b in batches], lane=lane)
            torch.cuda.synchronize()
            for i, b in enumerate(batches):
                np.testing.assert_array_equal(_bits(b, T), want[i], err_msg=f"member {i} lane {lane}")
        cnt = m.last_counts()
        assert (cnt - np.diag(np.diag(cnt))).sum() > 0  # probes crossed members
        assert sum(b["n_lock"] for b in batches) > 0    # locks travelled to member 0
        # the drop-in entry is unaffected by the transport (host routing)
        np.testing.assert_array_equal(m.check_readsets(parts[0]) != 0, want[0])
    finally:
        m.close()
        one.close()


def _routed_device_batch(mb, dev, bits_words):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    b = dict(lo=t(mb["lo"]), hi=t(mb["hi"]), gid=t(mb["gid"]), snap=t(mb["snap"]), txn=t(mb["txn"]),
             lock_table=t(mb["lock_table"]), lock_snap=t(mb["lock_snap"]), lock_txn=t(mb["lock_txn"]))
    b["bits"] = torch.zeros(max(bits_words, 1), dtype=torch.int64, device=dev)
    b["verdict"] = torch.zeros(max(mb["n_txn"], 1), dtype=torch.uint8, device=dev)
    b["struct"] = hsc.ProbeBatch(mb["n"], b["lo"].data_ptr(), b["hi"].data_ptr(), b["gid"].data_ptr(),
                                 b["snap"].data_ptr(), b["txn"].data_ptr(), mb["n_lock"],
                                 b["lock_table"].data_ptr(), b["lock_snap"].data_ptr(),
                                 b["lock_txn"].data_ptr(), mb["n_txn"], b["verdict"].data_ptr(),
                                 b["bits"].data_ptr())
    return b


@pytest.mark.parametrize("n,loop", [(2, False), (4, False), (2, True), (3, True)])
def test_probe_routed_at_marshal(oracle_mod, n, loop):
    """hsc_multi_probe_routed: the global batch = n owners' shares (sizes not
    multiples of 64), each share marshalled and routed on the host
    (hsc_multi_marshal_routed), every member probes only the ranges that
    overlap its piece, the bitmaps are OR-ed per owner (peer reads, or the
    per-rank slice exchange by loopback copies)."""
    a = config3_arrays(n_writes=200_000, n_txn=2500 * n + 7)
    log = config3_log(a)
    one = Validator(0)
    m = MultiValidator([0] * n)
    try:
        m.set_mode(hsc.MULTI_PIECES)
        one.ingest_log(log)
        m.ingest_log(log)
        m.check_readsets(a.readsets.subset(np.arange(4)))  # built and partitioned
        m.set_transport(loop)
        dev = torch.device("cuda", 0)
        cuts = [0] + [2500 * i + 3 * i for i in range(1, n)] + [a.readsets.ntxn]
        shares = [a.readsets.subset(np.arange(cuts[i], cuts[i + 1])) for i in range(n)]
        want = [one.check_readsets(s) != 0 for s in shares]
        rt = m.routed_shares(shares, list(range(n)))
        routed = [rt[i] for i in range(n)]
        ob = routed[0]["owner_base"]
        batches = [_routed_device_batch(routed[i], dev, int((ob[i + 1] - ob[i]) // 64)) for i in range(n)]
        assert sum(r["n"] for r in routed) >= sum(m.marshal(s)["n"] for s in shares)
        assert all(r["n_lock"] == 0 for r in routed[1:])
        torch.cuda.synchronize()
        for lane in (0, 1):
            for b in batches:
                b["bits"].zero_()
            torch.cuda.synchronize()
            m.probe_routed([b["struct"] for b in batches], ob, lane=lane)
            torch.cuda.synchronize()
            for i, b in enumerate(batches):
                T = shares[i].ntxn
                got = np.unpackbits(b["bits"].cpu().numpy().view(np.uint8), bitorder="little")[:T]
                got = np.maximum(got, routed[0]["forced"][i]).astype(bool)
                np.testing.assert_array_equal(got, want[i], err_msg=f"owner {i} lane {lane}")
    finally:
        m.close()
        one.close()


def test_lone_calls_route_to_one_member(oracle_mod):
    """The drop-in entry on a 2-member context, one read set per call (the
    per-transaction pattern of db/toblock.c:4777-4800): the host routing
    sends each call only to the members its ranges overlap, whose small
    kernels answer it."""
    from comdb2_amd.workloads import config2
    # one int64 index (narrow windows: the small path); one range per read
    # set, so most calls touch one member (a read set of 10 uniform ranges
    # nearly always touches both halves of the key space)
    c2 = config2(n_commits=4000, n_txn=60, value_bits=24, width=1 << 10, ranges_per_txn=1)
    log, rs = c2.log, c2.readsets
    want, _, _ = oracle_mod.check(log, rs)
    m = MultiValidator([0, 0])
    try:
        m.set_mode(hsc.MULTI_PIECES)
        m.ingest_log(log)
        got = np.array([m.check_readsets(rs.subset(np.array([t])))[0] for t in range(rs.ntxn)])
        np.testing.assert_array_equal(got != 0, want != 0)
        st = m.route_stats()
        assert st["calls"] >= rs.ntxn
        assert st["member_checks"] < 2 * st["calls"]  # some calls touched one member only
        small = sum(m.member(i).small_stats()["calls"] for i in range(2))
        assert small >= st["member_checks"] // 2
    finally:
        m.close()


def test_replicas_lone_calls_run_one_member_each(oracle_mod):
    """A replicated window (AUTO: the window fits): every lone drop-in call
    runs exactly one member's small kernel, the members taking turns; a large
    batch is cut into one slice per member.  Verdicts equal the oracle."""
    from comdb2_amd.workloads import config2
    c2 = config2(n_commits=4000, n_txn=400, value_bits=24, width=1 << 10)
    log, rs = c2.log, c2.readsets
    want, _, _ = oracle_mod.check(log, rs)
    m = MultiValidator([0, 0, 0])
    try:
        m.ingest_log(log)
        got = np.array([m.check_readsets(rs.subset(np.array([t])))[0] for t in range(60)])
        np.testing.assert_array_equal(got != 0, want[:60] != 0)
        assert m.mode == hsc.MULTI_REPLICAS
        st = m.route_stats()
        assert st["member_checks"] == st["calls"] == 60  # one member per call
        small = [m.member(i).small_stats()["calls"] for i in range(3)]
        assert sum(small) == 60 and min(small) > 0  # every member took calls
        # the whole batch through the drop-in batch entry: sliced over the members
        arrs = hsc.NativeCurRangeArrs(rs)
        try:
            big = m.check_batch(arrs)
        finally:
            arrs.close()
        np.testing.assert_array_equal(big != 0, want != 0)
        # concurrent callers through the context's collector
        arrs = hsc.NativeCurRangeArrs(rs)
        try:
            got, cst = m.concurrent_check(arrs, 16, collect=False)
        finally:
            arrs.close()
        np.testing.assert_array_equal(got[:rs.ntxn] != 0, want != 0)
    finally:
        m.close()


def test_replicas_adopted_and_device_batches(oracle_mod):
    """Every member ingests the whole window from device rows; with
    HSC_MULTI_REPLICAS hsc_multi_adopt needs no splitters and refuses members
    holding different rows; device batches are probed by each member against
    its replica (no routing)."""
    from comdb2_amd.workloads import config2
    c2 = config2(n_commits=20_000, n_txn=2000, value_bits=24, width=1 << 8)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets)
    one = Validator(0)
    one.ingest_log(c2.log)
    gid, words, lsn = one.export_window(all_versions=True)
    one.close()
    order = np.argsort(lsn, kind="stable")
    dev = torch.device("cuda", 0)

    def ingest(m, i, sel):
        tg = torch.from_numpy(np.ascontiguousarray(gid[sel])).to(dev)
        tw = torch.from_numpy(np.ascontiguousarray(words[:, sel]).reshape(-1).view(np.int64)).to(dev)
        tl = torch.from_numpy(np.ascontiguousarray(lsn[sel]).view(np.int64)).to(dev)
        torch.cuda.synchronize()
        m.member(i).ingest_device(len(sel), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                                  c2.params["end_lsn"])

    m = MultiValidator([0, 0])
    try:
        m.register_group("t1", 0, 9)
        m.set_mode(hsc.MULTI_REPLICAS)
        ingest(m, 0, order)
        ingest(m, 1, order[: len(order) // 2])  # not a replica
        with pytest.raises(hsc.HscError):
            m.adopt()
        ingest(m, 1, order)
        m.adopt()
        assert m.mode == hsc.MULTI_REPLICAS
        m.set_end(c2.params["end_lsn"])
        np.testing.assert_array_equal(m.check_readsets(c2.readsets) != 0, want != 0)
        # device batches: member i probes read sets [i T/2, (i+1) T/2) against its replica
        T = c2.readsets.ntxn
        halves = [c2.readsets.subset(np.arange(i * T // 2, (i + 1) * T // 2)) for i in range(2)]
        batches = [_device_batch(m.member(i), halves[i], dev) for i in range(2)]
        torch.cuda.synchronize()
        m.probe_device_multi([b["struct"] for b in batches], lane=0)
        torch.cuda.synchronize()
        for i in range(2):
            np.testing.assert_array_equal(_bits(batches[i], halves[i].ntxn),
                                          want[i * T // 2:(i + 1) * T // 2] != 0)
    finally:
        m.close()


def test_rccl_world1_rank_context(oracle_mod):
    """A per-rank (RCCL) context at world 1 on the box's one GPU: librccl
    loaded and the communicators built; one piece, so the drop-in batch and a
    device batch are probed where they are (no routing kernels, no exchange)
    -- the world-1 step of bench.py --rank-path."""
    ids = MultiValidator.unique_ids()
    m = MultiValidator(rank=0, world=1, ids=ids, device=0)
    try:
        assert (m.world, m.rank, m.nlocal) == (1, 0, 1)
        log, rs = random_case(950, n_commits=200, n_txn=80)
        want, _, _ = oracle_mod.check(log, rs)
        m.ingest_log(log)
        np.testing.assert_array_equal(m.check_readsets(rs) != 0, want != 0)
        b = _device_batch(m, rs, torch.device("cuda", 0))
        torch.cuda.synchronize()
        m.probe_device_multi([b["struct"]], lane=1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_bits(b, rs.ntxn), want != 0)
    finally:
        m.close()


def test_adopted_member_windows(oracle_mod):
    """Members ingested directly from device rows (each exactly its piece),
    hsc_multi_adopt, then the drop-in check on the multi context."""
    from comdb2_amd.workloads import config2
    c2 = config2(n_commits=20_000, n_txn=2000, value_bits=24, width=1 << 8)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets)
    one = Validator(0)
    one.ingest_log(c2.log)
    gid, words, lsn = one.export_window(all_versions=True)
    one.close()
    m = MultiValidator([0, 0])
    try:
        assert m.register_group("t1", 0, 9) == 0
        S = 1
        # the splitter is a key of the window; member 1's piece starts at its
        # first version (all versions of a key live on one member)
        mid = len(gid) // 2
        same = (gid == gid[mid]) & (words == words[:, [mid]]).all(axis=0)
        cut = int(np.nonzero(same)[0][0])
        m.set_splitters(gid[[cut]], words[:, [cut]])
        dev = torch.device("cuda", 0)
        for i, (a, e) in enumerate(((0, cut), (cut, len(gid)))):
            # versions in log order inside the piece (the rows of one key ascend)
            order = np.argsort(lsn[a:e], kind="stable") + a
            tg = torch.from_numpy(np.ascontiguousarray(gid[order])).to(dev)
            tw = torch.from_numpy(np.ascontiguousarray(words[:, order]).reshape(-1).view(np.int64)).to(dev)
            tl = torch.from_numpy(np.ascontiguousarray(lsn[order]).view(np.int64)).to(dev)
            torch.cuda.synchronize()
            m.member(i).ingest_device(e - a, words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                                      c2.params["end_lsn"])
        m.adopt()
        with pytest.raises(hsc.HscError):  # appends go to the members of an adopted context
            m.append_writes([("t1", 0, b"\x08" * 9, int(c2.params["end_lsn"]) + 1)])
        m.set_end(c2.params["end_lsn"])
        got = m.check_readsets(c2.readsets)
        assert S == 1
        # device windows have no log: the DB_SET-on-a-non-record rule is off,
        # and these snapshots are all record LSNs, so the verdicts are the oracle's
        np.testing.assert_array_equal(got != 0, want != 0)
    finally:
        m.close()


def test_adopt_checks_splitters_and_pieces():
    """hsc_multi_adopt refuses a world > 1 context without splitters (every
    probe would go to member 0) and members holding keys outside their piece."""
    from comdb2_amd.workloads import config2
    c2 = config2(n_commits=2000, n_txn=10, value_bits=24, width=1 << 8)
    one = Validator(0)
    one.ingest_log(c2.log)
    gid, words, lsn = one.export_window(all_versions=True)
    one.close()
    dev = torch.device("cuda", 0)

    def ingest(m, i, sel):
        order = sel[np.argsort(lsn[sel], kind="stable")]
        tg = torch.from_numpy(np.ascontiguousarray(gid[order])).to(dev)
        tw = torch.from_numpy(np.ascontiguousarray(words[:, order]).reshape(-1).view(np.int64)).to(dev)
        tl = torch.from_numpy(np.ascontiguousarray(lsn[order]).view(np.int64)).to(dev)
        torch.cuda.synchronize()
        m.member(i).ingest_device(len(order), words.shape[0], tg.data_ptr(), tw.data_ptr(),
                                  tl.data_ptr(), c2.params["end_lsn"])

    mid = len(gid) // 2
    cut = int(np.nonzero((gid == gid[mid]) & (words == words[:, [mid]]).all(axis=0))[0][0])
    halves = (np.arange(cut), np.arange(cut, len(gid)))
    m = MultiValidator([0, 0])
    try:
        m.register_group("t1", 0, 9)
        for i in range(2):
            ingest(m, i, halves[i])
        with pytest.raises(hsc.HscError):  # no splitters
            m.adopt()
        m.set_splitters(gid[[cut]], words[:, [cut]])
        m.adopt()
    finally:
        m.close()
    m = MultiValidator([0, 0])
    try:
        m.register_group("t1", 0, 9)
        for i in range(2):
            ingest(m, i, halves[1 - i])  # pieces swapped
        m.set_splitters(gid[[cut]], words[:, [cut]])
        with pytest.raises(hsc.HscError):
            m.adopt()
    finally:
        m.close()
