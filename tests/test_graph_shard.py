"""Config 4 over N GPUs: the dependency graph + SCC sharded by key
(comdb2_amd/shard.py sharded_scc; hsc_dep_graph_build / _cover / _cut /
_scc_cut).  The cover lemma (every txn of a nontrivial component lies inside
[dst, src] of a backward edge) and the whole flow are checked on CPU with a
Python model of the four device steps -- simulated shards and world_size 2
over gloo -- against Tarjan (oracle/scc_oracle.c) on the unsharded history;
the -m gpu tests run the same flow through the C ABI, one context per shard
on one GPU."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(__file__))
from test_graph import py_edges, py_scc  # noqa: E402

from comdb2_amd import shard  # noqa: E402
from comdb2_amd.workloads import config4_history  # noqa: E402

CASES = [
    dict(seed=1, n_txn=1500, n_keys=60, concurrent_frac=0.2, max_lag=6),
    dict(seed=2, n_txn=2500, n_keys=400, concurrent_frac=0.05, max_lag=32),
    dict(seed=3, n_txn=1200, n_keys=30, concurrent_frac=0.3, max_lag=8, zipf=1.2),
]


class ModelGraph:
    """The four device steps restated over Python edge sets (CPU tensors)."""

    def build(self, h):
        self.E, self.ntxn = py_edges(h), h.ntxn
        return {"edges": len(self.E)}

    def cover(self, cover):
        import torch
        diff = np.zeros(self.ntxn + 2, np.int64)
        for a, b in self.E:
            if a > b:
                diff[b] += 1
                diff[a + 1] -= 1
        c = (np.cumsum(diff)[: self.ntxn] > 0).astype(np.uint8)
        cover[: self.ntxn] = torch.from_numpy(c)

    def cut(self, cover):
        import torch
        cv = cover.numpy()
        rows = sorted((a << 32) | b for a, b in self.E if cv[a] and cv[b])
        return torch.tensor(rows, dtype=torch.int64)

    def scc_cut(self, ntxn, cover, rows, scc):
        import torch
        cv = cover.numpy()
        E = {}
        for r in rows.tolist():
            if r == -1:
                continue
            a, b = r >> 32, r & 0xFFFFFFFF
            assert cv[a] and cv[b]
            E[(a, b)] = 1
        scc[:ntxn] = torch.from_numpy(py_scc(ntxn, E).astype(np.int32))
        return {}


def _cover_of(E, n):
    diff = np.zeros(n + 2, np.int64)
    for a, b in E:
        if a > b:
            diff[b] += 1
            diff[a + 1] -= 1
    return np.cumsum(diff)[:n] > 0


@pytest.mark.parametrize("kw", CASES)
def test_cover_lemma(kw):
    h = config4_history(**kw)
    E = py_edges(h)
    scc = py_scc(h.ntxn, E)
    cyc = np.bincount(scc, minlength=h.ntxn)[scc] > 1
    assert cyc.any()
    cov = _cover_of(E, h.ntxn)
    assert not (cyc & ~cov).any()
    if kw["concurrent_frac"] <= 0.05:
        assert cov.mean() < 0.5  # the cut is a small part of the graph


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("kw", CASES)
def test_key_shards_partition_edges(kw, world):
    h = config4_history(**kw)
    E = py_edges(h)
    parts = [py_edges(shard.history_shard(h, r, world)) for r in range(world)]
    union = {}
    for p in parts:
        for e, t in p.items():
            union[e] = union.get(e, 0) | t
    assert union == E
    # simulated ranks: OR of covers, union of cuts, SCC of the cut = Tarjan
    cov = np.zeros(h.ntxn, bool)
    for p in parts:
        cov |= _cover_of(p, h.ntxn)
    cut = {e: 1 for p in parts for e in p if cov[e[0]] and cov[e[1]]}
    np.testing.assert_array_equal(py_scc(h.ntxn, cut), py_scc(h.ntxn, E))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for i, kw in enumerate(CASES):
        h = config4_history(**kw)
        scc, st = shard.sharded_scc(ModelGraph(), shard.history_shard(h, rank, world), h.ntxn,
                                    torch.device("cpu"))
        out[f"scc{i}_{rank}"] = scc.numpy()
    np.savez(out_path + f".{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_oracle(tmp_path, oracle_mod):
    import torch.multiprocessing as mp
    out = str(tmp_path / "scc")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    for i, kw in enumerate(CASES):
        h = config4_history(**kw)
        s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
        want = oracle_mod.scc(h.ntxn, s, d)
        for r in range(2):
            got = np.load(out + f".{r}.npz")[f"scc{i}_{r}"]
            np.testing.assert_array_equal(got.astype(np.uint32), want)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("kw", CASES + [
    dict(n_txn=200000, n_keys=5000, concurrent_frac=0.05, max_lag=32),
    dict(n_txn=300000, n_keys=300, concurrent_frac=0.3, max_lag=8, zipf=1.2),
    dict(n_txn=1000000, n_keys=100000),
])
def test_gpu_key_shards_match_oracle(oracle_mod, kw, world):
    """N contexts on one GPU stand in for N ranks: OR of covers, concatenated
    (padded) cuts, SCC of the cut on shard 0 = Tarjan over the whole history."""
    import torch
    from comdb2_amd.hsc import Validator
    h = config4_history(**kw)
    dev = torch.device("cuda", 0)
    vs = [Validator(0) for _ in range(world)]
    gs = [shard.GpuGraph(v, dev, full=(r == 1)) for r, v in enumerate(vs)]  # raw and full builds
    try:
        for r, g in enumerate(gs):
            hs = shard.history_shard(h, r, world)
            g.build(shard.device_history(hs, dev) if r % 2 else hs)
        cover = torch.zeros(h.ntxn, dtype=torch.uint8, device=dev)
        for g in gs:
            c = torch.zeros_like(cover)
            g.cover(c)
            cover = torch.maximum(cover, c)
        cuts = [g.cut(cover) for g in gs]
        pad = torch.full((7,), -1, dtype=torch.int64, device=dev)
        rows = torch.cat([x for c in cuts for x in (c, pad)])
        scc = torch.empty(h.ntxn, dtype=torch.int32, device=dev)
        st = gs[0].scc_cut(h.ntxn, cover, rows, scc)
        s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
        want = oracle_mod.scc(h.ntxn, s, d)
        np.testing.assert_array_equal(scc.cpu().numpy().astype(np.uint32), want)
        cyc = np.bincount(want, minlength=h.ntxn)[want] > 1
        assert st["txns_in_cycles"] == int(cyc.sum())
        assert st["cut_nodes"] == int(cover.sum().item())
        # the whole-history call agrees and the cover holds every cycle
        full, _ = vs[0].dep_graph_scc(h)
        np.testing.assert_array_equal(full, want)
        assert not (cyc & (cover.cpu().numpy() == 0)).any()
    finally:
        for v in vs:
            v.close()


@pytest.mark.gpu
def test_gpu_scc_cut_rejects_rows_outside_cover():
    import torch
    from comdb2_amd.hsc import HscError, Validator
    v = Validator(0)
    try:
        dev = torch.device("cuda", 0)
        cover = torch.tensor([1, 1, 0, 1], dtype=torch.uint8, device=dev)
        rows = torch.tensor([(0 << 32) | 2], dtype=torch.int64, device=dev)
        scc = torch.empty(4, dtype=torch.int32, device=dev)
        with pytest.raises(HscError):
            shard.GpuGraph(v, dev).scc_cut(4, cover, rows, scc)
        rows = torch.tensor([(0 << 32) | 1, (1 << 32) | 3, (3 << 32) | 0, -1], dtype=torch.int64,
                            device=dev)
        shard.GpuGraph(v, dev).scc_cut(4, cover, rows, scc)
        assert scc.cpu().tolist() == [3, 3, 2, 3]
    finally:
        v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("kw", CASES + [
    dict(n_txn=300000, n_keys=300, concurrent_frac=0.3, max_lag=8, zipf=1.2),
    dict(n_txn=1000000, n_keys=100000),
])
def test_gpu_multi_graph_scc_matches_oracle(oracle_mod, kw, world):
    """hsc_multi_graph_scc: the sharded step behind the C ABI -- members of an
    in-process multi context on the one GPU, each with its key shard's
    device-resident ops: covers OR-ed over the members, cuts gathered to
    member 0, its colouring SCC copied to every member = Tarjan over the
    whole history (oracle/scc_oracle.c)."""
    import torch
    from comdb2_amd.hsc import MultiValidator
    h = config4_history(**kw)
    dev = torch.device("cuda", 0)
    m = MultiValidator([0] * world)
    try:
        shards = [shard.device_history(shard.history_shard(h, r, world), dev) for r in range(world)]
        sccs = [torch.zeros(h.ntxn, dtype=torch.int32, device=dev) for _ in range(world)]
        torch.cuda.synchronize()
        st = m.graph_scc(shards, h.ntxn, [x.data_ptr() for x in sccs])
        s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
        want = oracle_mod.scc(h.ntxn, s, d)
        for r in range(world):
            np.testing.assert_array_equal(sccs[r].cpu().numpy().astype(np.uint32), want,
                                          err_msg=f"member {r}")
        cyc = np.bincount(want, minlength=h.ntxn)[want] > 1
        assert st["txns_in_cycles"] == int(cyc.sum())
        assert set(st["phase_ms"]) == {"build_cover", "cover_merge", "cut_union", "scc"}
        # a second call over the same members (buffers reused) agrees
        st2 = m.graph_scc(shards, h.ntxn, [sccs[0].data_ptr()] + [None] * (world - 1))
        np.testing.assert_array_equal(sccs[0].cpu().numpy().astype(np.uint32), want)
        assert st2["cut_nodes"] == st["cut_nodes"]
    finally:
        m.close()


def _multi_scc(h, world=1):
    import torch
    from comdb2_amd.hsc import MultiValidator
    dev = torch.device("cuda", 0)
    m = MultiValidator([0] * world)
    try:
        shards = [shard.device_history(shard.history_shard(h, r, world), dev) for r in range(world)]
        scc = torch.zeros(max(h.ntxn, 1), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        m.graph_scc(shards, h.ntxn, [scc.data_ptr()] + [None] * (world - 1))
        return scc[:h.ntxn].cpu().numpy().astype(np.uint32)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["shuffled", "hot_key", "hot_key_shuffled", "hot_mix", "wide_cover",
                                  "back_overflow"])
def test_gpu_multi_graph_scc_build_paths(oracle_mod, case, monkeypatch):
    """The raw build's paths: ops out of txn order (the writer sort then takes
    every pass: the txn bits are not skipped), and hot keys whose writers
    crowd single directory buckets past a bucket line's entries (the overflow
    search of pk): four keys only, or half of 2000 keys' ops moved onto key 0
    (its writers ~1000x denser than the buckets are sized for).  Components =
    Tarjan's.  The cut: by the covered txns' op ranges (txn-sorted ops), by
    every row (shuffled), and every row again after the op-range pass finds
    more covered txns than its list holds (wide_cover: > 65536).  The cover:
    from the listed backward rows, or from interval diffs of every raw row
    once the list overflows (back_overflow: a 16-row list)."""
    from comdb2_amd.workloads import History
    kw = dict(n_txn=20000, n_keys=4, concurrent_frac=0.3, max_lag=16) if case.startswith("hot_key") else \
        dict(seed=9, n_txn=20000, n_keys=2000, concurrent_frac=0.2, max_lag=16)
    if case == "back_overflow":
        monkeypatch.setenv("HSC_GRAPH_BACK_CAP", "16")
    if case == "wide_cover":
        kw = dict(seed=11, n_txn=200000, n_keys=2000, concurrent_frac=0.9, max_lag=64)  # ~185k covered
    h = config4_history(**kw)
    if case == "hot_mix":
        hot = np.random.default_rng(5).random(len(h.key)) < 0.5
        h = History(h.txn, np.where(hot, np.zeros_like(h.key), h.key), h.is_write, h.observed, h.ntxn)
    if case.endswith("shuffled"):
        p = np.random.default_rng(4).permutation(len(h.txn))
        h = History(h.txn[p], h.key[p], h.is_write[p], h.observed[p], h.ntxn)
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    want = oracle_mod.scc(h.ntxn, s, d)
    np.testing.assert_array_equal(_multi_scc(h), want)
    np.testing.assert_array_equal(_multi_scc(h, world=2), want)


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["read_observed", "write_observed", "txn"])
def test_gpu_multi_graph_scc_rejects_ids_out_of_range(field):
    """An op naming a txn >= ntxn fails the call: its txn (the place pass's
    check, before any edge is built) or its observed writer, a read's or a
    write's (the edge pass's check, which emits no row for it)."""
    from comdb2_amd.hsc import HscError
    from comdb2_amd.workloads import History
    h = config4_history(n_txn=3000, n_keys=100)
    obs, txn = h.observed.copy(), h.txn.copy()
    if field == "txn":
        txn[-1] = h.ntxn + 5  # (the last op: the txn order stays)
    else:
        i = int(np.nonzero(h.is_write == (1 if field == "write_observed" else 0))[0][7])
        obs[i] = h.ntxn + 5
    with pytest.raises(HscError, match="out of range"):
        _multi_scc(History(txn, h.key, h.is_write, obs, h.ntxn))
