"""Dependency graph (WR/WW/RW) + SCC.

Parity is unpinned by the reference (it has no cycle checker): the C oracle
(oracle/scc_oracle.c: Adya edges + Tarjan) is cross-checked here against an
independent Python model and hand-built histories with known cycles, and the
GPU path (-m gpu) must reproduce the oracle's edges and components exactly."""
import numpy as np
import pytest
import torch  # imported before any test initialises HIP (tensors for ingest_device)

from comdb2_amd.workloads import History, config4_history, history_from_edn, history_to_edn


def hist(rows, ntxn):
    """rows: (txn, key, 'r'|'w', observed writer or -1)."""
    t, k, w, o = zip(*rows)
    return History(np.array(t, np.uint32), np.array(k, np.uint64),
                   np.array([x == "w" for x in w], np.uint8), np.array(o, np.int64), ntxn)


def py_edges(h):
    writers = {}
    for t, k, w in zip(h.txn, h.key, h.is_write):
        if w:
            writers.setdefault(int(k), set()).add(int(t))
    order = {k: sorted(v) for k, v in writers.items()}
    E = {}
    for k, ws in order.items():
        for a, b in zip(ws, ws[1:]):
            E[(a, b)] = E.get((a, b), 0) | 1
    for t, k, w, o in zip(h.txn, h.key, h.is_write, h.observed):
        if w:
            continue
        t, k, o = int(t), int(k), int(o)
        if o >= 0 and o != t:
            E[(o, t)] = E.get((o, t), 0) | 2
        nxt = [x for x in order.get(k, []) if (x > o if o >= 0 else True)]
        if nxt and nxt[0] != t:
            E[(t, nxt[0])] = E.get((t, nxt[0]), 0) | 4
    return E


def py_scc(n, E):
    """Kosaraju; returns the largest member of each node's component."""
    adj = [[] for _ in range(n)]
    radj = [[] for _ in range(n)]
    for a, b in E:
        adj[a].append(b)
        radj[b].append(a)
    seen, order = [False] * n, []
    for s in range(n):
        if seen[s]:
            continue
        stack = [(s, iter(adj[s]))]
        seen[s] = True
        while stack:
            v, it = stack[-1]
            nxt = next(it, None)
            if nxt is None:
                order.append(v)
                stack.pop()
            elif not seen[nxt]:
                seen[nxt] = True
                stack.append((nxt, iter(adj[nxt])))
    comp = [-1] * n
    for s in reversed(order):
        if comp[s] >= 0:
            continue
        members, st = [], [s]
        comp[s] = s
        while st:
            v = st.pop()
            members.append(v)
            for u in radj[v]:
                if comp[u] < 0:
                    comp[u] = s
                    st.append(u)
        m = max(members)
        for v in members:
            comp[v] = m
    return np.array(comp, dtype=np.uint32)


WRITE_SKEW = hist([(0, 1, "r", -1), (0, 2, "w", -1), (1, 2, "r", -1), (1, 1, "w", -1)], 2)
# serialstep s1's ring restated: T_i reads x_i (stale, initial) and writes x_{i+1}
RING4 = hist([(i, i, "r", -1) for i in range(4)] + [(i, (i + 1) % 4, "w", -1) for i in range(4)], 4)
SERIAL = hist([(0, 1, "w", -1), (1, 1, "r", 0), (1, 1, "w", -1), (2, 1, "r", 1)], 3)


@pytest.mark.parametrize("h,cycles", [(WRITE_SKEW, [[0, 1]]), (RING4, [[0, 1, 2, 3]]),
                                      (SERIAL, [])])
def test_oracle_known_cycles(oracle_mod, h, cycles):
    s, d, t = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    scc = oracle_mod.scc(h.ntxn, s, d)
    got = sorted(sorted(np.nonzero(scc == c)[0].tolist()) for c in set(scc.tolist())
                 if (scc == c).sum() > 1)
    assert got == cycles


@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_python_model(oracle_mod, seed):
    h = config4_history(seed=seed, n_txn=1500, n_keys=60, concurrent_frac=0.2, max_lag=6)
    s, d, t = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    E = py_edges(h)
    assert sorted(E.items()) == sorted(zip(zip(s.tolist(), d.tolist()), t.tolist()))
    np.testing.assert_array_equal(oracle_mod.scc(h.ntxn, s, d), py_scc(h.ntxn, E))


def test_edn_round_trip():
    h = config4_history(n_txn=500, n_keys=40)
    h2 = history_from_edn(history_to_edn(h))
    for k in ("txn", "key", "is_write", "observed"):
        np.testing.assert_array_equal(getattr(h, k), getattr(h2, k))


@pytest.mark.gpu
@pytest.mark.parametrize("h", [WRITE_SKEW, RING4, SERIAL])
def test_gpu_known_cycles(validator, oracle_mod, h):
    scc, st = validator.dep_graph_scc(h)
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    np.testing.assert_array_equal(scc, oracle_mod.scc(h.ntxn, s, d))


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [
    dict(n_txn=20000, n_keys=2000),
    dict(n_txn=200000, n_keys=5000, concurrent_frac=0.05, max_lag=32),
    dict(n_txn=100000, n_keys=300, concurrent_frac=0.3, max_lag=8, zipf=1.2),  # hot keys
    dict(n_txn=1000000, n_keys=100000),
    # the per-GPU share of BASELINE config 4 at 8 GPUs: 100M ops / 8 = 12.6M ops
    dict(n_txn=2_100_000, n_keys=210_000),
])
def test_gpu_graph_matches_oracle(validator, oracle_mod, kw):
    h = config4_history(**kw)
    scc, st = validator.dep_graph_scc(h)
    s, d, t = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    gs, gd, gt = validator.dep_graph_edges()
    np.testing.assert_array_equal(gs, s)
    np.testing.assert_array_equal(gd, d)
    np.testing.assert_array_equal(gt, t)
    np.testing.assert_array_equal(scc, oracle_mod.scc(h.ntxn, s, d))
    assert st["edges"] == len(s)


@pytest.mark.gpu
@pytest.mark.parametrize("keymap", ["clusters", "hashed", "shifted"])
def test_gpu_graph_key_layouts_match_oracle(validator, oracle_mod, keymap):
    """The writers' (key, txn) pairs sort as packed words when their varying
    bits fit 64 (a bucket directory over the packed range then answers each
    read's next-writer search), else as whole rows with a plain binary
    search: keys in two far-apart clusters (packed, a huge empty stretch
    between the directory's buckets), 64-bit hashed keys (rows), keys
    shifted to the top bits of the word (packed)."""
    from comdb2_amd.workloads import History
    h = config4_history(n_txn=60000, n_keys=3000, concurrent_frac=0.1, max_lag=16)
    k = h.key.astype(np.uint64)
    if keymap == "clusters":
        k = np.where(k % 2 == 1, k + np.uint64(1 << 40), k)
    elif keymap == "hashed":
        k = (k * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0xD1B54A32D192ED03)
    else:
        k = k << np.uint64(50)
    h = History(h.txn, k, h.is_write, h.observed, h.ntxn)
    scc, st = validator.dep_graph_scc(h)
    s, d, t = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    gs, gd, gt = validator.dep_graph_edges()
    np.testing.assert_array_equal(gs, s)
    np.testing.assert_array_equal(gd, d)
    np.testing.assert_array_equal(gt, t)
    np.testing.assert_array_equal(scc, oracle_mod.scc(h.ntxn, s, d))


def _cover_frac(h, s, d):
    back = s > d
    diff = np.zeros(h.ntxn + 1, np.int64)
    np.add.at(diff, d[back].astype(np.int64), 1)
    np.add.at(diff, s[back].astype(np.int64) + 1, -1)
    return float((np.cumsum(diff)[:h.ntxn] > 0).mean())


# high concurrency: half the txns read a snapshot up to max_lag commits old
STRESS = [dict(n_txn=200000, n_keys=20000, concurrent_frac=0.5, max_lag=512),
          dict(n_txn=100000, n_keys=1000, concurrent_frac=0.5, max_lag=256)]  # giant SCCs


@pytest.mark.parametrize("kw", STRESS[:1])
def test_stress_history_covers_most_txns(oracle_mod, kw):
    h = config4_history(**kw)
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    assert _cover_frac(h, s, d) >= 0.10


@pytest.mark.gpu
@pytest.mark.parametrize("kw", STRESS)
def test_gpu_stress_graph_matches_tarjan(validator, oracle_mod, kw):
    h = config4_history(**kw)
    scc, st = validator.dep_graph_scc(h)
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    assert _cover_frac(h, s, d) >= 0.10
    np.testing.assert_array_equal(scc, oracle_mod.scc(h.ntxn, s, d))
    assert st["nontrivial_sccs"] > 0
    print(f"stress {kw}: rounds {st['rounds']} iterations {st['iterations']} "
          f"build {st['build_ms']:.2f} ms scc {st['scc_ms']:.2f} ms")


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(n_txn=3000, n_keys=200, concurrent_frac=0.3, max_lag=16),
                                dict(n_txn=60000, n_keys=4000, concurrent_frac=0.5, max_lag=128)])
def test_gpu_rw_pairs_feed_the_graph(oracle_mod, kw):
    """the validator's (read set, writer) pairs -- every writer
    a read did not see -- become the graph's rw edges; with the history's ww
    and wr edges the components equal Tarjan's over the history graph."""
    from comdb2_amd.hsc import Validator
    from comdb2_amd.workloads import history_window, int64_words
    h = config4_history(**kw)
    hw = history_window(h)
    v = Validator(0)
    try:
        v.register_group("t1", 0, 9)
        dev = torch.device("cuda", 0)
        gid = torch.zeros(len(hw.keys), dtype=torch.int32, device=dev)
        words = torch.from_numpy(int64_words(hw.keys).reshape(-1).view(np.int64)).to(dev)
        lsn = torch.from_numpy(hw.lsn.view(np.int64)).to(dev)
        v.ingest_device(len(hw.keys), 2, gid.data_ptr(), words.data_ptr(), lsn.data_ptr(),
                        hw.end_lsn)
        torch.cuda.synchronize()
        txn, wl = v.rw_edges(hw.readsets)
        assert len(txn) > 0
        v.dep_graph_stage_rw_pairs(np.arange(h.ntxn), hw.commit_lsn, np.arange(h.ntxn))
        v.dep_graph_build(h, full=True, no_rw=True)
        scc, st = v.dep_graph_scc_built(h.ntxn)
        s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
        np.testing.assert_array_equal(scc, oracle_mod.scc(h.ntxn, s, d))
        assert st["nontrivial_sccs"] > 0 and st["rw"] > 0
    finally:
        v.close()
