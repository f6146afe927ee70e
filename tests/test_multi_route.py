"""CPU: the routing rule of the multi-GPU context (hsc_route.hip,
hsc_multi.cpp) restated in numpy over a host-only context's marshalled
probes.  The window is cut at composite (gid, key words) splitters; a probe
goes to every member d in [owner(gid || lo), owner(gid || hi)] with owner(K) =
#splitters <= K; table locks go to member 0.  Each member's probes are
evaluated against its piece only (tests/probe_model.py) and the OR over the
members must equal the unpartitioned evaluation and the oracle -- including
splitters inside a group's key run, where ranges straddle two pieces."""
import numpy as np
import pytest

from comdb2_amd.hsc import MultiValidator, Validator
from comdb2_amd.workloads import random_case
from probe_model import WindowModel, evaluate


def composite_le(sp_gid, sp_w, g, x):
    """[S] bool: splitter k <= (g, x) in (gid, words) order."""
    S = len(sp_gid)
    out = np.zeros(S, bool)
    for k in range(S):
        a = (int(sp_gid[k]),) + tuple(int(w) for w in sp_w[:, k])
        b = (int(g),) + tuple(int(w) for w in x)
        out[k] = a <= b
    return out


def owner(sp_gid, sp_w, g, x):
    return int(composite_le(sp_gid, sp_w, g, x).sum())


def key_words(key, W):
    b = bytes(key) + bytes(8 * W - len(key))
    return [int.from_bytes(b[8 * j:8 * j + 8], "big") for j in range(W)]


def route(m, sp_gid, sp_w, world):
    dest = [[] for _ in range(world)]
    for i in range(m["n"]):
        g = int(m["gid"][i])
        ra = owner(sp_gid, sp_w, g, m["lo"][:, i])
        rb = owner(sp_gid, sp_w, g, m["hi"][:, i])
        assert ra <= rb
        for d in range(ra, rb + 1):
            dest[d].append(i)
    return dest


def sub_batch(m, idx, with_locks):
    idx = np.asarray(idx, np.int64)
    out = dict(m)
    out.update(n=len(idx), lo=m["lo"][:, idx], hi=m["hi"][:, idx], gid=m["gid"][idx],
               snap=m["snap"][idx], txn=m["txn"][idx])
    if not with_locks:
        out.update(n_lock=0, lock_table=m["lock_table"][:0], lock_snap=m["lock_snap"][:0],
                   lock_txn=m["lock_txn"][:0])
    return out


@pytest.mark.parametrize("seed,world", [(0, 2), (1, 3), (2, 4), (3, 8), (4, 2), (5, 5)])
def test_routed_pieces_or_to_the_whole(oracle_mod, seed, world):
    log, rs = random_case(1200 + seed, n_commits=160, n_txn=50, value_range=24)
    want, _, _ = oracle_mod.check(log, rs)
    v = Validator(-1)
    try:
        v.ingest_log(log)
        m = v.marshal(rs)
        W = m["words"]
        whole = WindowModel(log)
        # every distinct window key as (gid, words); splitters drawn among them
        # (so pieces cut inside key runs) plus a few between groups
        gid_of = {}
        keys = []
        for (tb, ix, kl), (ks, _) in whole.groups.items():
            g = None
            for gg in range(256):
                try:
                    t, i2, l2 = v.group_info(gg)
                except Exception:
                    break
                if v.table_name(t) == tb and i2 == ix and l2 == kl:
                    g = gg
                    break
            assert g is not None
            gid_of[(tb, ix, kl)] = g
            keys += [(g, tuple(key_words(k, W))) for k in ks]
        keys.sort()
        rng = np.random.default_rng(seed)
        pick = sorted(rng.choice(len(keys), size=world - 1, replace=False).tolist())
        sp_gid = np.array([keys[p][0] for p in pick], np.uint32)
        sp_w = np.array([keys[p][1] for p in pick], np.uint64).T.reshape(W, world - 1)
        dest = route(m, sp_gid, sp_w, world)
        assert sum(len(d) for d in dest) >= m["n"]
        verdict = np.zeros(m["n_txn"], np.uint8)
        for d in range(world):
            def in_piece(tb, ix, key, d=d):
                g = gid_of[(tb, ix, len(key))]
                return owner(sp_gid, sp_w, g, key_words(key, W)) == d
            piece = WindowModel(log, key_filter=in_piece)
            part = sub_batch(m, dest[d], with_locks=(d == 0))
            verdict |= evaluate(v, part, piece, table_max_by_name=whole.table_max)
        verdict = np.maximum(verdict, m["forced"])
        np.testing.assert_array_equal(verdict != 0, want != 0)
        np.testing.assert_array_equal(verdict, np.maximum(evaluate(v, m, whole), m["forced"]))
    finally:
        v.close()


def test_multi_context_needs_a_device():
    from comdb2_amd import hsc
    if hsc.load().hsc_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(hsc.HscError):
        MultiValidator([0, 0])
