"""CPU: the native host logic (log decode, dictionaries, marshaller) through a
host-only context, checked against an independent Python restatement of the
marshalling rules and -- combined with the probe-level join model -- against
the oracle.  No GPU is used."""
import numpy as np
import pytest

from comdb2_amd.formats import LogBuilder, Range, ReadSets
from comdb2_amd.hsc import Validator
from comdb2_amd.workloads import config2, random_case
from probe_model import WindowModel, committed_writes, evaluate


@pytest.fixture()
def host():
    v = Validator(-1)
    yield v
    v.close()


def model_marshal(log, rs, v):
    """Python restatement of the marshaller: per read set the forced verdict,
    the lock probes and the range probes (as sorted lists)."""
    commits, dangling = committed_writes(log)
    end = int(log.end_lsn)
    recs = set(int(x) for x in log.lsn)
    poison = max([d for d in dangling] + [c for c, _, b in commits if b] + [0])
    groups = {}  # (tbname, ix) -> [(gid, klen)]
    gid = 0
    while True:
        try:
            tid, ix, kl = v.group_info(gid)
        except Exception:
            break
        groups.setdefault((v.table_name(tid), ix), []).append((gid, kl))
        gid += 1
    W = max([1] + [(kl + 7) // 8 for lst in groups.values() for _, kl in lst])
    out = []
    for t in range(rs.ntxn):
        S = int(rs.snap[t])
        if S >= end:
            out.append((0, [], []))
            continue
        if S not in recs or poison > S:
            out.append((1, [], []))
            continue
        rows = list(range(int(rs.txn_off[t]), int(rs.txn_off[t + 1])))
        first, span = {}, {}
        for k, r in enumerate(rows):
            tb = rs.tbnames[rs.table[r]]
            if v.table_id(tb) < 0:
                continue
            first.setdefault(tb, int(rs.islocked[r]))
            b, _ = span.get((tb, int(rs.idxnum[r])), (k, k))
            span[(tb, int(rs.idxnum[r]))] = (b, k)
        locks, probes = [], []
        for tb, lk in first.items():
            if lk:
                locks.append((v.table_id(tb), S))
        for (tb, ix), (b, e) in span.items():
            if first[tb]:
                continue
            for g, kl in groups.get((tb, ix), []):
                for r in rows[b:e + 1]:
                    lkey = bytes(rs.keys[int(rs.lkey_off[r]):int(rs.lkey_off[r]) + int(rs.lkeylen[r])])
                    rkey = bytes(rs.keys[int(rs.rkey_off[r]):int(rs.rkey_off[r]) + int(rs.rkeylen[r])])
                    lo = b"\x00" * kl if rs.lflag[r] else (lkey[:kl] + b"\x00" * kl)[:kl]
                    hi = b"\xff" * kl if rs.rflag[r] else (rkey[:kl] + b"\xff" * kl)[:kl]
                    if lo > hi:
                        continue
                    pad = lambda x: tuple(int.from_bytes((x + bytes(8 * W))[8 * j:8 * j + 8], "big")
                                          for j in range(W))
                    probes.append((g, pad(lo), pad(hi), S))
        out.append((0, sorted(locks), sorted(probes)))
    return W, out


def native_by_txn(m):
    W, n = m["words"], m["n"]
    probes = [[] for _ in range(m["n_txn"])]
    locks = [[] for _ in range(m["n_txn"])]
    for i in range(n):
        probes[int(m["txn"][i])].append((int(m["gid"][i]), tuple(int(x) for x in m["lo"][:, i]),
                                         tuple(int(x) for x in m["hi"][:, i]), int(m["snap"][i])))
    for i in range(m["n_lock"]):
        locks[int(m["lock_txn"][i])].append((int(m["lock_table"][i]), int(m["lock_snap"][i])))
    return [(int(m["forced"][t]), sorted(locks[t]), sorted(probes[t])) for t in range(m["n_txn"])]


@pytest.mark.parametrize("seed", range(10))
def test_native_marshal_matches_model(host, seed):
    log, rs = random_case(seed, broken=(seed % 3 == 0), max_ranges=10)
    host.ingest_log(log)
    m = host.marshal(rs)
    W, want = model_marshal(log, rs, host)
    assert m["words"] == W
    got = native_by_txn(m)
    for t in range(rs.ntxn):
        assert got[t] == want[t], t


@pytest.mark.parametrize("seed", range(10))
def test_marshal_plus_join_model_matches_oracle(host, oracle_mod, seed):
    log, rs = random_case(50 + seed, broken=(seed % 2 == 1))
    host.ingest_log(log)
    m = host.marshal(rs)
    verdict = evaluate(host, m, WindowModel(log))
    want, _, _ = oracle_mod.check(log, rs)
    np.testing.assert_array_equal((verdict | m["forced"]) != 0, want != 0)


def test_config2_small_marshal_plus_join_model(host, oracle_mod):
    c2 = config2(n_commits=2000, n_txn=400, value_bits=20, width=1 << 10, snap_recent=0.5)
    host.ingest_log(c2.log)
    m = host.marshal(c2.readsets)
    assert m["n"] == c2.readsets.nranges       # one group, no empty ranges dropped
    verdict = evaluate(host, m, WindowModel(c2.log))
    want, _, _ = oracle_mod.check(c2.log, c2.readsets)
    np.testing.assert_array_equal((verdict | m["forced"]) != 0, want != 0)


def test_host_only_context_refuses_device_work(host):
    log, rs = random_case(3)
    host.ingest_log(log)
    from comdb2_amd.hsc import HscError
    with pytest.raises(HscError):
        host.check_readsets(rs)


def test_config3_and_config5_host_path(host, oracle_mod):
    from comdb2_amd.workloads import config3, config5
    log, rs = config3(n_writes=20000, n_txn=800)
    host.ingest_log(log)
    m = host.marshal(rs)
    assert m["words"] == 8 and m["n_lock"] > 0
    want, _, _ = oracle_mod.check(log, rs, nthreads=8)
    got = evaluate(host, m, WindowModel(log)) | m["forced"]
    np.testing.assert_array_equal(got != 0, want != 0)
    c5 = config5(n_commits=20000, n_txn=1000, snap_recent=0.002)
    host.ingest_log(c5.log)
    m = host.marshal(c5.readsets)
    want, _, _ = oracle_mod.check(c5.log, c5.readsets, nthreads=8)
    got = evaluate(host, m, WindowModel(c5.log)) | m["forced"]
    np.testing.assert_array_equal(got != 0, want != 0)
