"""CPU: the CPU sort-join baseline (oracle/sortjoin.c) against the oracle on
marshalled batches -- it is bench.py's second CPU line, so its verdicts must
equal the reference semantics before its rate means anything."""
import numpy as np
import pytest

from comdb2_amd.hsc import Validator
from comdb2_amd.workloads import config2, config2_device_window, config3, random_case
from probe_model import WindowModel


def window_rows(v, log):
    """(gid, words [W][n], lsn, ngroups, table_max[ntables]) of the committed
    writes of `log`, grouped the way the native dictionaries number them."""
    model = WindowModel(log)
    W = v.words
    groups = []
    gid = 0
    while True:
        try:
            groups.append(v.group_info(gid))
        except Exception:
            break
        gid += 1
    g_of = {(v.table_name(t), ix, kl): g for g, (t, ix, kl) in enumerate(groups)}
    gids, words, lsns = [], [], []
    for (tb, ix, kl), (keys, ls) in model.groups.items():
        g = g_of[(tb, ix, kl)]
        for k, l in zip(keys, ls):
            kb = k + bytes(8 * W - len(k))
            gids.append(g)
            words.append([int.from_bytes(kb[8 * j:8 * j + 8], "big") for j in range(W)])
            lsns.append(l)
    ntab = max([t for t, _, _ in groups] + [-1]) + 1
    tmax = np.zeros(max(ntab, 1), np.uint64)
    for t in range(ntab):
        tmax[t] = model.table_max.get(v.table_name(t), 0)
    w = np.array(words, np.uint64).reshape(-1, W).T.copy() if words else np.zeros((W, 0), np.uint64)
    return (np.array(gids, np.uint32), w, np.array(lsns, np.uint64), len(groups), tmax)


@pytest.fixture()
def host():
    v = Validator(-1)
    yield v
    v.close()


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("threads", [1, 4])
def test_sortjoin_matches_oracle_random(host, oracle_mod, seed, threads):
    log, rs = random_case(300 + seed, broken=(seed % 3 == 2))
    host.ingest_log(log)
    m = host.marshal(rs)
    gid, words, lsn, ng, tmax = window_rows(host, log)
    sj = oracle_mod.SortJoin(gid, words, lsn, ng)
    got, _ = sj.probe(m, tmax, nthreads=threads)
    want, _, _ = oracle_mod.check(log, rs)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_sortjoin_config2_small(host, oracle_mod):
    c2 = config2(n_commits=3000, n_txn=600, value_bits=20, width=1 << 10, snap_recent=0.5)
    host.ingest_log(c2.log)
    m = host.marshal(c2.readsets)
    gid, words, lsn = config2_device_window(c2)
    # raw log-order rows (duplicates included): the baseline sorts and dedupes
    sj = oracle_mod.SortJoin(gid, words, lsn, 1)
    assert sj.rows == len(np.unique(words[0] * np.uint64(1 << 8) + (words[1] >> np.uint64(56))))
    got, _ = sj.probe(m, np.array([c2.log.end_lsn], np.uint64), nthreads=4)
    want, _, _ = oracle_mod.check(c2.log, c2.readsets, nthreads=4)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_sortjoin_composite_keys(host, oracle_mod):
    log, rs = config3(n_writes=6000, n_txn=300)
    host.ingest_log(log)
    m = host.marshal(rs)
    gid, words, lsn, ng, tmax = window_rows(host, log)
    sj = oracle_mod.SortJoin(gid, words, lsn, ng)
    got, _ = sj.probe(m, tmax, nthreads=4)
    want, _, _ = oracle_mod.check(log, rs, nthreads=4)
    np.testing.assert_array_equal(got != 0, want != 0)
