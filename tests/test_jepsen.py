"""CPU: Jepsen-format histories -> dependency-graph histories
(comdb2_amd/jepsen.py): the register client's EDN
(linearizable/ctest/register.c:282-370) and Adya's G2 inserts
(linearizable/jepsen/src/jepsen/adya.clj:13-83).  Parity of the graph is
unpinned by the reference (it has no cycle checker); the known answers here
are the G2 checker's illegal keys (adya.clj:57-83) and injected lost
updates, checked with the oracle's edges + Tarjan (oracle/scc_oracle.c)."""
import numpy as np
import pytest

from comdb2_amd import jepsen as J


def components(oracle_mod, h):
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    scc = oracle_mod.scc(h.ntxn, s, d)
    sizes = np.bincount(scc, minlength=h.ntxn)
    return scc, {int(c) for c in np.nonzero(sizes > 1)[0]}


def test_edn_subset():
    forms = J.parse_edn('{:type :ok :f :cas :process 3 :value [1 4] :uid 77 :time 12}\n'
                        '{:type :ok, :f :read, :value nil, :uid nil, :flag true, :s "x y"}')
    assert forms[0] == {":type": ":ok", ":f": ":cas", ":process": 3, ":value": [1, 4],
                        ":uid": 77, ":time": 12}
    assert forms[1][":value"] is None and forms[1][":flag"] is True and forms[1][":s"] == "x y"
    with pytest.raises(ValueError):
        J.parse_edn("{:type :ok")


def test_register_lines_as_register_c_prints_them():
    """The exact line formats of register.c:282-370: invoke / ok / fail of
    read, write and cas; pairing by :process, fails dropped, commit order by
    completion time, WR by (uid, value), the cas read by its value."""
    text = "\n".join([
        "{:type :invoke :f :write :value 3 :process 0 :uid 11 :time 1}",
        "{:type :invoke :f :read :value nil :process 1 :time 2}",
        "{:type :ok :f :write :process 0 :value 3 :uid 11 :time 5}",
        "{:type :ok :f :read :process 1 :value nil :uid nil :time 4}",
        "{:type :invoke :f :cas :value [3 4] :process 0 :uid 12 :time 6}",
        "{:type :ok :f :cas :process 0 :value [3 4] :uid 12 :time 8}",
        "{:type :invoke :f :write :value 1 :process 2 :uid 13 :time 6}",
        "{:type :fail :f :write :process 2 :value 1 :uid 13 :time 9}",
        "{:type :invoke :f :read :value nil :process 1 :time 9}",
        "{:type :ok :f :read :process 1 :value 3 :uid 11 :time 10}",
        "{:type :invoke :f :cas :value [0 2] :process 2 :uid 14 :time 11}",
    ])
    ops = J.history_from_jepsen_edn(text)
    assert (ops.ok, ops.failed, ops.info, ops.unpaired, ops.dangling) == (4, 1, 0, 1, 0)
    h = ops.history
    # txns: 0 read(nil) @4, 1 write 3 @5, 2 cas [3 4] @8, 3 read (3, uid 11) @10
    rows = list(zip(h.txn.tolist(), h.is_write.tolist(), h.observed.tolist()))
    assert rows == [(0, 0, -1), (1, 1, -1), (2, 0, 1), (2, 1, -1), (3, 0, 1)]


def test_dangling_reads_are_dropped():
    text = ("{:type :invoke :f :read :value nil :process 1 :time 1}\n"
            "{:type :ok :f :read :process 1 :value 2 :uid 99 :time 2}\n")
    ops = J.history_from_jepsen_edn(text)
    assert ops.dangling == 1 and ops.history.nops == 0 and ops.ok == 1


@pytest.mark.parametrize("seed", range(4))
def test_adya_g2_cycles_are_the_g2_checkers_illegal_keys(oracle_mod, seed):
    text, bad = J.adya_g2_edn(seed, n_keys=400, anomaly=0.05)
    ops = J.history_from_jepsen_edn(text)
    assert sorted(J.g2_illegal(ops)) == bad
    scc, comps = components(oracle_mod, ops.history)
    keys = set()
    for c in comps:
        members = np.nonzero(scc == c)[0]
        assert len(members) == 2
        ks = {ops.txn_ops[int(t)][":value"][0] for t in members}
        assert len(ks) == 1
        keys |= ks
    assert sorted(keys) == bad


@pytest.mark.parametrize("seed", range(4))
def test_register_lost_updates_are_cycles(oracle_mod, seed):
    text, lost = J.register_history_edn(seed, n_ops=3000, lost_update=0.05, stale_read=0.05)
    ops = J.history_from_jepsen_edn(text)
    assert ops.unpaired == 0 and ops.failed > 0
    scc, comps = components(oracle_mod, ops.history)
    assert lost > 0 and len(comps) > 0
    clean, _ = J.register_history_edn(seed, n_ops=3000, lost_update=0.0, stale_read=0.0)
    _, none = components(oracle_mod, J.history_from_jepsen_edn(clean).history)
    assert not none  # a serial execution without anomalies has no cycle


GOLDEN_FILETEST = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                              "jepsen_filetest_history.txt")


def test_reference_filetest_history(oracle_mod):
    """The reference's own knossos fixture (linearizable/filetest/history.txt,
    copied as data to tests/golden/): one EDN vector of a cas-register history
    without :uid -- a write of 1, then a read returning 1.  The read observed
    the write by its value: a 2-txn graph with one wr edge and no cycle, as
    filetest.clj's knossos check finds it valid."""
    ops = J.history_from_jepsen_edn(open(GOLDEN_FILETEST).read())
    assert (ops.ok, ops.failed, ops.info, ops.unpaired, ops.dangling) == (2, 0, 0, 0, 0)
    h = ops.history
    assert h.ntxn == 2
    rows = list(zip(h.txn.tolist(), h.is_write.tolist(), h.observed.tolist()))
    assert rows == [(0, 1, -1), (1, 0, 0)]
    s, d, t = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    assert list(zip(s.tolist(), d.tolist())) == [(0, 1)]
    scc, comps = components(oracle_mod, h)
    assert not comps and scc.tolist() == [0, 1]


def test_info_writes_observed_by_a_read_committed():
    """:info ops are indeterminate: a write a later read observed did commit
    (it joins at its invoke), an unobserved one is dropped -- otherwise the
    read would dangle and its edges (here the rw edge of a lost update) would
    vanish."""
    text = "\n".join([
        "{:type :invoke :f :write :value 1 :process 0 :uid 5 :time 1}",
        "{:type :info :f :write :process 0 :value 1 :uid 5 :time 3}",
        "{:type :invoke :f :write :value 2 :process 1 :uid 6 :time 4}",
        "{:type :info :f :write :process 1 :value 2 :uid 6 :time 5}",
        "{:type :invoke :f :read :value nil :process 2 :time 6}",
        "{:type :ok :f :read :process 2 :value 1 :uid 5 :time 7}",
    ])
    ops = J.history_from_jepsen_edn(text)
    assert (ops.ok, ops.info, ops.info_recovered, ops.dangling) == (1, 2, 1, 0)
    h = ops.history
    assert h.ntxn == 2
    rows = list(zip(h.txn.tolist(), h.is_write.tolist(), h.observed.tolist()))
    assert rows == [(0, 1, -1), (1, 0, 0)]
