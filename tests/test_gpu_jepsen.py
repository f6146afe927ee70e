"""GPU: dependency graphs + SCC (hsc_dep_graph_scc) of Jepsen-format
histories parsed by comdb2_amd/jepsen.py -- the register client's EDN
(linearizable/ctest/register.c:282-370, with injected lost updates and stale
reads, several independent registers) and Adya G2 insert histories
(linearizable/jepsen/src/jepsen/adya.clj:13-55) -- equal the oracle's edges +
Tarjan (oracle/scc_oracle.c); the G2 components are exactly the G2 checker's
illegal keys (adya.clj:57-83)."""
import numpy as np
import pytest

from comdb2_amd import jepsen as J

pytestmark = pytest.mark.gpu


def _tarjan(oracle_mod, h):
    s, d, _ = oracle_mod.dep_edges(h.txn, h.key, h.is_write, h.observed)
    return oracle_mod.scc(h.ntxn, s, d)


@pytest.mark.parametrize("n_keys", [1, 64])
def test_register_history_scc_equals_tarjan(validator, oracle_mod, n_keys):
    text, lost = J.register_history_edn(11 + n_keys, n_ops=60_000, n_procs=16, n_keys=n_keys,
                                        lost_update=0.03, stale_read=0.05)
    ops = J.history_from_jepsen_edn(text)
    h = ops.history
    scc, st = validator.dep_graph_scc(h)
    want = _tarjan(oracle_mod, h)
    np.testing.assert_array_equal(scc, want)
    assert lost > 0 and st["nontrivial_sccs"] > 0


def test_adya_g2_history_scc_equals_tarjan_and_the_g2_checker(validator, oracle_mod):
    text, bad = J.adya_g2_edn(5, n_keys=20_000, anomaly=0.02)
    ops = J.history_from_jepsen_edn(text)
    h = ops.history
    scc, st = validator.dep_graph_scc(h)
    np.testing.assert_array_equal(scc, _tarjan(oracle_mod, h))
    sizes = np.bincount(scc, minlength=h.ntxn)
    keys = sorted({ops.txn_ops[int(t)][":value"][0] for t in np.nonzero(sizes[scc] > 1)[0]})
    assert keys == bad == sorted(J.g2_illegal(ops))
    assert st["nontrivial_sccs"] == len(bad)


def test_reference_filetest_history_on_the_gpu(validator, oracle_mod):
    """linearizable/filetest/history.txt (the reference's knossos fixture, as
    data in tests/golden/): the GPU graph has the one wr edge and no cycle."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "jepsen_filetest_history.txt")
    h = J.history_from_jepsen_edn(open(path).read()).history
    scc, st = validator.dep_graph_scc(h)
    assert scc.tolist() == [0, 1] and st["nontrivial_sccs"] == 0
    s, d, t = validator.dep_graph_edges()
    assert (s.tolist(), d.tolist(), t.tolist()) == ([0], [1], [2])  # type 2 = wr
    np.testing.assert_array_equal(scc, _tarjan(oracle_mod, h))
