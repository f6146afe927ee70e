"""Config 3 (composite keys over 32 (table, index) groups) through a window
built from arrays (hsc_window_ingest_device, the multi-GPU bench's path: each
rank ingests only its groups) against the log-based oracle
(oracle/serial_oracle.c over the same workload as a log)."""
import numpy as np
import pytest

from comdb2_amd import shard
from comdb2_amd.hsc import Validator
from comdb2_amd.workloads import config3, config3_arrays

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def device_validator(a, groups=None):
    v = Validator(0)
    for g, (tb, ix, L) in enumerate(a.groups):
        assert v.register_group(tb, ix, L) == g
    gid, words, lsn = a.window(groups)
    dev = torch.device("cuda", 0)
    tg = torch.from_numpy(gid).to(dev)
    tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
    tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
    v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                    a.end_lsn)
    torch.cuda.synchronize()
    v.merge_table_max(a.table_max)  # data-row writes lock tables too
    return v


@pytest.mark.parametrize("kw", [dict(n_writes=30000, n_txn=1500),
                                dict(seed=11, n_writes=60000, n_txn=2000, keys_per_commit=5)])
def test_config3_device_window_matches_oracle(oracle_mod, kw):
    log, rs = config3(**kw)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    a = config3_arrays(**kw)
    v = device_validator(a)
    try:
        got = v.check_readsets(rs) != 0
    finally:
        v.close()
    np.testing.assert_array_equal(got, want)
    assert 0 < want.sum() < len(want)


def test_config3_group_shards_merge_to_oracle(oracle_mod):
    """Two group shards (LPT over group sizes), each rank's window holding only
    its groups and probing only its groups' ranges (rank 0 also the table
    locks): the OR of the two verdicts equals the unsharded oracle."""
    kw = dict(seed=3, n_writes=40000, n_txn=1500)
    log, rs = config3(**kw)
    want = oracle_mod.check(log, rs, nthreads=8)[0] != 0
    a = config3_arrays(**kw)
    sizes = {g: int((a.w_group == g).sum()) for g in range(len(a.groups))}
    sh = shard.GroupShards(sizes, 2)
    merged = np.zeros(rs.ntxn, dtype=bool)
    for r in range(2):
        mine = [g for g, o in sh.owner.items() if o == r]
        v = device_validator(a, mine)
        try:
            m = v.marshal(rs)
            sub = shard.route(m, sh.range_mask(m, r), sh.lock_mask(m, r))
            merged |= probe_sub(v, sub)
        finally:
            v.close()
    np.testing.assert_array_equal(merged, want)


def probe_sub(v, m):
    from comdb2_amd import hsc
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    T = m["n_txn"]
    b = dict(lo=t(m["lo"]), hi=t(m["hi"]), gid=t(m["gid"]), snap=t(m["snap"]), txn=t(m["txn"]),
             lt=t(m["lock_table"]), ls=t(m["lock_snap"]), lx=t(m["lock_txn"]))
    verdict = torch.zeros(T, dtype=torch.uint8, device=dev)
    bitmap = torch.zeros((T + 63) // 64, dtype=torch.int64, device=dev)
    pb = hsc.ProbeBatch(m["n"], b["lo"].data_ptr(), b["hi"].data_ptr(), b["gid"].data_ptr(),
                        b["snap"].data_ptr(), b["txn"].data_ptr(), m["n_lock"], b["lt"].data_ptr(),
                        b["ls"].data_ptr(), b["lx"].data_ptr(), T, verdict.data_ptr(),
                        bitmap.data_ptr())
    v.probe_device(pb)
    v.synchronize()
    # the bitmap comes from the plan + join (no pack pass): equal to the bytes
    bits = np.unpackbits(bitmap.cpu().numpy().view(np.uint8), bitorder="little")[:T]
    np.testing.assert_array_equal(bits.astype(bool), verdict.cpu().numpy() != 0)
    return np.maximum(verdict.cpu().numpy(), m["forced"]) != 0
