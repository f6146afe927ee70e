"""The OSQL_SERIAL wire decoder (hsc_wire.cpp).

Layout restated from db/osqlcomm.c:748-766,809-826,909-993 and the buf_put
byte-swap of every 2/4/8-byte item (bbinc/endian_core.amd64.h:17-44).  The
reference's encoder lives in a TU that needs protoc-c output, so there are no
reference byte vectors: the hand-assembled message below, decode(encode(rs))
and the oracle's verdicts on the decoded read sets pin it."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import Range, ReadSets
from comdb2_amd.hsc import HscError, Validator
from comdb2_amd.workloads import random_case
from test_marshal import model_marshal, native_by_txn


@pytest.fixture()
def host():
    v = Validator(-1)
    yield v
    v.close()


def receiver_view(rs):
    """What serial_readset_get rebuilds (db/osqlcomm.c:948-993): locked ranges
    come back with lflag = rflag = 1, no keys, idxnum = currange_new's -2."""
    out = []
    for t in range(rs.ntxn):
        rows = []
        for r in range(int(rs.txn_off[t]), int(rs.txn_off[t + 1])):
            tb = rs.tbnames[int(rs.table[r])]
            if int(rs.islocked[r]):
                rows.append((tb, 1, -2, 1, 1, b"", b""))
                continue
            k = lambda o, n: bytes(rs.keys[int(o):int(o) + int(n)])
            rows.append((tb, 0, int(rs.idxnum[r]), int(rs.lflag[r]), int(rs.rflag[r]),
                         b"" if rs.lflag[r] else k(rs.lkey_off[r], rs.lkeylen[r]),
                         b"" if rs.rflag[r] else k(rs.rkey_off[r], rs.rkeylen[r])))
        out.append((int(rs.snap[t]), rows))
    return out


@pytest.mark.parametrize("seed", range(10))
def test_wire_round_trip(host, seed):
    _, rs = random_case(1000 + seed, max_ranges=12)
    d = host.decode_serial(F.encode_serial(rs))
    assert receiver_view(d) == receiver_view(rs)


def test_wire_bytes_of_one_message(host):
    """A hand-assembled payload: ints and the 8-byte key are byte-reversed on
    the wire, the 3-byte name "t1\\0" and the 9-byte key are not."""
    k9 = F.enc_int64(7)
    k8 = b"ABCDEFGH"
    rs = ReadSets.from_lists([[Range("t1", 0, k9, k8)]], [F.lsn(2, 0x100)])
    buf, off, ln = F.encode_serial(rs)
    be = lambda v: int(v).to_bytes(4, "big")
    body = (be(3) + b"t1\x00" + be(0) + be(0) + be(0) + be(9) + k9 + be(0) + be(8) + k8[::-1])
    want = be(len(body)) + be(1) + be(2) + be(0x100) + body
    assert bytes(buf[: int(ln[0])]) == want
    d = host.decode_serial((buf, off, ln))
    assert bytes(d.keys[int(d.rkey_off[0]):int(d.rkey_off[0]) + 8]) == k8
    assert int(d.snap[0]) == F.lsn(2, 0x100)


@pytest.mark.parametrize("seed", range(6))
def test_wire_marshal_matches_model(seed):
    log, rs = random_case(1100 + seed, broken=(seed % 2 == 0), max_ranges=10)
    v = Validator(-1)
    try:
        v.ingest_log(log)
        d = v.decode_serial(F.encode_serial(rs))
        W, want = model_marshal(log, d, v)
        assert native_by_txn(v.marshal(d)) == want
    finally:
        v.close()


def test_truncated_message_fails_closed(host):
    log, rs = random_case(3)
    host.ingest_log(log)
    buf, off, ln = F.encode_serial(rs)
    ln = ln.copy()
    ln[1] -= 5
    with pytest.raises(HscError):
        host.decode_serial((buf, off, ln))


def test_wire_oracle_on_decoded(host, oracle_mod):
    """Oracle verdicts of the receiver's view equal those of the sender's
    read sets when no range is locked with a non-default index (the only
    difference the wire introduces)."""
    log, rs = random_case(1200, max_ranges=8)
    d = host.decode_serial(F.encode_serial(rs))
    a, _, _ = oracle_mod.check(log, rs)
    b, _, _ = oracle_mod.check(log, d)
    differs = [t for t in range(rs.ntxn) if (a[t] != 0) != (b[t] != 0)]
    for t in differs:  # only via the locked-range idxnum rewrite
        rows = range(int(rs.txn_off[t]), int(rs.txn_off[t + 1]))
        assert any(int(rs.islocked[r]) and int(rs.idxnum[r]) != -2 for r in rows)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_check_serial_matches_oracle(validator, oracle_mod, seed):
    log, rs = random_case(1300 + seed, broken=(seed % 3 == 1))
    validator.ingest_log(log)
    msgs = F.encode_serial(rs)
    got = validator.check_serial(msgs)
    want, _, _ = oracle_mod.check(log, validator.decode_serial(msgs))
    np.testing.assert_array_equal(got != 0, want != 0)
