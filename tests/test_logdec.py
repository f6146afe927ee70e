"""CPU: the raw log-record decoder (hsc_logdec.cpp, SURVEY.md §8(f) row 1 /
§8(a) A7-A8) through a host-only context.

The byte layouts are restated from bdb/llog.src:26-225 and
berkdb/dist/gen_rec_endian.awk:550-630 (formats.encode_raw); the reference's
generated llog_auto.c encoders are not buildable here (awk-generated code),
so there are no reference byte vectors: decode(encode(log)) must reproduce the
log, and the decoded stream must give the oracle's verdicts.  Parity of the
byte layout itself is unpinned beyond that restatement."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.hsc import HscError, Validator
from comdb2_amd.workloads import config1_events, random_case, replay
from test_marshal import model_marshal, native_by_txn


@pytest.fixture()
def host():
    v = Validator(-1)
    yield v
    v.close()


def same_log(a, b):
    np.testing.assert_array_equal(a.lsn, b.lsn)
    np.testing.assert_array_equal(a.rectype, b.rectype)
    np.testing.assert_array_equal(a.isabort, b.isabort)
    logical = np.isin(a.rectype, list(F.LLOG_LAYOUTS))
    regop = np.isin(a.rectype, list(F.REGOP_TYPES))
    np.testing.assert_array_equal(a.prev[logical | regop], b.prev[logical | regop])
    for i in range(a.nrec):
        t = int(a.rectype[i])
        if t in F.DTA_TYPES or t in F.IX_TYPES:
            assert a.tbnames[a.table[i]] == b.tbnames[b.table[i]], i
        if t in F.IX_TYPES:
            assert int(a.ix[i]) == int(b.ix[i])
            ka = bytes(a.keys[int(a.key_off[i]):int(a.key_off[i]) + int(a.keylen[i])])
            kb = bytes(b.keys[int(b.key_off[i]):int(b.key_off[i]) + int(b.keylen[i])])
            assert ka == kb, i


@pytest.mark.parametrize("seed", range(12))
def test_decode_round_trip(host, seed):
    log, _ = random_case(700 + seed, broken=(seed % 4 == 3))
    raw = F.encode_raw(log)
    got = host.decode_raw(raw)
    same_log(log, got)
    assert got.end_lsn == log.end_lsn


@pytest.mark.parametrize("seed", range(6))
def test_raw_ingest_marshal_equals_soa_ingest(seed):
    log, rs = random_case(800 + seed, broken=(seed % 2 == 1), max_ranges=10)
    a, b = Validator(-1), Validator(-1)
    try:
        a.ingest_log(log)
        b.ingest_raw(F.encode_raw(log))
        W, want = model_marshal(log, rs, a)
        assert native_by_txn(a.marshal(rs)) == want
        # table ids may be numbered differently: compare through the model
        W2, want2 = model_marshal(log, rs, b)
        assert native_by_txn(b.marshal(rs)) == want2
        fa, fb = a.marshal(rs)["forced"], b.marshal(rs)["forced"]
        np.testing.assert_array_equal(fa, fb)
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_raw_ingest_matches_oracle(validator, oracle_mod, seed):
    """bytes -> decoder -> device window -> join == oracle on the SoA log."""
    log, rs = random_case(900 + seed, broken=(seed % 3 == 2))
    validator.ingest_raw(F.encode_raw(log))
    got = validator.check_readsets(rs)
    want, _, _ = oracle_mod.check(log, rs)
    np.testing.assert_array_equal(got != 0, want != 0)


def test_keyless_record_needs_reconstructed_key(host):
    lb = F.LogBuilder(["t1"])
    lb.begin(1)
    lb.write(1, F.REC_UNDO_ADD_IX, "t1", 0, F.enc_int64(5))
    lb.commit(1)
    raw = F.encode_raw(lb.build())
    host.decode_raw(raw)  # with the side table: fine
    bare = F.RawLog(raw.lsn, raw.off, raw.len, raw.buf, raw.end_lsn,
                    np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.int32),
                    np.zeros(1, np.uint8))
    with pytest.raises(HscError):
        host.decode_raw(bare)


def test_truncated_record_is_an_error(host):
    lb = F.LogBuilder(["t1"])
    lb.begin(1)
    lb.write(1, F.REC_UNDO_UPD_IX, "t1", 0, F.enc_int64(5))
    lb.commit(1)
    raw = F.encode_raw(lb.build())
    raw.len[1] -= 3
    with pytest.raises(HscError):
        host.decode_raw(raw)


def test_layout_bytes_of_one_record():
    """Hand-assembled undo_upd_ix (llog.src:108-117) against the encoder."""
    key = F.enc_int64(-1)
    rec = F.encode_record(F.REC_UNDO_UPD_IX, prev=F.lsn(1, 100), isabort=0, tbname="t1", ix=2,
                          key=key, hdr_prev=F.lsn(1, 99), txnid=0x80000001, salt=0)
    g = (0x0123456700000000).to_bytes(8, "little")
    want = (b"\x00\x00\x27\x1b" + b"\x80\x00\x00\x01" + b"\x00\x00\x00\x01\x00\x00\x00\x63"
            + b"\x00\x00\x00\x03t1\x00" + g + g + g + b"\x00\x00\x00\x01\x00\x00\x00\x64"
            + b"\x00\x00\x00\x02" + b"\x00\x00\x00\x09" + key + b"\x00\x00\x00\x00")
    assert rec == want
