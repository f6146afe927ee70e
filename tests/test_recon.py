"""CPU: index-key reconstruction from the physical log.

undo_add_ix / undo_del_ix / undo_del_ix_lk records carry no key; the
reference rebuilds it by walking the berkdb prev_lsn chain from the record's
header prev_lsn over __db_addrem / __db_big / __db_pg_free[data] records
(bdb_reconstruct_add / _delete -> get_next_addrem_buffer, bdb/rowlocks.c:
209-617, called from bdb/serializable.c:120-133,170-184,242-258).  The product
runs that walk in its raw decoder (comdb2_amd/csrc/hsc_logdec.cpp); the oracle
restates it in C (oracle/recon_oracle.c).

* hand-built chains pin each rule with the key derived by hand from the
  reference's control flow (not from either implementation);
* server-shaped logs (formats.encode_raw_physical: inline and overflow keys,
  splits, debug / pg_alloc records, the pg_free pattern, unexpected item
  types) decode to the keys the logical log holds, in the product and in the
  oracle, with no recon side table;
* adversarial chains (items missing, of the wrong length, skipped by a
  pg_free, malformed headers) give the same keys or fail on the same record in
  both;
* appends: a raw log taken in pieces (walks reaching into earlier pieces)
  leaves the window in the state of the whole log.
Run plainly here and under ASan + UBSan by tests/test_sanitize.py."""
import re

import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.formats import LLog, RawLog
from comdb2_amd.hsc import HscError, Validator
from comdb2_amd.workloads import random_case
from test_logdec import same_log

oracle = pytest.importorskip("oracle")


@pytest.fixture(scope="module")
def host():
    v = Validator(-1)
    yield v
    v.close()


def logical_rows(d: LLog, lsns) -> LLog:
    m = np.isin(d.lsn, lsns)
    return LLog(lsn=d.lsn[m], rectype=d.rectype[m], prev=d.prev[m], isabort=d.isabort[m],
                table=d.table[m], ix=d.ix[m], key_off=d.key_off[m], keylen=d.keylen[m],
                keys=d.keys, tbnames=d.tbnames, end_lsn=d.end_lsn)


def raw_of(recs, end_lsn) -> RawLog:
    off = np.cumsum([0] + [len(r) for _, r in recs])[:-1]
    e = np.zeros(0, np.uint64)
    return RawLog(lsn=np.array([l for l, _ in recs], np.uint64), off=np.asarray(off, np.uint64),
                  len=np.array([len(r) for _, r in recs], np.uint32),
                  buf=np.frombuffer(b"".join(r for _, r in recs), np.uint8).copy(),
                  end_lsn=end_lsn, recon_lsn=e, recon_off=e.copy(),
                  recon_len=np.zeros(0, np.int32), recon_keys=np.zeros(1, np.uint8))


def raw_slice(raw: RawLog, a: int, b: int) -> RawLog:
    end = int(raw.lsn[b]) if b < len(raw.lsn) else int(raw.end_lsn)
    return RawLog(lsn=raw.lsn[a:b], off=raw.off[a:b], len=raw.len[a:b], buf=raw.buf, end_lsn=end,
                  recon_lsn=raw.recon_lsn, recon_off=raw.recon_off, recon_len=raw.recon_len,
                  recon_keys=raw.recon_keys)


class Chain:
    """One transaction's records in log order: ltran_start, physical records,
    the keyless index record (header prev_lsn = the last physical record),
    ltran_commit, regop."""

    def __init__(self):
        self.recs, self.lsn, self.last = [], (1 << 32) | 28, 0

    def put(self, make):
        rec = make(self.last)
        self.recs.append((self.lsn, rec))
        self.last = self.lsn
        self.lsn += 64
        return self.recs[-1][0]

    def addrem(self, opcode, hdr=b"", dbt=b""):
        return self.put(lambda p: F.encode_addrem(p, opcode, hdr, dbt))

    def big(self, opcode, chunk):
        return self.put(lambda p: F.encode_big(p, opcode, chunk))

    def other(self, t):
        return self.put(lambda p: F.encode_phys_other(t, p))

    def build(self, rectype, keylen, dtalen=8):
        start = self.recs[0][0] if self.recs else None
        if start is None:
            raise ValueError
        undo = self.put(lambda p: F.encode_record(rectype, start, 0, "tb", 2, b"?" * keylen, p,
                                                  dtalen=dtalen))
        commit = self.put(lambda p: F.encode_record(F.REC_LTRAN_COMMIT, undo, 0, None, 0, None, p))
        self.put(lambda p: F.encode_record(F.REC_TXN_REGOP, commit, 0, None, 0, None, p))
        return raw_of(self.recs, self.lsn), undo

    def start(self):
        return self.put(lambda p: F.encode_record(F.REC_LTRAN_START, 0, 0, None, 0, None, 0))


def decoded_key(v, raw, undo):
    """(product key, oracle key) of the keyless record at LSN undo; None for
    a reconstruction the implementation rejects."""
    try:
        p = v.decode_raw(raw)
        i = int(np.nonzero(p.lsn == undo)[0][0])
        pk = bytes(p.keys[int(p.key_off[i]):int(p.key_off[i]) + int(p.keylen[i])])
    except HscError:
        pk = None
    try:
        o = oracle.decode_raw(raw)
        i = int(np.nonzero(o.lsn == undo)[0][0])
        ok = bytes(o.keys[int(o.key_off[i]):int(o.key_off[i]) + int(o.keylen[i])])
    except oracle.OracleUndefined:
        ok = None
    return pk, ok


K = b"\x08\x80\x00\x00\x00\x00\x00\x00\x2a"  # enc_int64(42)
GEN = bytes(range(1, 9))
ADD, REM, ADDB, REMB = F.DB_ADD_DUP, F.DB_REM_DUP, F.DB_ADD_BIG, F.DB_REM_BIG


def case_add_plain(c):      # DB_ADD_DUP, no header: the item is the dbt (:300-321)
    c.addrem(ADD, b"", K), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, K


def case_add_type0(c):      # a header whose B_TYPE is 0 also means "item in dbt"
    c.addrem(ADD, b"\x00\x00\x80", K), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, K


def case_add_overflow(c):   # BOVERFLOW header: tlen, then the pages back to front (:326-337,382-399)
    c.big(ADDB, K[:2]), c.big(ADDB, K[2:5]), c.big(ADDB, K[5:])
    c.addrem(ADD, F.boverflow(len(K)), b""), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, K


def case_add_keydata_data(c):  # data item as a B_KEYDATA header: the data walk stops there
    c.addrem(ADD, b"", K), c.addrem(ADD, F.bkeydata(GEN), GEN)
    return F.REC_UNDO_ADD_IX, K


def case_del_keydata(c):    # DB_REM_DUP: the item is the page's BKEYDATA (delete flag set)
    c.addrem(REM, F.bkeydata(K, 0x80)), c.addrem(REM, F.bkeydata(GEN))
    return F.REC_UNDO_DEL_IX, K


def case_del_overflow(c):
    c.big(REMB, K[:4]), c.big(REMB, K[4:])
    c.addrem(REM, F.boverflow(len(K), flags=0x80)), c.addrem(REM, F.bkeydata(GEN))
    return F.REC_UNDO_DEL_IX_LK, K


def case_pgfree_skip(c):    # the addrem right after a pg_free (walking back) is skipped (:275-289)
    c.addrem(ADD, b"", K), c.other(F.REC_DB_PG_ALLOC)
    c.addrem(ADD, b"", b"\xee" * len(K)), c.other(F.REC_DB_PG_FREE), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, K


def case_pgfree_sticky(c):  # ... and every addrem after it until another record type:
    # the real key is skipped too and the walk takes the decoy logged before it
    decoy = b"\x08\x80" + b"\x00" * 6 + b"\x07"
    c.addrem(ADD, b"", decoy), c.other(F.REC_DB_PG_ALLOC)
    c.addrem(ADD, b"", K), c.addrem(ADD, b"", b"\xee" * len(K))
    c.other(F.REC_DB_PG_FREEDATA), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, decoy


def case_debug_keeps_skip(c):  # a debug record does not end the skip
    decoy = b"\x08\x80" + b"\x00" * 6 + b"\x05"
    c.addrem(ADD, b"", decoy), c.other(F.REC_DB_PG_ALLOC), c.addrem(ADD, b"", K)
    c.other(F.REC_DB_DEBUG), c.other(F.REC_DB_PG_FREE), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, decoy


def case_unexpected_type(c):  # a B_DUPLICATE item: "Unexpected type", the walk goes on
    c.addrem(REM, F.bkeydata(K)), c.addrem(REM, bytes([4, 0, F.B_DUPLICATE]) + b"dupx")
    c.addrem(REM, F.bkeydata(GEN))
    return F.REC_UNDO_DEL_IX, K


def case_del_first_pair(c):  # delete keeps the first two items found (walking back)
    c.addrem(REM, F.bkeydata(b"\x08" + b"\x11" * 8)), c.addrem(REM, F.bkeydata(K))
    c.addrem(REM, F.bkeydata(GEN))
    return F.REC_UNDO_DEL_IX, K


def case_del_refill(c):     # an item larger than the buffer clears its slot's have flag
    # (:309-310) and the loop continues until both slots hold one again: the
    # key is the last walk's buffer
    c.addrem(REM, F.bkeydata(K)), c.addrem(REM, F.bkeydata(GEN))
    c.addrem(ADD, b"", b"\x55" * 40)
    return F.REC_UNDO_DEL_IX, K


def case_add_too_long(c):   # a key item longer than keylen is never copied: undefined
    c.addrem(ADD, b"", K + b"\x00"), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, None


def case_missing_key(c):    # the walk runs back to ltran_start without a key item
    c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, None


def case_short_overflow(c):  # pages short of tlen: the walk ends at ltran_start
    c.big(ADDB, K[4:]), c.addrem(ADD, F.boverflow(len(K)), b""), c.addrem(ADD, b"", GEN)
    return F.REC_UNDO_ADD_IX, None


CASES = [case_add_plain, case_add_type0, case_add_overflow, case_add_keydata_data,
         case_del_keydata, case_del_overflow, case_pgfree_skip, case_pgfree_sticky,
         case_debug_keeps_skip, case_unexpected_type, case_del_first_pair, case_del_refill,
         case_add_too_long, case_missing_key, case_short_overflow]


@pytest.mark.parametrize("case", CASES, ids=lambda f: f.__name__[5:])
def test_hand_built_chains(host, case):
    c = Chain()
    c.start()
    rectype, want = case(c)
    raw, undo = c.build(rectype, len(K))
    pk, ok = decoded_key(host, raw, undo)
    assert ok == want, "oracle"
    assert pk == want, "product"


@pytest.mark.parametrize("seed", range(16))
def test_server_shaped_logs_decode_to_the_logical_keys(host, seed):
    keylens = (9, 18, 5) if seed % 2 else (64, 40, 27)
    log, _ = random_case(1300 + seed, n_commits=60, keylens=keylens, broken=(seed % 4 == 3))
    raw = F.encode_raw_physical(log, seed=seed, overflow=0.4)
    assert len(raw.recon_lsn) == 0 and len(raw.lsn) > log.nrec
    p = host.decode_raw(raw)
    o = oracle.decode_raw(raw)
    same_log(log, logical_rows(p, log.lsn))
    same_log(log, logical_rows(o, log.lsn))
    same_log(o, p)


@pytest.mark.parametrize("seed", range(24))
def test_adversarial_chains_agree_with_the_oracle(host, seed):
    log, _ = random_case(1400 + seed, n_commits=50, keylens=(9, 8, 18))
    raw = F.encode_raw_physical(log, seed=seed, adversarial=(0.02, 0.1, 0.4)[seed % 3])
    try:
        o, oe = oracle.decode_raw(raw), None
    except oracle.OracleUndefined as e:
        o, oe = None, e
    try:
        p, pe = host.decode_raw(raw), None
    except HscError as e:
        p, pe = None, e
    assert (oe is None) == (pe is None), (oe, pe)
    if oe is None:
        same_log(o, p)
    else:
        assert re.search(r"record (\d+)", str(oe)).group(1) == \
            re.search(r"record (\d+)", str(pe)).group(1)


def state(v, rs):
    m = v.marshal(rs)
    return (v.table_max().tolist(), v.end_lsn,
            {k: (m[k].tolist() if hasattr(m[k], "tolist") else m[k]) for k in m})


@pytest.mark.parametrize("seed", range(8))
def test_raw_appends_walk_into_earlier_pieces(seed):
    """ingest_raw of a prefix, append_raw of the rest in pieces cut anywhere
    (also between a key's physical records and its logical record): the
    marshalled probes of every read set equal those of the logical log."""
    log, rs = random_case(1500 + seed, n_commits=60, keylens=(9, 30), broken=(seed % 3 == 0))
    raw = F.encode_raw_physical(log, seed=seed, overflow=0.5)
    whole = Validator(-1)
    whole.ingest_log(log)
    want = state(whole, rs)
    whole.close()
    rng = np.random.default_rng(seed)
    cuts = sorted(set(rng.integers(1, len(raw.lsn), size=6).tolist()))
    pieces = [0] + cuts + [len(raw.lsn)]
    v = Validator(-1)
    v.ingest_raw(raw_slice(raw, 0, pieces[1]))
    for a, b in zip(pieces[1:], pieces[2:]):
        v.append_raw(raw_slice(raw, a, b))
    got = state(v, rs)
    v.close()
    assert got == want


def test_a_new_ingest_forgets_earlier_records(host):
    """Walks of an ingested raw log see only its own records: a keyless record
    whose items were in a previous log fails to decode."""
    c = Chain()
    c.start()
    case_add_plain(c)
    raw, undo = c.build(F.REC_UNDO_ADD_IX, len(K))
    v = Validator(-1)
    try:
        v.ingest_raw(raw)
        later = raw_slice(raw, len(raw.lsn) - 3, len(raw.lsn))  # the logical records only
        with pytest.raises(HscError):
            v.ingest_raw(later)
    finally:
        v.close()
