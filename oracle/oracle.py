"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement
(oracle/serial_oracle.c) of comdb2's serializable check.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.  The product
(comdb2_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle_serial.so")
sys.path.insert(0, os.path.dirname(_HERE))

from comdb2_amd.formats import LLog, ReadSets  # noqa: E402  (data containers only)

_p = C.c_void_p
_lib = None


class _OrLog(C.Structure):
    _fields_ = [("nrec", C.c_size_t), ("lsn", _p), ("rectype", _p), ("prev", _p),
                ("isabort", _p), ("table", _p), ("ix", _p), ("key_off", _p), ("keylen", _p),
                ("keys", _p), ("tbnames", C.POINTER(C.c_char_p)), ("ntbnames", C.c_int),
                ("end_lsn", C.c_uint64)]


class _SjProbes(C.Structure):
    _fields_ = [("n", C.c_size_t), ("lo", _p), ("hi", _p), ("gid", _p), ("snap", _p), ("txn", _p),
                ("n_lock", C.c_size_t), ("lock_table", _p), ("lock_snap", _p), ("lock_txn", _p),
                ("table_max", _p), ("ntables", C.c_uint32)]


class _RoLog(C.Structure):
    _fields_ = [("nrec", C.c_size_t), ("lsn", _p), ("off", _p), ("len", _p), ("buf", _p)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        lib.or_serial_check_many.restype = C.c_double
        lib.or_serial_check_many.argtypes = [C.POINTER(_OrLog), _p, C.c_int, C.c_int, C.c_int,
                                             C.POINTER(C.c_int)]
        lib.or_build_arrs.restype = _p
        lib.or_build_arrs.argtypes = [C.c_int] + [_p] * 12 + [C.POINTER(C.c_char_p)]
        lib.or_free_arrs.restype = None
        lib.or_free_arrs.argtypes = [_p, C.c_int]
        lib.dg_edges.restype = C.c_size_t
        lib.dg_edges.argtypes = [C.c_size_t, _p, _p, _p, _p, C.POINTER(_p), C.POINTER(_p),
                                 C.POINTER(_p)]
        lib.dg_free.argtypes = [_p]
        lib.dg_scc.argtypes = [C.c_uint32, C.c_size_t, _p, _p, _p]
        lib.sj_build.restype = _p
        lib.sj_build.argtypes = [C.c_size_t, C.c_int, C.c_uint32, _p, _p, _p, C.POINTER(C.c_double)]
        lib.sj_free.argtypes = [_p]
        lib.sj_rows.restype = C.c_size_t
        lib.sj_rows.argtypes = [_p]
        lib.sj_probe.restype = C.c_double
        lib.sj_probe.argtypes = [_p, C.POINTER(_SjProbes), C.c_int, _p]
        lib.co_coalesce.restype = C.c_long
        lib.co_coalesce.argtypes = [C.c_int] + [_p] * 10 + [_p, C.c_uint64, C.POINTER(C.c_char_p),
                                                            C.c_int] + [_p] * 10
        lib.ro_reconstruct.restype = C.c_int
        lib.ro_reconstruct.argtypes = [C.POINTER(_RoLog), C.c_int, C.c_uint64, C.c_int, C.c_int,
                                       _p, C.POINTER(C.c_int)]
        lib.or_serial_check.restype = C.c_int
        lib.or_serial_check.argtypes = [C.POINTER(_OrLog), _p, C.POINTER(C.c_uint),
                                        C.POINTER(C.c_uint), C.c_int]
        _lib = lib
    return _lib


def _names(tbnames):
    arr = (C.c_char_p * max(1, len(tbnames)))()
    for i, n in enumerate(tbnames):
        arr[i] = n.encode()
    return arr


class OracleLog:
    """An LLog pinned for the oracle (keeps the arrays alive)."""

    def __init__(self, log: LLog):
        self.cols = [np.ascontiguousarray(a) for a in (
            log.lsn.astype(np.uint64), log.rectype.astype(np.uint32), log.prev.astype(np.uint64),
            log.isabort.astype(np.int16), log.table.astype(np.int32), log.ix.astype(np.int16),
            log.key_off.astype(np.uint64), log.keylen.astype(np.int32), log.keys.astype(np.uint8))]
        self.names = _names(log.tbnames)
        self.s = _OrLog(log.nrec, *[c.ctypes.data for c in self.cols], self.names,
                        len(log.tbnames), int(log.end_lsn))


def check(log, rs: ReadSets, regop_only: int = 0, nthreads: int = 1):
    """bdb_osql_serial_check per read set.  Returns (rc int32[ntxn],
    post-call snapshot LSNs uint64[ntxn], wall seconds of the checks)."""
    lib = load()
    ol = log if isinstance(log, OracleLog) else OracleLog(log)
    cols = [np.ascontiguousarray(a) for a in (
        rs.txn_off.astype(np.int64), rs.snap.astype(np.uint64), rs.table.astype(np.int32),
        rs.idxnum.astype(np.int32), rs.lflag.astype(np.int32), rs.rflag.astype(np.int32),
        rs.islocked.astype(np.int32), rs.lkeylen.astype(np.int32), rs.rkeylen.astype(np.int32),
        rs.lkey_off.astype(np.uint64), rs.rkey_off.astype(np.uint64), rs.keys.astype(np.uint8))]
    names = _names(rs.tbnames)
    arrs = lib.or_build_arrs(rs.ntxn, *[c.ctypes.data for c in cols], names)
    try:
        rc = np.zeros(max(1, rs.ntxn), dtype=np.int32)
        secs = lib.or_serial_check_many(C.byref(ol.s), arrs, rs.ntxn, regop_only, nthreads,
                                        rc.ctypes.data_as(C.POINTER(C.c_int)))
        # read back (file, offset) written by the full checks
        ptrs = C.cast(arrs, C.POINTER(C.POINTER(C.c_uint * 4)))
        post = np.zeros(rs.ntxn, dtype=np.uint64)
        for i in range(rs.ntxn):
            hdr = ptrs[i].contents  # size, cap, file, offset
            post[i] = (int(hdr[2]) << 32) | int(hdr[3])
    finally:
        lib.or_free_arrs(arrs, rs.ntxn)
    return rc[: rs.ntxn], post, secs


def dep_edges(txn, key, is_write, observed):
    """WR/WW/RW edges of a history (Adya): (src, dst, type bits) sorted by
    (src, dst), type bits 1 = ww, 2 = wr, 4 = rw."""
    lib = load()
    cols = [np.ascontiguousarray(txn, np.uint32), np.ascontiguousarray(key, np.uint64),
            np.ascontiguousarray(is_write, np.uint8), np.ascontiguousarray(observed, np.int64)]
    ps, pd, pt = _p(), _p(), _p()
    m = lib.dg_edges(len(cols[0]), *[c.ctypes.data for c in cols], C.byref(ps), C.byref(pd),
                     C.byref(pt))
    out = []
    for p in (ps, pd, pt):
        a = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(max(m, 1),))[:m].copy()
        lib.dg_free(p)
        out.append(a)
    return tuple(out)


def scc(n, src, dst):
    """Tarjan: scc[v] = largest node id of v's strongly connected component."""
    lib = load()
    src = np.ascontiguousarray(src, np.uint32)
    dst = np.ascontiguousarray(dst, np.uint32)
    out = np.zeros(max(1, n), dtype=np.uint32)
    lib.dg_scc(n, len(src), src.ctypes.data, dst.ctypes.data, out.ctypes.data)
    return out[:n]


class SortJoin:
    """CPU BASELINE: the build's own multi-threaded sort-join (oracle/sortjoin.c)
    over a write window given as rows (gid u32[n], words u64[W][n], lsn u64[n])."""

    def __init__(self, gid, words, lsn, ngroups: int):
        self.lib = load()
        words = np.ascontiguousarray(np.asarray(words, np.uint64).reshape(-1, len(lsn)))
        self.W = words.shape[0]
        gid = np.ascontiguousarray(gid, np.uint32)
        lsn = np.ascontiguousarray(lsn, np.uint64)
        secs = C.c_double()
        self.w = self.lib.sj_build(len(lsn), self.W, ngroups, gid.ctypes.data, words.ctypes.data,
                                   lsn.ctypes.data, C.byref(secs))
        if not self.w:
            raise MemoryError("sj_build")
        self.build_s = secs.value
        self.rows = self.lib.sj_rows(self.w)

    def probe(self, m: dict, table_max, nthreads: int = 1):
        """m: a marshalled batch (Validator.marshal).  Returns (verdict uint8
        [n_txn] including m['forced'], wall seconds of the probe phase)."""
        assert m["words"] == self.W
        keep = [np.ascontiguousarray(m["lo"], np.uint64), np.ascontiguousarray(m["hi"], np.uint64),
                np.ascontiguousarray(m["gid"], np.uint32), np.ascontiguousarray(m["snap"], np.uint64),
                np.ascontiguousarray(m["txn"], np.uint32),
                np.ascontiguousarray(m["lock_table"], np.uint32),
                np.ascontiguousarray(m["lock_snap"], np.uint64),
                np.ascontiguousarray(m["lock_txn"], np.uint32),
                np.ascontiguousarray(table_max, np.uint64)]
        s = _SjProbes(m["n"], *[k.ctypes.data for k in keep[:5]], m["n_lock"],
                      *[k.ctypes.data for k in keep[5:]], len(keep[8]))
        verdict = np.ascontiguousarray(m["forced"], np.uint8).copy()
        secs = self.lib.sj_probe(self.w, C.byref(s), nthreads, verdict.ctypes.data)
        return verdict, secs

    def close(self):
        if self.w:
            self.lib.sj_free(self.w)
            self.w = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def coalesce(rs: ReadSets) -> ReadSets:
    """currangearr_coalesce (db/sqlglue.c:305-311) of every read set
    (oracle/coalesce_oracle.c).  The result keeps rs.keys; its key offsets
    point into it."""
    import dataclasses
    lib = load()
    nr = len(rs.table)
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    ins = [np.ascontiguousarray(rs.txn_off, np.int64), i32(rs.table), i32(rs.idxnum), i32(rs.lflag),
           i32(rs.rflag), i32(rs.islocked), i32(rs.lkeylen), i32(rs.rkeylen),
           np.ascontiguousarray(rs.lkey_off, np.uint64), np.ascontiguousarray(rs.rkey_off, np.uint64)]
    keys = np.ascontiguousarray(rs.keys, np.uint8)
    names = (C.c_char_p * max(1, len(rs.tbnames)))(*[n.encode() for n in rs.tbnames])
    out_off = np.zeros(rs.ntxn + 1, np.int64)
    outs = [np.zeros(nr, np.int32) for _ in range(7)] + [np.zeros(nr, np.uint64) for _ in range(2)]
    tot = lib.co_coalesce(rs.ntxn, *[a.ctypes.data for a in ins], keys.ctypes.data, len(keys),
                          names, len(rs.tbnames), out_off.ctypes.data, *[a.ctypes.data for a in outs])
    if tot < 0:
        raise ValueError("co_coalesce: a range names no table")
    o = [a[:tot].copy() for a in outs]
    return dataclasses.replace(rs, txn_off=out_off, table=o[0], idxnum=o[1], lflag=o[2], rflag=o[3],
                               islocked=o[4], lkeylen=o[5], rkeylen=o[6], lkey_off=o[7],
                               rkey_off=o[8])


# ---------------------------------------------------------------------------
# raw log decode with index-key reconstruction (recon_oracle.c)
# ---------------------------------------------------------------------------
class OracleUndefined(Exception):
    """A keyless index record whose key the reference would leave
    (partly) uninitialised, or a walk over malformed physical bytes."""


_LAYOUTS = {  # bdb/llog.src:26-225 field programs (formats.LLOG_LAYOUTS letters)
    10003: "TiiGGPD", 10004: "TIGGPkd", 10005: "GPGA", 10006: "Gi", 10007: "GPL",
    10008: "TGGPiiiD", 10009: "TGIGPDkd", 10010: "TGGGPiiDDi", 10011: "TGGGPIKi",
    10013: "TiiGGP", 10014: "TIGGPKi", 10015: "TGGPiii", 10016: "TGIGPkd",
    10017: "TGGGPiii", 10018: "TGGGPIKi"}


def decode_raw(raw) -> LLog:
    """Oracle decode of a raw log (formats.RawLog): llog records by their
    bdb/llog.src layouts; the keys of undo_add_ix / undo_del_ix[_lk] by the
    restated bdb_reconstruct_add / _delete walk from undolsn = the header
    prev_lsn (bdb/serializable.c:120-133,170-184,242-258) -- or from the
    recon side table when it names undolsn.  Raises OracleUndefined when a
    key is not fully defined by the walk."""
    lib = load()
    cols = [np.ascontiguousarray(raw.lsn, np.uint64), np.ascontiguousarray(raw.off, np.uint64),
            np.ascontiguousarray(raw.len, np.uint32), np.ascontiguousarray(raw.buf, np.uint8)]
    rl = _RoLog(len(cols[0]), *[c.ctypes.data for c in cols])
    recon = {int(u): bytes(raw.recon_keys[int(o):int(o) + int(n)])
             for u, o, n in zip(raw.recon_lsn, raw.recon_off, raw.recon_len)}
    buf = bytes(raw.buf)
    be = lambda b, o: int.from_bytes(b[o:o + 4], "big")  # noqa: E731
    rows, keys, names, tid = [], bytearray(), [], {}
    for i in range(len(cols[0])):
        o, n = int(raw.off[i]), int(raw.len[i])
        r = buf[o:o + n]
        if n < 16:
            raise OracleUndefined(f"record {i}: truncated header")
        t, hprev = be(r, 0), (be(r, 8) << 32) | be(r, 12)
        row = dict(lsn=int(raw.lsn[i]), t=t, prev=hprev, isabort=0, table=-1, ix=0, koff=0,
                   klen=0)
        prog = _LAYOUTS.get(t)
        if prog is not None:
            row["prev"] = 0
            q, key, klen, dtalen = 16, None, 0, 0
            for f in prog:
                if f in "TDK":
                    sz = be(r, q)
                    d = r[q + 4:q + 4 + sz]
                    if len(d) < sz:
                        raise OracleUndefined(f"record {i}: truncated")
                    q += 4 + sz
                    if f == "T":
                        nm = d.split(b"\x00")[0].decode("utf-8", "surrogateescape")
                        row["table"] = tid.setdefault(nm, len(names))
                        if row["table"] == len(names):
                            names.append(nm)
                    elif f == "K":
                        key, klen = d, sz
                elif f == "G":
                    q += 8
                elif f in "PL":
                    v = (be(r, q) << 32) | be(r, q + 4)
                    q += 8
                    if f == "P":
                        row["prev"] = v
                else:
                    v = be(r, q)
                    q += 4
                    if f == "I":
                        row["ix"] = int(np.int16(np.uint16(v & 0xFFFF)))
                    elif f == "k":
                        klen = v
                    elif f == "d":
                        dtalen = v
                    elif f == "A":
                        row["isabort"] = int(np.int16(np.uint16(v & 0xFFFF)))
                if q > n:
                    raise OracleUndefined(f"record {i}: truncated")
            if t in (10004, 10009, 10016):
                if hprev in recon:
                    key = recon[hprev]
                else:
                    kb = np.zeros(max(klen, 1), np.uint8)
                    defined = C.c_int(0)
                    lib.ro_reconstruct(C.byref(rl), 0 if t == 10004 else 1, hprev, klen, dtalen,
                                       kb.ctypes.data, C.byref(defined))
                    if not defined.value:
                        raise OracleUndefined(f"record {i}: key not reconstructed")
                    key = bytes(kb[:klen])
            if key is not None:
                row["koff"], row["klen"] = len(keys), len(key)
                keys += key
        rows.append(row)
    col = lambda k, dt: np.array([x[k] for x in rows], dtype=dt)  # noqa: E731
    return LLog(lsn=col("lsn", np.uint64), rectype=col("t", np.uint32), prev=col("prev", np.uint64),
                isabort=col("isabort", np.int16), table=col("table", np.int32),
                ix=col("ix", np.int16), key_off=col("koff", np.uint64),
                keylen=col("klen", np.int32),
                keys=np.frombuffer(bytes(keys) or b"\x00", np.uint8).copy(), tbnames=names,
                end_lsn=int(raw.end_lsn))
