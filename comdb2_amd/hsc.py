"""ctypes bindings of ``libhsc.so`` (the C ABI in ``include/hip_serial.h``).

The shared library is built in-tree (``comdb2_amd/lib/libhsc.so``) by
``__graft_entry__.build()`` / ``make -C comdb2_amd/csrc``.  There is no
fallback: if the library is missing, or no GPU is visible, the validator
raises.  Python is only plumbing here -- marshalling and the verdicts run in
the native library and on the GPU.

Interface names follow the reference:
  * :func:`bdb_osql_serial_check` <- ``bdb/serializable.c:571``
  * :class:`CurRange` / :class:`CurRangeArr` <- ``db/comdb2.h:1105-1124``
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from .formats import KEY_NULL, LLog, Range, ReadSets

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HSC_LIB") or os.path.join(_HERE, "lib", "libhsc.so")

HSC_OK, HSC_EINVAL, HSC_EDEVICE, HSC_ENOMEM, HSC_ELOG, HSC_ESTATE = 0, -1, -2, -3, -4, -5


class HscError(RuntimeError):
    pass


_p = C.c_void_p
_u64p = C.POINTER(C.c_uint64)


class CurRange(C.Structure):
    """Layout mirror of CurRange (db/comdb2.h:1105-1115)."""
    _fields_ = [("tbname", C.c_char_p), ("idxnum", C.c_int), ("lkey", _p), ("rkey", _p),
                ("lflag", C.c_int), ("lkeylen", C.c_int), ("rflag", C.c_int),
                ("rkeylen", C.c_int), ("islocked", C.c_int)]


class CurRangeArr(C.Structure):
    """Layout mirror of CurRangeArr (db/comdb2.h:1117-1124)."""
    _fields_ = [("size", C.c_int), ("cap", C.c_int), ("file", C.c_uint), ("offset", C.c_uint),
                ("hash", _p), ("ranges", C.POINTER(C.POINTER(CurRange)))]


class _LLog(C.Structure):
    _fields_ = [("nrec", C.c_size_t), ("lsn", _p), ("rectype", _p), ("prev", _p),
                ("isabort", _p), ("table", _p), ("ix", _p), ("key_off", _p), ("keylen", _p),
                ("keys", _p), ("tbnames", C.POINTER(C.c_char_p)), ("ntbnames", C.c_int),
                ("end_lsn", C.c_uint64)]


class _RawLog(C.Structure):
    _fields_ = [("nrec", C.c_size_t), ("lsn", _p), ("off", _p), ("len", _p), ("buf", _p),
                ("end_lsn", C.c_uint64), ("nrecon", C.c_size_t), ("recon_lsn", _p),
                ("recon_off", _p), ("recon_len", _p), ("recon_keys", _p)]


class _SerialMsgs(C.Structure):
    _fields_ = [("nmsg", C.c_size_t), ("buf", _p), ("off", _p), ("len", _p)]


class _ReadSets(C.Structure):
    _fields_ = [("ntxn", C.c_int), ("txn_off", _p), ("snap", _p), ("table", _p),
                ("idxnum", _p), ("lflag", _p), ("rflag", _p), ("islocked", _p),
                ("lkeylen", _p), ("rkeylen", _p), ("lkey_off", _p), ("rkey_off", _p),
                ("keys", _p), ("tbnames", C.POINTER(C.c_char_p)), ("ntbnames", C.c_int)]


class _Write(C.Structure):
    """hsc_write: one decoded committed write."""
    _fields_ = [("tbname", C.c_char_p), ("idxnum", C.c_int), ("key", _p), ("keylen", C.c_int),
                ("commit_lsn", C.c_uint64)]


class ProbeBatch(C.Structure):
    """hsc_probe_batch: device pointers (ints) of a resident probe batch."""
    _fields_ = [("n", C.c_size_t), ("lo", _p), ("hi", _p), ("gid", _p), ("snap", _p),
                ("txn", _p), ("n_lock", C.c_size_t), ("lock_table", _p), ("lock_snap", _p),
                ("lock_txn", _p), ("n_txn", C.c_size_t), ("verdict", _p), ("bitmap", _p)]


class Timing(C.Structure):
    _fields_ = [("locate_ms", C.c_float), ("plan_ms", C.c_float), ("scatter_ms", C.c_float),
                ("join_ms", C.c_float), ("pack_ms", C.c_float), ("probe_total_ms", C.c_float),
                ("ingest_ms", C.c_float), ("records", C.c_uint64), ("tiles", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class _History(C.Structure):
    _fields_ = [("nops", C.c_size_t), ("ntxn", C.c_uint32), ("txn", _p), ("key", _p),
                ("is_write", _p), ("observed", _p)]


class GraphStats(C.Structure):
    _fields_ = [("edges", C.c_uint64), ("ww", C.c_uint64), ("wr", C.c_uint64), ("rw", C.c_uint64),
                ("nontrivial_sccs", C.c_uint32), ("txns_in_cycles", C.c_uint32),
                ("rounds", C.c_uint32), ("iterations", C.c_uint32), ("build_ms", C.c_float),
                ("scc_ms", C.c_float), ("cut_nodes", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class OpsDev(C.Structure):
    """hsc_ops_dev: one key shard's history ops on its member's GPU."""
    _fields_ = [("nops", C.c_size_t), ("txn", _p), ("key", _p), ("is_write", _p), ("observed", _p)]


class Marshalled(C.Structure):
    _fields_ = [("n", C.c_size_t), ("n_lock", C.c_size_t), ("n_txn", C.c_size_t),
                ("words", C.c_int), ("lo", _u64p), ("hi", _u64p),
                ("gid", C.POINTER(C.c_uint32)), ("snap", _u64p), ("txn", C.POINTER(C.c_uint32)),
                ("lock_table", C.POINTER(C.c_uint32)), ("lock_snap", _u64p),
                ("lock_txn", C.POINTER(C.c_uint32)), ("forced", C.POINTER(C.c_uint8))]


class CollectorStats(C.Structure):
    _fields_ = [("calls", C.c_uint64), ("batches", C.c_uint64), ("max_batch", C.c_uint64),
                ("busy_ns", C.c_uint64), ("gate_ns", C.c_uint64), ("handout_ns", C.c_uint64),
                ("pass_ns", C.c_uint64)]


class SmallStats(C.Structure):
    _fields_ = [("calls", C.c_uint64), ("marshal_ns", C.c_uint64), ("launch_ns", C.c_uint64),
                ("wait_ns", C.c_uint64), ("slot_waits", C.c_uint64), ("lock_ns", C.c_uint64)]


class BatchStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("marshals", "read_sets", "ranges", "parts_ns", "alloc_ns",
                                          "assemble_ns", "launch_ns", "wait_ns")]


class ProtocolTxn(C.Structure):
    """hsc_protocol_txn: one txn of the commit-protocol harness."""
    _fields_ = [("arr", _p), ("writes", _p), ("nwrites", C.c_int)]


class ProtocolResult(C.Structure):
    _fields_ = [("seconds", C.c_double), ("commits", C.c_uint64), ("aborts", C.c_uint64),
                ("regop_probes", C.c_uint64), ("full_checks", C.c_uint64),
                ("regop_p50_us", C.c_double), ("regop_p99_us", C.c_double),
                ("regop_p999_us", C.c_double), ("regop_max_us", C.c_double),
                ("full_p50_us", C.c_double), ("full_p99_us", C.c_double),
                ("hold_p50_us", C.c_double), ("hold_p99_us", C.c_double),
                ("commit_p50_us", C.c_double), ("commit_p99_us", C.c_double)]


class ConcurrentResult(C.Structure):
    _fields_ = [("seconds", C.c_double), ("calls", C.c_uint64), ("lat_mean_us", C.c_double),
                ("lat_p50_us", C.c_double), ("lat_p99_us", C.c_double)]


# Every symbol include/hip_serial.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "hsc_ctx_create", "hsc_ctx_destroy", "hsc_set_stream", "hsc_last_error", "hsc_device_count",
    "hsc_window_ingest_log", "hsc_window_append", "hsc_window_set_end", "hsc_window_reset",
    "hsc_window_build", "hsc_register_group", "hsc_window_ingest_device", "hsc_window_words",
    "hsc_window_keys", "hsc_window_end", "hsc_window_max_commit", "hsc_window_export", "hsc_set_fold", "hsc_fold_stats", "hsc_append_stats", "hsc_set_paths", "hsc_window_sort_path", "hsc_table_id",
    "hsc_table_name", "hsc_group_info", "hsc_table_max", "hsc_merge_table_max",
    "hip_bdb_osql_serial_check", "hip_serial_check_batch", "hsc_check_readsets",
    "hsc_marshal_readsets", "hsc_probe_device", "hsc_pack_verdicts", "hsc_or_bitmaps",
    "hsc_synchronize",
    "hsc_get_timing",
    "hsc_enable_timing", "hsc_dep_graph_scc", "hsc_dep_graph_edges",
    "hsc_window_ingest_raw", "hsc_decode_log", "hsc_decode_serial", "hsc_check_serial",
    "hsc_set_layout", "hsc_window_layout", "hsc_coalesce_readsets", "hsc_rw_edges",
    "hsc_window_code_words", "hsc_window_tile_key_words", "hsc_window_append_log", "hsc_window_append_raw",
    "hsc_window_delta_rows", "hsc_set_threads", "hsc_currangearrs_build",
    "hsc_currangearrs_free", "hsc_collector_create", "hsc_collector_destroy",
    "hsc_collector_check", "hsc_collector_get_stats", "hsc_collector_set_inflight",
    "hsc_set_autocollect",
    "hsc_small_stats", "hsc_harness_concurrent",
    "hsc_dep_graph_build", "hsc_dep_graph_stage_rw_pairs", "hsc_dep_graph_scc_built", "hsc_dep_graph_build_device", "hsc_dep_graph_cover", "hsc_dep_graph_cut", "hsc_dep_graph_scc_cut",
    "hsc_multi_create", "hsc_multi_unique_ids", "hsc_multi_create_rank", "hsc_multi_world",
    "hsc_multi_rank", "hsc_multi_local", "hsc_multi_member", "hsc_multi_set_splitters",
    "hsc_multi_adopt", "hsc_multi_probe_device", "hsc_multi_stats", "hsc_multi_last_counts",
    "hsc_multi_phase_stats", "hsc_multi_set_transport", "hsc_multi_probe_routed",
    "hsc_multi_marshal_routed", "hsc_multi_routed_member", "hsc_multi_enable_timing",
    "hsc_multi_member_probe_ms", "hsc_multi_route_stats", "hsc_multi_graph_scc",
    "hsc_multi_graph_phase_ms",
    "hsc_marshal_arrs", "hsc_batch_stats", "hsc_regop_stats", "hsc_harness_commit_protocol",
    "hsc_multi_set_mode", "hsc_multi_mode", "hsc_multi_routed_phase_stats",
]
MULTI_AUTO, MULTI_PIECES, MULTI_REPLICAS = 0, 1, 2
MULTI_ID_BYTES = 2 * 128  # hsc_multi_unique_ids: one RCCL id per lane

(LAYOUT_AUTO, LAYOUT_WIDE, LAYOUT_NARROW, LAYOUT_NARROW_DIRECT, LAYOUT_NARROW_TILES,
 LAYOUT_NARROW_CODES, LAYOUT_COMPACT, LAYOUT_COMPACT_WIDE) = 0, 1, 2, 3, 4, 5, 6, 7
# hsc_set_paths flags (include/hip_serial.h)
(PATH_NO_SMALL, PATH_NO_PACKED_SORT, PATH_TILE_DIR, PATH_CO_SERIAL, PATH_CO_RUN_THREAD,
 PATH_NO_COMP_NARROW, PATH_NO_CT_POINTS) = 1, 2, 4, 8, 16, 32, 64

_lib: Optional[C.CDLL] = None


def load() -> C.CDLL:
    """Load libhsc.so (raises HscError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HscError(f"{LIB_PATH} missing: run __graft_entry__.build() "
                       "(make -C comdb2_amd/csrc)")
    lib = C.CDLL(LIB_PATH)
    ctx_pp = C.POINTER(_p)
    sig = {
        "hsc_ctx_create": (C.c_int, [C.c_int, ctx_pp]),
        "hsc_ctx_destroy": (None, [_p]),
        "hsc_set_stream": (C.c_int, [_p, _p]),
        "hsc_last_error": (C.c_char_p, [_p]),
        "hsc_device_count": (C.c_int, []),
        "hsc_window_ingest_log": (C.c_int, [_p, C.POINTER(_LLog)]),
        "hsc_window_append": (C.c_int, [_p, _p, C.c_size_t]),
        "hsc_window_set_end": (C.c_int, [_p, C.c_uint64]),
        "hsc_window_reset": (C.c_int, [_p]),
        "hsc_window_build": (C.c_int, [_p]),
        "hsc_register_group": (C.c_int, [_p, C.c_char_p, C.c_int, C.c_int]),
        "hsc_window_ingest_device": (C.c_int, [_p, C.c_size_t, C.c_int, _p, _p, _p, C.c_uint64]),
        "hsc_window_words": (C.c_int, [_p]),
        "hsc_window_code_words": (C.c_int, [_p]),
        "hsc_window_tile_key_words": (C.c_int, [_p]),
        "hsc_window_keys": (C.c_size_t, [_p]),
        "hsc_window_end": (C.c_uint64, [_p]),
        "hsc_window_max_commit": (C.c_uint64, [_p]),
        "hsc_window_export": (C.c_long, [_p, C.c_int, _p, _p, _p, C.c_size_t]),
        "hsc_set_fold": (C.c_int, [_p, C.c_size_t, C.c_int]),
        "hsc_fold_stats": (C.c_int, [_p, _p]),
        "hsc_append_stats": (C.c_int, [_p, _p]),
        "hsc_set_paths": (C.c_int, [_p, C.c_uint]),
        "hsc_window_sort_path": (C.c_int, [_p]),
        "hsc_table_id": (C.c_int, [_p, C.c_char_p]),
        "hsc_table_name": (C.c_char_p, [_p, C.c_int]),
        "hsc_group_info": (C.c_int, [_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int)]),
        "hsc_table_max": (C.c_int, [_p, _p, C.c_int]),
        "hsc_merge_table_max": (C.c_int, [_p, _p, C.c_int]),
        "hip_bdb_osql_serial_check": (C.c_int, [_p, _p, C.POINTER(C.c_uint), C.POINTER(C.c_uint), C.c_int]),
        "hip_serial_check_batch": (C.c_int, [_p, C.POINTER(_p), C.POINTER(C.c_uint),
                                             C.POINTER(C.c_uint), C.c_int, C.c_int,
                                             C.POINTER(C.c_int)]),
        "hsc_check_readsets": (C.c_int, [_p, C.POINTER(_ReadSets), C.POINTER(C.c_int)]),
        "hsc_marshal_readsets": (C.c_int, [_p, C.POINTER(_ReadSets), C.POINTER(C.POINTER(Marshalled))]),
        "hsc_probe_device": (C.c_int, [_p, C.POINTER(ProbeBatch)]),
        "hsc_pack_verdicts": (C.c_int, [_p, _p, C.c_size_t, _p]),
        "hsc_or_bitmaps": (C.c_int, [_p, _p, C.c_int, C.c_size_t, _p]),
        "hsc_synchronize": (C.c_int, [_p]),
        "hsc_get_timing": (C.c_int, [_p, C.POINTER(Timing)]),
        "hsc_enable_timing": (C.c_int, [_p, C.c_int]),
        "hsc_dep_graph_scc": (C.c_int, [_p, C.POINTER(_History), _p, C.POINTER(GraphStats)]),
        "hsc_dep_graph_edges": (C.c_int, [_p, _p, _p, _p, C.c_size_t, C.POINTER(C.c_size_t)]),
        "hsc_dep_graph_build": (C.c_int, [_p, C.POINTER(_History), C.c_int, C.POINTER(GraphStats)]),
        "hsc_dep_graph_cover": (C.c_int, [_p, _p]),
        "hsc_dep_graph_stage_rw_pairs": (C.c_int, [_p, C.c_uint32, _p, C.c_size_t, _p, _p]),
        "hsc_dep_graph_scc_built": (C.c_int, [_p, _p, C.POINTER(GraphStats)]),
        "hsc_dep_graph_build_device": (C.c_int, [_p, C.c_size_t, C.c_uint32, _p, _p, _p, _p,
                                                 C.c_int, C.POINTER(GraphStats)]),
        "hsc_dep_graph_cut": (C.c_int, [_p, _p, _p, C.c_size_t, C.POINTER(C.c_size_t)]),
        "hsc_dep_graph_scc_cut": (C.c_int, [_p, C.c_uint32, _p, _p, C.c_size_t, _p,
                                            C.POINTER(GraphStats)]),
        "hsc_window_ingest_raw": (C.c_int, [_p, C.POINTER(_RawLog)]),
        "hsc_decode_log": (C.c_int, [_p, C.POINTER(_RawLog), C.POINTER(C.POINTER(_LLog))]),
        "hsc_decode_serial": (C.c_int, [_p, C.POINTER(_SerialMsgs),
                                        C.POINTER(C.POINTER(_ReadSets))]),
        "hsc_check_serial": (C.c_int, [_p, C.POINTER(_SerialMsgs), C.POINTER(C.c_int)]),
        "hsc_set_layout": (C.c_int, [_p, C.c_int]),
        "hsc_set_threads": (C.c_int, [_p, C.c_int]),
        "hsc_window_append_log": (C.c_int, [_p, C.POINTER(_LLog)]),
        "hsc_window_append_raw": (C.c_int, [_p, C.POINTER(_RawLog)]),
        "hsc_window_delta_rows": (C.c_size_t, [_p]),
        "hsc_currangearrs_build": (C.c_int, [C.POINTER(_ReadSets), C.POINTER(C.POINTER(_p))]),
        "hsc_currangearrs_free": (None, [C.POINTER(_p), C.c_int]),
        "hsc_collector_create": (C.c_int, [_p, C.c_int, C.c_int, C.POINTER(_p)]),
        "hsc_collector_destroy": (None, [_p]),
        "hsc_collector_check": (C.c_int, [_p, _p, C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                          C.c_int]),
        "hsc_collector_get_stats": (C.c_int, [_p, C.POINTER(CollectorStats)]),
        "hsc_collector_set_inflight": (C.c_int, [_p, C.c_int]),
        "hsc_set_autocollect": (C.c_int, [_p, C.c_int]),
        "hsc_small_stats": (C.c_int, [_p, C.POINTER(SmallStats)]),
        "hsc_harness_concurrent": (C.c_int, [_p, _p, C.POINTER(_p), C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.POINTER(C.c_int),
                                             C.POINTER(ConcurrentResult)]),
        "hsc_regop_stats": (C.c_int, [_p, _p]),
        "hsc_harness_commit_protocol": (C.c_int, [_p, _p, C.c_int, _p, C.c_int, C.c_int, _p, _p,
                                                  _p, _p, C.POINTER(ProtocolResult)]),
        "hsc_window_layout": (C.c_int, [_p]),
        "hsc_batch_stats": (C.c_int, [_p, C.POINTER(BatchStats)]),
        "hsc_marshal_arrs": (C.c_int, [_p, C.POINTER(_p), _p, C.c_int,
                                       C.POINTER(C.POINTER(Marshalled))]),
        "hsc_multi_create": (C.c_int, [C.POINTER(C.c_int), C.c_int, ctx_pp]),
        "hsc_multi_unique_ids": (C.c_int, [_p, C.c_size_t]),
        "hsc_multi_create_rank": (C.c_int, [C.c_int, C.c_int, C.c_int, _p, C.c_size_t, ctx_pp]),
        "hsc_multi_world": (C.c_int, [_p]),
        "hsc_multi_rank": (C.c_int, [_p]),
        "hsc_multi_local": (C.c_int, [_p]),
        "hsc_multi_member": (_p, [_p, C.c_int]),
        "hsc_multi_set_splitters": (C.c_int, [_p, C.c_size_t, _p, _p, C.c_int]),
        "hsc_multi_adopt": (C.c_int, [_p]),
        "hsc_multi_probe_device": (C.c_int, [_p, _p, C.c_int]),
        "hsc_multi_stats": (C.c_int, [_p, _p]),
        "hsc_multi_last_counts": (C.c_int, [_p, _p, C.c_int]),
        "hsc_multi_phase_stats": (C.c_int, [_p, _p]),
        "hsc_multi_routed_phase_stats": (C.c_int, [_p, _p]),
        "hsc_multi_set_mode": (C.c_int, [_p, C.c_int]),
        "hsc_multi_mode": (C.c_int, [_p]),
        "hsc_multi_set_transport": (C.c_int, [_p, C.c_int]),
        "hsc_multi_probe_routed": (C.c_int, [_p, _p, _p, C.c_int]),
        "hsc_multi_marshal_routed": (C.c_int, [_p, C.POINTER(_ReadSets), C.c_int, C.c_uint32,
                                               C.POINTER(C.POINTER(Marshalled))]),
        "hsc_multi_route_stats": (C.c_int, [_p, _p]),
        "hsc_multi_graph_scc": (C.c_int, [_p, _p, C.c_uint32, _p, C.POINTER(GraphStats)]),
        "hsc_multi_graph_phase_ms": (C.c_int, [_p, _p]),
        "hsc_multi_routed_member": (C.c_int, [_p, C.c_int, C.POINTER(C.POINTER(Marshalled))]),
        "hsc_multi_enable_timing": (C.c_int, [_p, C.c_int]),
        "hsc_multi_member_probe_ms": (C.c_int, [_p, _p, C.c_int]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name) and os.environ.get("HSC_LIB"):
            continue  # A/B build of an older library: bind what it has
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _names(tbnames: Sequence[str]):
    arr = (C.c_char_p * max(1, len(tbnames)))()
    for i, n in enumerate(tbnames):
        arr[i] = n.encode()
    return arr


def llog_struct(log: LLog):
    """(struct, keepalive) for an LLog."""
    cols = dict(lsn=np.ascontiguousarray(log.lsn, np.uint64),
                rectype=np.ascontiguousarray(log.rectype, np.uint32),
                prev=np.ascontiguousarray(log.prev, np.uint64),
                isabort=np.ascontiguousarray(log.isabort, np.int16),
                table=np.ascontiguousarray(log.table, np.int32),
                ix=np.ascontiguousarray(log.ix, np.int16),
                key_off=np.ascontiguousarray(log.key_off, np.uint64),
                keylen=np.ascontiguousarray(log.keylen, np.int32),
                keys=np.ascontiguousarray(log.keys, np.uint8))
    names = _names(log.tbnames)
    s = _LLog(log.nrec, *[_ptr(cols[k]) for k in ("lsn", "rectype", "prev", "isabort", "table",
                                                  "ix", "key_off", "keylen", "keys")],
              names, len(log.tbnames), int(log.end_lsn))
    return s, (cols, names)


def rawlog_struct(raw):
    cols = [np.ascontiguousarray(raw.lsn, np.uint64), np.ascontiguousarray(raw.off, np.uint64),
            np.ascontiguousarray(raw.len, np.uint32), np.ascontiguousarray(raw.buf, np.uint8),
            np.ascontiguousarray(raw.recon_lsn, np.uint64),
            np.ascontiguousarray(raw.recon_off, np.uint64),
            np.ascontiguousarray(raw.recon_len, np.int32),
            np.ascontiguousarray(raw.recon_keys, np.uint8)]
    s = _RawLog(len(cols[0]), *[_ptr(c) for c in cols[:4]], int(raw.end_lsn), len(cols[4]),
                *[_ptr(c) for c in cols[4:]])
    return s, cols


def readsets_struct(rs: ReadSets):
    cols = dict(txn_off=np.ascontiguousarray(rs.txn_off, np.int64),
                snap=np.ascontiguousarray(rs.snap, np.uint64),
                table=np.ascontiguousarray(rs.table, np.int32),
                idxnum=np.ascontiguousarray(rs.idxnum, np.int32),
                lflag=np.ascontiguousarray(rs.lflag, np.int32),
                rflag=np.ascontiguousarray(rs.rflag, np.int32),
                islocked=np.ascontiguousarray(rs.islocked, np.int32),
                lkeylen=np.ascontiguousarray(rs.lkeylen, np.int32),
                rkeylen=np.ascontiguousarray(rs.rkeylen, np.int32),
                lkey_off=np.ascontiguousarray(rs.lkey_off, np.uint64),
                rkey_off=np.ascontiguousarray(rs.rkey_off, np.uint64),
                keys=np.ascontiguousarray(rs.keys, np.uint8))
    names = _names(rs.tbnames)
    order = ("txn_off", "snap", "table", "idxnum", "lflag", "rflag", "islocked", "lkeylen",
             "rkeylen", "lkey_off", "rkey_off", "keys")
    s = _ReadSets(rs.ntxn, *[_ptr(cols[k]) for k in order], names, len(rs.tbnames))
    return s, (cols, names)


class _Coalesced(C.Structure):
    _fields_ = [("ntxn", C.c_int), ("txn_off", _p), ("table", _p), ("idxnum", _p),
                ("lflag", _p), ("rflag", _p), ("islocked", _p), ("lkeylen", _p),
                ("rkeylen", _p), ("lkey_off", _p), ("rkey_off", _p)]


class CurRangeArrays:
    """Heap-style CurRangeArr objects (ctypes) built from Python ranges, kept
    alive together; what a comdb2 caller would pass to the drop-in entry."""

    def __init__(self, sets: Sequence[Sequence[Range]], snaps: Sequence[int]):
        self._keep: list = []
        self.arrs: List[CurRangeArr] = []
        for rs, s in zip(sets, snaps):
            ptrs = (C.POINTER(CurRange) * max(2, len(rs)))()
            for i, r in enumerate(rs):
                cr = CurRange()
                nm = C.create_string_buffer(r.tbname.encode())
                cr.tbname = C.cast(nm, C.c_char_p)
                cr.idxnum = r.idxnum
                for side, k in (("l", r.lkey), ("r", r.rkey)):
                    if k is None:
                        setattr(cr, side + "key", None)
                        setattr(cr, side + "keylen", 0)
                    else:
                        b = C.create_string_buffer(bytes(k), max(1, len(k)))
                        self._keep.append(b)
                        setattr(cr, side + "key", C.cast(b, _p))
                        setattr(cr, side + "keylen", len(k))
                cr.lflag, cr.rflag, cr.islocked = r.lflag, r.rflag, r.islocked
                self._keep += [nm, cr]
                ptrs[i] = C.pointer(cr)
            a = CurRangeArr(len(rs), max(2, len(rs)), int(s) >> 32, int(s) & 0xFFFFFFFF, None,
                            ptrs)
            self._keep.append(ptrs)
            self.arrs.append(a)

    def pointers(self):
        arr = (_p * max(1, len(self.arrs)))()
        for i, a in enumerate(self.arrs):
            arr[i] = C.cast(C.pointer(a), _p)
        return arr


class NativeCurRangeArrs:
    """CurRangeArr objects built by the library's harness helper
    (hsc_currangearrs_build) from flat read sets: heap CurRange's with
    strdup'd names and malloc'd keys, as a comdb2 master holds them.  Much
    faster than :class:`CurRangeArrays` for large batches."""

    def __init__(self, rs: ReadSets):
        self.lib = load()
        s, keep = readsets_struct(rs)
        out = C.POINTER(_p)()
        rc = self.lib.hsc_currangearrs_build(C.byref(s), C.byref(out))
        if rc != HSC_OK:
            raise HscError(f"hsc_currangearrs_build -> {rc}")
        self.ptrs, self.n = out, rs.ntxn

    def pointers(self):
        return self.ptrs

    def close(self):
        if self.ptrs:
            self.lib.hsc_currangearrs_free(self.ptrs, self.n)
            self.ptrs = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Validator:
    """One GPU's validator context (hsc_ctx).  device=-1: host-only context
    (log decode, dictionaries and marshalling; no checks)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        if device != -1 and self.lib.hsc_device_count() <= device:
            raise HscError(f"no HIP device {device} visible")
        ctx = _p()
        rc = self.lib.hsc_ctx_create(device, C.byref(ctx))
        if rc != HSC_OK:
            raise HscError(f"hsc_ctx_create({device}) = {rc}")
        self.ctx = ctx
        self._keep = None

    def close(self) -> None:
        if self.ctx:
            self.lib.hsc_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int, what: str) -> None:
        if rc != HSC_OK:
            msg = self.lib.hsc_last_error(self.ctx)
            raise HscError(f"{what} -> {rc}: {msg.decode() if msg else ''}")

    # window
    def ingest_log(self, log: LLog) -> None:
        s, keep = llog_struct(log)
        self._chk(self.lib.hsc_window_ingest_log(self.ctx, C.byref(s)), "hsc_window_ingest_log")

    def append_log(self, log: LLog) -> None:
        """Append the continuation of the window's log (hsc_window_append_log)."""
        s, keep = llog_struct(log)
        self._chk(self.lib.hsc_window_append_log(self.ctx, C.byref(s)), "hsc_window_append_log")

    def append_raw(self, raw) -> None:
        """Append raw log records (hsc_window_append_raw)."""
        s, keep = rawlog_struct(raw)
        self._chk(self.lib.hsc_window_append_raw(self.ctx, C.byref(s)), "hsc_window_append_raw")

    def append_writes(self, writes, end_lsn: Optional[int] = None) -> None:
        """hsc_window_append of decoded writes [(tbname, idxnum, key or None,
        commit_lsn)], then hsc_window_set_end(end_lsn) if given."""
        n = len(writes)
        arr = (_Write * max(1, n))()
        keep = []
        for i, (tb, ix, key, lsn_) in enumerate(writes):
            nm = C.create_string_buffer(tb.encode())
            keep.append(nm)
            arr[i].tbname = C.cast(nm, C.c_char_p)
            arr[i].idxnum = ix
            if key is None:
                arr[i].key = None
                arr[i].keylen = 0
            else:
                kb = C.create_string_buffer(bytes(key), max(1, len(key)))
                keep.append(kb)
                arr[i].key = C.cast(kb, _p)
                arr[i].keylen = len(key)
            arr[i].commit_lsn = int(lsn_)
        self._chk(self.lib.hsc_window_append(self.ctx, arr, n), "hsc_window_append")
        if end_lsn is not None:
            self._chk(self.lib.hsc_window_set_end(self.ctx, int(end_lsn)), "hsc_window_set_end")

    def set_end(self, end_lsn: int) -> None:
        """hsc_window_set_end: the log's end LSN (curlsn of full checks)."""
        self._chk(self.lib.hsc_window_set_end(self.ctx, int(end_lsn)), "hsc_window_set_end")

    @property
    def delta_rows(self) -> int:
        return self.lib.hsc_window_delta_rows(self.ctx)

    def ingest_raw(self, raw) -> None:
        """Decode a raw log stream (formats.RawLog) and ingest it."""
        s, keep = rawlog_struct(raw)
        self._chk(self.lib.hsc_window_ingest_raw(self.ctx, C.byref(s)), "hsc_window_ingest_raw")

    def decode_raw(self, raw) -> LLog:
        """Decode only; returns the decoded stream as an LLog (copies)."""
        s, keep = rawlog_struct(raw)
        out = C.POINTER(_LLog)()
        self._chk(self.lib.hsc_decode_log(self.ctx, C.byref(s), C.byref(out)), "hsc_decode_log")
        L = out.contents
        n = L.nrec

        def arr(p, cnt, dt):
            if cnt == 0 or not p:
                return np.zeros(cnt, dtype=dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(cnt,)).copy()
        keylen = arr(L.keylen, n, np.int32)
        key_off = arr(L.key_off, n, np.uint64)
        nkeys = int(max([int(key_off[i]) + int(keylen[i]) for i in range(n)] + [1]))
        return LLog(lsn=arr(L.lsn, n, np.uint64), rectype=arr(L.rectype, n, np.uint32),
                    prev=arr(L.prev, n, np.uint64), isabort=arr(L.isabort, n, np.int16),
                    table=arr(L.table, n, np.int32), ix=arr(L.ix, n, np.int16), key_off=key_off,
                    keylen=keylen, keys=arr(L.keys, nkeys, np.uint8),
                    tbnames=[L.tbnames[i].decode("utf-8", "surrogateescape") for i in range(L.ntbnames)],
                    end_lsn=int(L.end_lsn))

    def decode_serial(self, msgs) -> ReadSets:
        """Decode OSQL_SERIAL payloads (buf, off, len) to ReadSets (copies)."""
        buf, off, ln = [np.ascontiguousarray(a, dt) for a, dt in
                        zip(msgs, (np.uint8, np.uint64, np.uint64))]
        s = _SerialMsgs(len(off), _ptr(buf), _ptr(off), _ptr(ln))
        out = C.POINTER(_ReadSets)()
        self._chk(self.lib.hsc_decode_serial(self.ctx, C.byref(s), C.byref(out)),
                  "hsc_decode_serial")
        R = out.contents
        nt = R.ntxn

        def arr(p, cnt, dt):
            if cnt == 0 or not p:
                return np.zeros(cnt, dtype=dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(cnt,)).copy()
        txn_off = arr(R.txn_off, nt + 1, np.int64)
        nr = int(txn_off[-1]) if nt else 0
        cols = {k: arr(getattr(R, k), nr, np.int32) for k in
                ("table", "idxnum", "lflag", "rflag", "islocked", "lkeylen", "rkeylen")}
        lo, ro = arr(R.lkey_off, nr, np.uint64), arr(R.rkey_off, nr, np.uint64)
        nk = int(max([int(lo[i]) + int(cols["lkeylen"][i]) for i in range(nr) if lo[i] != KEY_NULL] +
                     [int(ro[i]) + int(cols["rkeylen"][i]) for i in range(nr) if ro[i] != KEY_NULL] +
                     [1]))
        return ReadSets(txn_off=txn_off, snap=arr(R.snap, nt, np.uint64), lkey_off=lo,
                        rkey_off=ro, keys=arr(R.keys, nk, np.uint8),
                        tbnames=[R.tbnames[i].decode("utf-8", "surrogateescape") for i in range(R.ntbnames)], **cols)

    def check_serial(self, msgs) -> np.ndarray:
        """Decode + full check of OSQL_SERIAL payloads; rc per message."""
        buf, off, ln = [np.ascontiguousarray(a, dt) for a, dt in
                        zip(msgs, (np.uint8, np.uint64, np.uint64))]
        s = _SerialMsgs(len(off), _ptr(buf), _ptr(off), _ptr(ln))
        out = np.zeros(max(1, len(off)), dtype=np.int32)
        self._chk(self.lib.hsc_check_serial(self.ctx, C.byref(s),
                                            out.ctypes.data_as(C.POINTER(C.c_int))),
                  "hsc_check_serial")
        return out[: len(off)]

    def register_group(self, tbname: str, idxnum: int, keylen: int) -> int:
        g = self.lib.hsc_register_group(self.ctx, tbname.encode(), idxnum, keylen)
        if g < 0:
            self._chk(g, "hsc_register_group")
        return g

    def ingest_device(self, n: int, words: int, gid_ptr: int, words_ptr: int, lsn_ptr: int,
                      end_lsn: int) -> None:
        self._chk(self.lib.hsc_window_ingest_device(self.ctx, n, words, gid_ptr, words_ptr,
                                                    lsn_ptr, end_lsn), "hsc_window_ingest_device")

    @property
    def words(self) -> int:
        return self.lib.hsc_window_words(self.ctx)

    def set_layout(self, layout: int) -> None:
        """LAYOUT_AUTO (narrow tiles when the window fits them) or LAYOUT_WIDE."""
        self._chk(self.lib.hsc_set_layout(self.ctx, layout), "hsc_set_layout")

    @property
    def layout(self) -> int:
        """LAYOUT_NARROW, LAYOUT_COMPACT or LAYOUT_WIDE: the current window's."""
        return self.lib.hsc_window_layout(self.ctx)

    @property
    def sort_path(self) -> str:
        """How the last build sorted its rows: "radix", "packed" or "codes"."""
        return ("radix", "packed", "codes")[self.lib.hsc_window_sort_path(self.ctx)]

    @property
    def code_words(self) -> int:
        """Words per probed window row (compact codes: WC < words)."""
        return self.lib.hsc_window_code_words(self.ctx)

    @property
    def tile_key_words(self) -> int:
        """Compact windows: words of the compact-tile keys gid || code that
        batches probe (hsc_ctiles.hip); 0 when the window has none."""
        return self.lib.hsc_window_tile_key_words(self.ctx)

    @property
    def keys(self) -> int:
        return self.lib.hsc_window_keys(self.ctx)

    @property
    def end_lsn(self) -> int:
        return self.lib.hsc_window_end(self.ctx)

    def set_fold(self, rows: int = 0, background: bool = True) -> None:
        """Fold the delta run into the main window at `rows` rows (0: default),
        in the background or inline in the next check (hsc_set_fold)."""
        self._chk(self.lib.hsc_set_fold(self.ctx, rows, int(background)), "hsc_set_fold")

    def fold_stats(self) -> dict:
        out = np.zeros(4, np.uint64)
        self._chk(self.lib.hsc_fold_stats(self.ctx, out.ctypes.data), "hsc_fold_stats")
        return {"started": int(out[0]), "swapped": int(out[1]), "inline": int(out[2]),
                "last_fold_us": int(out[3])}

    def set_paths(self, flags: int) -> None:
        """Restrict the context's paths (PATH_* flags; 0 = automatic):
        hsc_set_paths, for tests and A/B runs."""
        self._chk(self.lib.hsc_set_paths(self.ctx, int(flags)), "hsc_set_paths")

    def append_stats(self) -> dict:
        """Appends kept in the pending tail, merges of the tail into the
        delta run, rows waiting now (hsc_append_stats)."""
        out = np.zeros(3, np.uint64)
        self._chk(self.lib.hsc_append_stats(self.ctx, out.ctypes.data), "hsc_append_stats")
        return {"pending_appends": int(out[0]), "pending_merges": int(out[1]),
                "pending_rows": int(out[2])}

    def export_window(self, all_versions: bool = False):
        """(gid u32[n], words u64[W, n], lsn u64[n]) of the built window in
        (group, key) order: the newest version per key, or every version
        (hsc_window_export; the delta run is folded in first)."""
        n = self.lib.hsc_window_export(self.ctx, int(all_versions), None, None, None, 0)
        self._chk(min(int(n), 0), "hsc_window_export")
        W = self.words
        gid = np.zeros(max(n, 1), np.uint32)
        words = np.zeros((W, max(n, 1)), np.uint64)
        lsn = np.zeros(max(n, 1), np.uint64)
        if n:
            m = self.lib.hsc_window_export(self.ctx, int(all_versions), gid.ctypes.data,
                                           words.ctypes.data, lsn.ctypes.data, n)
            self._chk(min(int(m), 0), "hsc_window_export")
            assert m == n
        return gid[:n], words[:, :n], lsn[:n]

    # checks
    def check_readsets(self, rs: ReadSets) -> np.ndarray:
        s, keep = readsets_struct(rs)
        out = np.zeros(max(1, rs.ntxn), dtype=np.int32)
        rc = self.lib.hsc_check_readsets(self.ctx, C.byref(s), out.ctypes.data_as(C.POINTER(C.c_int)))
        self._chk(rc, "hsc_check_readsets")
        return out[: rs.ntxn]

    def set_threads(self, n: int) -> None:
        """Host threads of the marshal (0: the box's CPUs)."""
        self._chk(self.lib.hsc_set_threads(self.ctx, n), "hsc_set_threads")

    def check_batch(self, arrs, regop_only: int = 0, file: Optional[np.ndarray] = None,
                    offset: Optional[np.ndarray] = None) -> np.ndarray:
        """hip_serial_check_batch over CurRangeArrays / NativeCurRangeArrs.
        file / offset: uint32[n] in/out snapshot LSNs (None: each array's own
        file / offset, updated in place)."""
        n = len(arrs.arrs) if hasattr(arrs, "arrs") else arrs.n
        out = np.zeros(max(1, n), dtype=np.int32)
        u32p = C.POINTER(C.c_uint)
        fp = file.ctypes.data_as(u32p) if file is not None else None
        op = offset.ctypes.data_as(u32p) if offset is not None else None
        rc = self.lib.hip_serial_check_batch(self.ctx, arrs.pointers(), fp, op, regop_only, n,
                                             out.ctypes.data_as(C.POINTER(C.c_int)))
        self._chk(rc, "hip_serial_check_batch")
        return out[:n]

    def batch_stats(self) -> dict:
        """Marshal / batch phase totals (hsc_batch_stats), in ms and counts."""
        st = BatchStats()
        self._chk(self.lib.hsc_batch_stats(self.ctx, C.byref(st)), "hsc_batch_stats")
        d = {k: getattr(st, k) for k, _ in BatchStats._fields_}
        return {k: (v / 1e6 if k.endswith("_ns") else v) for k, v in d.items()}

    def small_stats(self) -> dict:
        """Small-batch path phase totals (hsc_small_stats): calls and the mean
        host marshal, slot launch and done-word wait per call (us), and the
        mean wait for the context lock per hip_serial_check_batch call."""
        st = SmallStats()
        self._chk(self.lib.hsc_small_stats(self.ctx, C.byref(st)), "hsc_small_stats")
        n = max(1, st.calls)
        return {"calls": st.calls, "marshal_us": st.marshal_ns / 1e3 / n,
                "launch_us": st.launch_ns / 1e3 / n, "wait_us": st.wait_ns / 1e3 / n,
                "slot_waits": st.slot_waits, "lock_us": st.lock_ns / 1e3 / n}

    def regop_stats(self) -> dict:
        """regop_only probes answered from the published snapshot / locked."""
        out = np.zeros(2, np.uint64)
        self._chk(self.lib.hsc_regop_stats(self.ctx, out.ctypes.data), "hsc_regop_stats")
        return {"fast": int(out[0]), "locked": int(out[1])}

    def commit_protocol(self, txns, events, nthreads: int):
        """db/toblock.c:4757-4836 replayed natively (hsc_harness_commit_protocol)
        by nthreads threads over events [('begin' | 'commit', workloads.Txn)]:
        snapshots taken at begin, commits through the commit_lock protocol
        (regop probe under the write lock, full check outside it, append).
        -> (rc int32[n], commit_seq int64[n], snap u64[n], check_end u64[n],
        stats dict); txns indexed as in `txns`."""
        from .formats import DTA_TYPES
        n = len(txns)
        idx = {t.name: i for i, t in enumerate(txns)}
        rs = ReadSets.from_lists([t.reads for t in txns], [0] * n)
        arrs = NativeCurRangeArrs(rs)
        keep = []
        pt = (ProtocolTxn * max(1, n))()
        ptrs = arrs.pointers()
        for i, t in enumerate(txns):
            ws = (_Write * max(1, len(t.writes)))()
            for j, (rt, tb, ix, key) in enumerate(t.writes):
                nm = C.create_string_buffer(tb.encode())
                dta = rt in DTA_TYPES or key is None
                kb = None if dta else C.create_string_buffer(bytes(key), max(1, len(key)))
                keep += [nm, kb]
                ws[j].tbname = C.cast(nm, C.c_char_p)
                ws[j].idxnum = -2 if dta else ix
                ws[j].key = None if dta else C.cast(kb, _p)
                ws[j].keylen = 0 if dta else len(key)
            keep.append(ws)
            pt[i].arr = ptrs[i]
            pt[i].writes = C.cast(ws, _p)
            pt[i].nwrites = len(t.writes)
        ev = np.array([idx[t.name] if e == "begin" else ~idx[t.name] for e, t in events], np.int32)
        rc = np.zeros(max(1, n), np.int32)
        seq = np.zeros(max(1, n), np.int64)
        snap = np.zeros(max(1, n), np.uint64)
        cend = np.zeros(max(1, n), np.uint64)
        res = ProtocolResult()
        r0 = self.regop_stats()
        try:
            self._chk(self.lib.hsc_harness_commit_protocol(
                self.ctx, pt, n, ev.ctypes.data, len(ev), nthreads, rc.ctypes.data, seq.ctypes.data,
                snap.ctypes.data, cend.ctypes.data, C.byref(res)), "hsc_harness_commit_protocol")
        finally:
            arrs.close()
        r1 = self.regop_stats()
        st = {k: getattr(res, k) for k, _ in ProtocolResult._fields_}
        st["threads"] = nthreads
        sec = max(res.seconds, 1e-9)
        st["commits_per_s"] = (res.commits + res.aborts) / sec  # commit attempts (checked txns)
        st["committed_per_s"] = res.commits / sec
        st["regop_fast"] = r1["fast"] - r0["fast"]
        st["regop_locked"] = r1["locked"] - r0["locked"]
        return rc[:n], seq[:n], snap[:n], cend[:n], st

    def concurrent_check(self, arrs, nthreads: int, rounds: int = 1, regop_only: int = 0,
                         collect: bool = True, max_batch: int = 0, max_wait_us: int = 0,
                         inflight: int = 0):
        """nthreads native caller threads checking arrs concurrently
        (hsc_harness_concurrent), each call one read set through a batching
        collector (hsc_collector_check) or, collect=False, one
        hip_bdb_osql_serial_check per call.  -> (verdicts int32[n], stats dict)."""
        n = len(arrs.arrs) if hasattr(arrs, "arrs") else arrs.n
        out = np.zeros(max(1, n), dtype=np.int32)
        col = _p()
        if collect:
            self._chk(self.lib.hsc_collector_create(self.ctx, max_batch, max_wait_us,
                                                    C.byref(col)), "hsc_collector_create")
            if inflight:
                self._chk(self.lib.hsc_collector_set_inflight(col, inflight),
                          "hsc_collector_set_inflight")
        res = ConcurrentResult()
        sm0 = SmallStats()
        self._chk(self.lib.hsc_small_stats(self.ctx, C.byref(sm0)), "hsc_small_stats")
        try:
            rc = self.lib.hsc_harness_concurrent(self.ctx, col, arrs.pointers(), n, nthreads,
                                                 rounds, regop_only,
                                                 out.ctypes.data_as(C.POINTER(C.c_int)),
                                                 C.byref(res))
            self._chk(rc, "hsc_harness_concurrent")
            st = {"threads": nthreads, "calls": res.calls, "seconds": res.seconds,
                  "checks_per_s": res.calls / res.seconds if res.seconds > 0 else 0.0,
                  "lat_mean_us": res.lat_mean_us, "lat_p50_us": res.lat_p50_us,
                  "lat_p99_us": res.lat_p99_us, "collector": bool(collect)}
            if collect:
                cs = CollectorStats()
                self._chk(self.lib.hsc_collector_get_stats(col, C.byref(cs)),
                          "hsc_collector_get_stats")
                st.update(batches=cs.batches, max_batch=cs.max_batch,
                          mean_batch=cs.calls / max(1, cs.batches),
                          device_pass_us=cs.pass_ns / 1e3 / max(1, cs.batches),
                          busy_frac=cs.busy_ns / 1e9 / max(res.seconds, 1e-9),
                          gate_us=cs.gate_ns / 1e3 / max(1, cs.batches),
                          handout_us=cs.handout_ns / 1e3 / max(1, cs.batches))
            sm = SmallStats()
            self._chk(self.lib.hsc_small_stats(self.ctx, C.byref(sm)), "hsc_small_stats")
            k = sm.calls - sm0.calls
            if k:  # device passes that took the small-batch path: mean phase times
                st["small_path"] = {"passes": k,
                                    "marshal_us": (sm.marshal_ns - sm0.marshal_ns) / 1e3 / k,
                                    "launch_us": (sm.launch_ns - sm0.launch_ns) / 1e3 / k,
                                    "wait_us": (sm.wait_ns - sm0.wait_ns) / 1e3 / k,
                                    "slot_waits": sm.slot_waits - sm0.slot_waits,
                                    "lock_us": (sm.lock_ns - sm0.lock_ns) / 1e3 / k}
        finally:
            if collect:
                self.lib.hsc_collector_destroy(col)
        return out[:n], st

    def rw_edges(self, rs: ReadSets):
        """(txn uint32[k], writer commit LSN uint64[k]): every (read set,
        writer) pair of the A0 join before its OR-reduction, sorted, unique
        (hsc_rw_edges; range probes only)."""
        s, keep = readsets_struct(rs)
        n = C.c_size_t()
        t = C.c_void_p()
        w = C.c_void_p()
        self._chk(self.lib.hsc_rw_edges(self.ctx, C.byref(s), C.byref(n), C.byref(t), C.byref(w)),
                  "hsc_rw_edges")
        k = n.value
        if k == 0:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint64)
        txn = np.ctypeslib.as_array(C.cast(t, C.POINTER(C.c_uint32)), shape=(k,)).copy()
        lsn = np.ctypeslib.as_array(C.cast(w, C.POINTER(C.c_uint64)), shape=(k,)).copy()
        return txn, lsn

    def coalesce(self, rs: ReadSets) -> ReadSets:
        """currangearr_coalesce (db/sqlglue.c:305-311) of every read set on the
        device; the result keeps rs.keys (its key offsets point into it)."""
        import dataclasses
        s, keep = readsets_struct(rs)
        out = _Coalesced()
        self._chk(self.lib.hsc_coalesce_readsets(self.ctx, C.byref(s), C.byref(out)),
                  "hsc_coalesce_readsets")
        T = out.ntxn
        off = np.ctypeslib.as_array(C.cast(out.txn_off, C.POINTER(C.c_int64)), shape=(T + 1,)).copy()
        n = int(off[-1])

        def arr(p, ct, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(n,)).astype(dt, copy=True)

        i32 = lambda p: arr(p, C.c_int32, np.int32)
        return dataclasses.replace(
            rs, txn_off=off, table=i32(out.table), idxnum=i32(out.idxnum), lflag=i32(out.lflag),
            rflag=i32(out.rflag), islocked=i32(out.islocked), lkeylen=i32(out.lkeylen),
            rkeylen=i32(out.rkeylen), lkey_off=arr(out.lkey_off, C.c_uint64, np.uint64),
            rkey_off=arr(out.rkey_off, C.c_uint64, np.uint64))

    def marshal_arrs(self, arrs, snaps, copy: bool = True):
        """hsc_marshal_arrs over NativeCurRangeArrs / CurRangeArrays (the host
        half of hip_serial_check_batch); copy=False returns only the counts."""
        n = len(arrs.arrs) if hasattr(arrs, "arrs") else arrs.n
        sn = np.ascontiguousarray(snaps, np.uint64)
        mp = C.POINTER(Marshalled)()
        self._chk(self.lib.hsc_marshal_arrs(self.ctx, arrs.pointers(), sn.ctypes.data, n,
                                            C.byref(mp)), "hsc_marshal_arrs")
        return self._marshalled(mp.contents) if copy else (mp.contents.n, mp.contents.n_lock)

    def marshal(self, rs: ReadSets) -> dict:
        """Marshal read sets into probe SoA (numpy copies)."""
        s, keep = readsets_struct(rs)
        mp = C.POINTER(Marshalled)()
        self._chk(self.lib.hsc_marshal_readsets(self.ctx, C.byref(s), C.byref(mp)),
                  "hsc_marshal_readsets")
        return self._marshalled(mp.contents)

    @staticmethod
    def _marshalled(m) -> dict:
        W, n, nl, nt = m.words, m.n, m.n_lock, m.n_txn

        def arr(p, cnt, dt):
            if cnt == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(p, shape=(cnt,)).astype(dt, copy=True)

        return dict(words=W, n=n, n_lock=nl, n_txn=nt,
                    lo=arr(m.lo, W * n, np.uint64).reshape(W, n) if n else np.zeros((W, 0), np.uint64),
                    hi=arr(m.hi, W * n, np.uint64).reshape(W, n) if n else np.zeros((W, 0), np.uint64),
                    gid=arr(m.gid, n, np.uint32), snap=arr(m.snap, n, np.uint64),
                    txn=arr(m.txn, n, np.uint32), lock_table=arr(m.lock_table, nl, np.uint32),
                    lock_snap=arr(m.lock_snap, nl, np.uint64), lock_txn=arr(m.lock_txn, nl, np.uint32),
                    forced=arr(m.forced, nt, np.uint8))

    def group_info(self, gid: int):
        t, ix, kl = C.c_int(), C.c_int(), C.c_int()
        self._chk(self.lib.hsc_group_info(self.ctx, gid, C.byref(t), C.byref(ix), C.byref(kl)),
                  "hsc_group_info")
        return t.value, ix.value, kl.value

    def table_name(self, tid: int):
        r = self.lib.hsc_table_name(self.ctx, tid)
        return None if r is None else r.decode()

    def table_id(self, name: str) -> int:
        return self.lib.hsc_table_id(self.ctx, name.encode())

    def table_max(self) -> np.ndarray:
        n = self.lib.hsc_table_max(self.ctx, None, 0)
        out = np.zeros(max(1, n), dtype=np.uint64)
        self.lib.hsc_table_max(self.ctx, out.ctypes.data, n)
        return out[:n]

    def merge_table_max(self, tm: np.ndarray) -> None:
        tm = np.ascontiguousarray(tm, dtype=np.uint64)
        self._chk(self.lib.hsc_merge_table_max(self.ctx, tm.ctypes.data, len(tm)),
                  "hsc_merge_table_max")

    # dependency graph + SCC (A10)
    def dep_graph_scc(self, h) -> tuple:
        """(scc[ntxn] = largest txn id of each txn's SCC, stats dict)."""
        cols = [np.ascontiguousarray(h.txn, np.uint32), np.ascontiguousarray(h.key, np.uint64),
                np.ascontiguousarray(h.is_write, np.uint8), np.ascontiguousarray(h.observed, np.int64)]
        hs = _History(len(cols[0]), h.ntxn, *[c.ctypes.data for c in cols])
        out = np.zeros(max(1, h.ntxn), dtype=np.uint32)
        st = GraphStats()
        self._chk(self.lib.hsc_dep_graph_scc(self.ctx, C.byref(hs), out.ctypes.data, C.byref(st)),
                  "hsc_dep_graph_scc")
        return out[: h.ntxn], st.as_dict()

    @staticmethod
    def _history(h):
        cols = [np.ascontiguousarray(h.txn, np.uint32), np.ascontiguousarray(h.key, np.uint64),
                np.ascontiguousarray(h.is_write, np.uint8), np.ascontiguousarray(h.observed, np.int64)]
        return _History(len(cols[0]), h.ntxn, *[c.ctypes.data for c in cols]), cols

    # -- sharded SCC (hsc_dep_graph_build / _cover / _cut / _scc_cut); the
    #    torch-tensor flow over ranks is comdb2_amd.shard.sharded_scc --------
    def dep_graph_stage_rw_pairs(self, readset_txn, commit_lsn, commit_txn) -> None:
        """The last rw_edges() pairs as rw edges of the next dep_graph_build
        (hsc_dep_graph_stage_rw_pairs)."""
        rt = np.ascontiguousarray(readset_txn, np.uint32)
        cl = np.ascontiguousarray(commit_lsn, np.uint64)
        ct = np.ascontiguousarray(commit_txn, np.uint32)
        self._chk(self.lib.hsc_dep_graph_stage_rw_pairs(self.ctx, len(rt), rt.ctypes.data, len(cl),
                                                        cl.ctypes.data, ct.ctypes.data),
                  "hsc_dep_graph_stage_rw_pairs")

    def dep_graph_scc_built(self, ntxn: int) -> tuple:
        """(scc[ntxn], stats) of the last full build (hsc_dep_graph_scc_built)."""
        out = np.zeros(max(1, ntxn), dtype=np.uint32)
        st = GraphStats()
        self._chk(self.lib.hsc_dep_graph_scc_built(self.ctx, out.ctypes.data, C.byref(st)),
                  "hsc_dep_graph_scc_built")
        return out[:ntxn], st.as_dict()

    def dep_graph_build(self, h, full: bool = False, no_rw: bool = False) -> dict:
        """full: sorted unique edges + CSR (dep_graph_edges, edge stats);
        else the raw edge rows only (all the cover / cut steps need).  no_rw:
        reads give wr edges only (rw edges staged from the validator)."""
        hs, keep = self._history(h)
        st = GraphStats()
        flags = (1 if full else 0) | (2 if no_rw else 0)
        self._chk(self.lib.hsc_dep_graph_build(self.ctx, C.byref(hs), flags, C.byref(st)),
                  "hsc_dep_graph_build")
        return st.as_dict()

    def dep_graph_build_device(self, nops: int, ntxn: int, txn_ptr: int, key_ptr: int,
                               is_write_ptr: int, observed_ptr: int, full: bool = False) -> dict:
        """Device-resident ops: txn u32, key u64, is_write u8, observed u32
        (0xFFFFFFFF = initial version)."""
        st = GraphStats()
        self._chk(self.lib.hsc_dep_graph_build_device(self.ctx, nops, ntxn, C.c_void_p(txn_ptr),
                                                      C.c_void_p(key_ptr), C.c_void_p(is_write_ptr),
                                                      C.c_void_p(observed_ptr), int(full),
                                                      C.byref(st)),
                  "hsc_dep_graph_build_device")
        return st.as_dict()

    def dep_graph_cover(self, cover_ptr: int) -> None:
        self._chk(self.lib.hsc_dep_graph_cover(self.ctx, C.c_void_p(cover_ptr)), "hsc_dep_graph_cover")

    def dep_graph_cut(self, cover_ptr: int, rows_ptr: Optional[int] = None, cap: int = 0) -> int:
        m = C.c_size_t()
        self._chk(self.lib.hsc_dep_graph_cut(self.ctx, C.c_void_p(cover_ptr), C.c_void_p(rows_ptr or 0),
                                             cap, C.byref(m)), "hsc_dep_graph_cut")
        return m.value

    def dep_graph_scc_cut(self, ntxn: int, cover_ptr: int, rows_ptr: int, m: int,
                          scc_ptr: int) -> dict:
        st = GraphStats()
        self._chk(self.lib.hsc_dep_graph_scc_cut(self.ctx, ntxn, C.c_void_p(cover_ptr),
                                                 C.c_void_p(rows_ptr), m, C.c_void_p(scc_ptr),
                                                 C.byref(st)), "hsc_dep_graph_scc_cut")
        return st.as_dict()

    def dep_graph_edges(self) -> tuple:
        n = C.c_size_t()
        self._chk(self.lib.hsc_dep_graph_edges(self.ctx, None, None, None, 0, C.byref(n)),
                  "hsc_dep_graph_edges")
        m = n.value
        a = [np.zeros(max(1, m), dtype=np.uint32) for _ in range(3)]
        self._chk(self.lib.hsc_dep_graph_edges(self.ctx, a[0].ctypes.data, a[1].ctypes.data,
                                               a[2].ctypes.data, m, C.byref(n)),
                  "hsc_dep_graph_edges")
        return tuple(x[:m] for x in a)

    def probe_device(self, batch: ProbeBatch) -> None:
        self._chk(self.lib.hsc_probe_device(self.ctx, C.byref(batch)), "hsc_probe_device")

    def pack_verdicts(self, verdict_ptr: int, n_txn: int, bitmap_ptr: int) -> None:
        self._chk(self.lib.hsc_pack_verdicts(self.ctx, verdict_ptr, n_txn, bitmap_ptr),
                  "hsc_pack_verdicts")

    def or_bitmaps(self, parts_ptr: int, nparts: int, words: int, out_ptr: int) -> None:
        """out[w] = OR of the nparts bitmaps parts[k * words + w] (device)."""
        self._chk(self.lib.hsc_or_bitmaps(self.ctx, parts_ptr, nparts, words, out_ptr),
                  "hsc_or_bitmaps")

    def set_autocollect(self, on: bool) -> None:
        """hip_bdb_osql_serial_check through the context's own collector
        (the default) or one device pass per call."""
        self._chk(self.lib.hsc_set_autocollect(self.ctx, 1 if on else 0), "hsc_set_autocollect")

    def set_stream(self, stream_handle: int) -> None:
        self._chk(self.lib.hsc_set_stream(self.ctx, stream_handle), "hsc_set_stream")

    def synchronize(self) -> None:
        self._chk(self.lib.hsc_synchronize(self.ctx), "hsc_synchronize")

    def enable_timing(self, on: bool = True) -> None:
        self._chk(self.lib.hsc_enable_timing(self.ctx, int(on)), "hsc_enable_timing")

    def timing(self) -> dict:
        t = Timing()
        self._chk(self.lib.hsc_get_timing(self.ctx, C.byref(t)), "hsc_get_timing")
        return t.as_dict()


class MultiValidator(Validator):
    """A multi-GPU context (hsc_multi_create / hsc_multi_create_rank): every
    Validator method that the C ABI allows on a multi context works on it
    (the drop-in checks, the collector, log ingest / appends); the window is
    spread over member contexts by composite-key splitters and every batch is
    routed between them on the GPUs.

    devices: members in this process (a device may repeat: several members on
    one GPU).  Or rank / world / ids (hsc_multi_unique_ids bytes, identical on
    every rank) and device: this process is one member of a per-rank context
    exchanging over RCCL."""

    def __init__(self, devices: Optional[Sequence[int]] = None, rank: Optional[int] = None,
                 world: Optional[int] = None, ids: Optional[bytes] = None, device: int = 0):
        self.lib = load()
        self._keep = None
        self.ctx = None
        ctx = _p()
        if devices is not None:
            devs = (C.c_int * len(devices))(*devices)
            rc = self.lib.hsc_multi_create(devs, len(devices), C.byref(ctx))
            what = f"hsc_multi_create({list(devices)})"
        else:
            buf = C.create_string_buffer(bytes(ids), len(ids))
            rc = self.lib.hsc_multi_create_rank(device, rank, world, buf, len(ids), C.byref(ctx))
            what = f"hsc_multi_create_rank(device {device}, rank {rank}, world {world})"
        if rc != HSC_OK:
            raise HscError(f"{what} = {rc}")
        self.ctx = ctx

    @staticmethod
    def unique_ids() -> bytes:
        lib = load()
        buf = C.create_string_buffer(MULTI_ID_BYTES)
        rc = lib.hsc_multi_unique_ids(buf, MULTI_ID_BYTES)
        if rc != HSC_OK:
            raise HscError(f"hsc_multi_unique_ids -> {rc}")
        return buf.raw

    @property
    def world(self) -> int:
        return self.lib.hsc_multi_world(self.ctx)

    @property
    def rank(self) -> int:
        return self.lib.hsc_multi_rank(self.ctx)

    @property
    def nlocal(self) -> int:
        return self.lib.hsc_multi_local(self.ctx)

    def member(self, i: int) -> Validator:
        """Member context i (owned by the multi context: not closed by the
        returned wrapper)."""
        v = Validator.__new__(_Member)
        v.lib, v._keep = self.lib, None
        v.ctx = _p(self.lib.hsc_multi_member(self.ctx, i))
        if not v.ctx:
            raise HscError(f"no member {i}")
        return v

    def set_splitters(self, gid: np.ndarray, words: np.ndarray) -> None:
        """world - 1 ascending composite splitters: gid u32[S], words u64[W, S]."""
        gid = np.ascontiguousarray(gid, np.uint32)
        words = np.ascontiguousarray(words, np.uint64).reshape(-1, len(gid)) if len(gid) else \
            np.zeros((1, 0), np.uint64)
        self._chk(self.lib.hsc_multi_set_splitters(self.ctx, len(gid), gid.ctypes.data,
                                                   words.ctypes.data, words.shape[0]),
                  "hsc_multi_set_splitters")

    def adopt(self) -> None:
        self._chk(self.lib.hsc_multi_adopt(self.ctx), "hsc_multi_adopt")

    def set_mode(self, mode: int) -> None:
        """Window placement: MULTI_AUTO, MULTI_PIECES or MULTI_REPLICAS
        (hsc_multi_set_mode)."""
        self._chk(self.lib.hsc_multi_set_mode(self.ctx, int(mode)), "hsc_multi_set_mode")

    @property
    def mode(self) -> int:
        """The placement in force: MULTI_PIECES or MULTI_REPLICAS."""
        return self.lib.hsc_multi_mode(self.ctx)

    def set_transport(self, loopback: bool) -> None:
        """In-process members: HSC_MULTI_LOOPBACK runs the per-rank exchange
        (send blocks, unpack, owner slices) with peer copies in place of RCCL."""
        self._chk(self.lib.hsc_multi_set_transport(self.ctx, int(bool(loopback))),
                  "hsc_multi_set_transport")

    def marshal_routed(self, rs: ReadSets, member: int, txn_base: int = 0) -> dict:
        """Marshal rs and route it on the host: member's columns (read-set
        numbers + txn_base; table locks for member 0), forced of the batch."""
        s, keep = readsets_struct(rs)
        mp = C.POINTER(Marshalled)()
        self._chk(self.lib.hsc_multi_marshal_routed(self.ctx, C.byref(s), member, txn_base,
                                                    C.byref(mp)), "hsc_multi_marshal_routed")
        return self._marshalled(mp.contents)

    def routed_shares(self, shares: Sequence[ReadSets], members: Sequence[int]) -> dict:
        """The global batch = the owners' shares (share o owned by member o):
        each marshalled once and routed on the host; per member in `members`
        its columns of all shares concatenated, read sets numbered batch-wide
        (share o from owner_base[o], every base a multiple of 64).
        -> {member: columns}; every entry carries owner_base and forced[o]
        (share o's host-decided verdicts)."""
        base = [0]
        for rs in shares:
            base.append(base[-1] + (rs.ntxn + 63) // 64 * 64)
        parts = {m: [] for m in members}
        forced = []
        for o, rs in enumerate(shares):
            s, keep = readsets_struct(rs)
            mp = C.POINTER(Marshalled)()
            who = members[0] if len(members) == 1 else -1  # -1: route to every member
            self._chk(self.lib.hsc_multi_marshal_routed(self.ctx, C.byref(s), who, base[o], C.byref(mp)),
                      "hsc_multi_marshal_routed")
            forced.append(self._marshalled(mp.contents)["forced"])
            for m in members:
                self._chk(self.lib.hsc_multi_routed_member(self.ctx, m, C.byref(mp)),
                          "hsc_multi_routed_member")
                parts[m].append(self._marshalled(mp.contents))
        out = {}
        for m, ps in parts.items():
            cat = lambda k: np.concatenate([p[k] for p in ps])
            out[m] = dict(words=ps[0]["words"], n=sum(p["n"] for p in ps),
                          n_lock=sum(p["n_lock"] for p in ps), n_txn=base[-1],
                          owner_base=np.array(base, np.uint64),
                          lo=np.concatenate([p["lo"] for p in ps], axis=1),
                          hi=np.concatenate([p["hi"] for p in ps], axis=1),
                          gid=cat("gid"), snap=cat("snap"), txn=cat("txn"), lock_table=cat("lock_table"),
                          lock_snap=cat("lock_snap"), lock_txn=cat("lock_txn"), forced=forced)
        return out

    def graph_scc(self, shards, ntxn: int, scc_ptrs) -> dict:
        """hsc_multi_graph_scc: shards[i] = local member i's key shard of the
        history on its GPU (shard.DeviceHistory or an object with nops / txn /
        key / is_write / observed tensors), scc_ptrs[i] = device u32[ntxn]
        (index 0 required).  -> member 0's SCC stats + host phase ms."""
        ops = (OpsDev * len(shards))()
        for i, h in enumerate(shards):
            ops[i].nops = h.nops
            ops[i].txn = h.txn.data_ptr()
            ops[i].key = h.key.data_ptr()
            ops[i].is_write = h.is_write.data_ptr()
            ops[i].observed = h.observed.data_ptr()
        ptrs = (_p * len(shards))(*[C.c_void_p(x) if x else None for x in scc_ptrs])
        st = GraphStats()
        self._chk(self.lib.hsc_multi_graph_scc(self.ctx, ops, ntxn, ptrs, C.byref(st)),
                  "hsc_multi_graph_scc")
        out = st.as_dict()
        ph = np.zeros(4, np.float64)
        self._chk(self.lib.hsc_multi_graph_phase_ms(self.ctx, ph.ctypes.data), "hsc_multi_graph_phase_ms")
        out["phase_ms"] = {"build_cover": ph[0], "cover_merge": ph[1], "cut_union": ph[2], "scc": ph[3]}
        return out

    def enable_member_timing(self, on: bool = True) -> None:
        self._chk(self.lib.hsc_multi_enable_timing(self.ctx, int(on)), "hsc_multi_enable_timing")

    def member_probe_ms(self) -> np.ndarray:
        """Per local member: its probe's device ms in the last routed batch."""
        out = np.zeros(max(1, self.nlocal), np.float32)
        self._chk(self.lib.hsc_multi_member_probe_ms(self.ctx, out.ctypes.data, len(out)),
                  "hsc_multi_member_probe_ms")
        return out[:self.nlocal]

    def probe_routed(self, batches: Sequence[ProbeBatch], owner_base: Sequence[int],
                     lane: int = 0) -> None:
        """Batches routed at marshal time (one per local member), read sets
        numbered batch-wide; owner o owns [owner_base[o], owner_base[o+1])."""
        arr = (ProbeBatch * len(batches))(*batches)
        ob = np.ascontiguousarray(owner_base, np.uint64)
        self._chk(self.lib.hsc_multi_probe_routed(self.ctx, arr, ob.ctypes.data, lane),
                  "hsc_multi_probe_routed")

    def prepare_routed(self, batches: Sequence[ProbeBatch], owner_base: Sequence[int]):
        """The arguments of hsc_multi_probe_routed built once (the ctypes
        array of member batches and the owner bases), for a caller that
        probes the same resident batches many times (bench.py's ring): the
        step is then one foreign call, no per-call marshalling in Python."""
        arr = (ProbeBatch * len(batches))(*batches)
        ob = np.ascontiguousarray(owner_base, np.uint64)
        return (arr, ob, C.c_void_p(ob.ctypes.data))

    def probe_routed_prepared(self, prep, lane: int = 0) -> None:
        rc = self.lib.hsc_multi_probe_routed(self.ctx, prep[0], prep[2], lane)
        if rc:
            self._chk(rc, "hsc_multi_probe_routed")

    def prepare_device(self, batches: Sequence[ProbeBatch]):
        return (ProbeBatch * len(batches))(*batches)

    def probe_device_prepared(self, arr, lane: int = 0) -> None:
        rc = self.lib.hsc_multi_probe_device(self.ctx, arr, lane)
        if rc:
            self._chk(rc, "hsc_multi_probe_device")

    def route_stats(self) -> dict:
        out = np.zeros(8, np.float64)
        self._chk(self.lib.hsc_multi_route_stats(self.ctx, out.ctypes.data), "hsc_multi_route_stats")
        return {"calls": int(out[0]), "member_checks": int(out[1]), "probes": int(out[2]),
                "rows": int(out[3]), "route_us_per_call": float(out[4]), "world": int(out[5]),
                "launch_us_per_call": float(out[6]), "wait_us_per_call": float(out[7])}

    def probe_device_multi(self, batches: Sequence[ProbeBatch], lane: int = 0) -> None:
        arr = (ProbeBatch * len(batches))(*batches)
        self._chk(self.lib.hsc_multi_probe_device(self.ctx, arr, lane), "hsc_multi_probe_device")

    def multi_stats(self) -> dict:
        out = np.zeros(4, np.uint64)
        self._chk(self.lib.hsc_multi_stats(self.ctx, out.ctypes.data), "hsc_multi_stats")
        return {"batches": int(out[0]), "probes": int(out[1]), "routed": int(out[2]),
                "local_members": int(out[3])}

    def phase_stats(self) -> dict:
        """Host time per routed batch, mean us (hsc_multi_phase_stats)."""
        out = np.zeros(7, np.float64)
        self._chk(self.lib.hsc_multi_phase_stats(self.ctx, out.ctypes.data), "hsc_multi_phase_stats")
        return {"batches": int(out[0]), "lane_wait_us": float(out[1]), "count_launch_us": float(out[2]),
                "count_wait_us": float(out[3]), "enqueue_us": float(out[4]),
                "routed_batches": int(out[5]), "routed_enqueue_us": float(out[6])}

    def routed_phase_stats(self) -> dict:
        """hsc_multi_probe_routed's host us per batch: lane waits, member probe
        launches, merges (hsc_multi_routed_phase_stats)."""
        out = np.zeros(4, np.float64)
        self._chk(self.lib.hsc_multi_routed_phase_stats(self.ctx, out.ctypes.data),
                  "hsc_multi_routed_phase_stats")
        return {"batches": int(out[0]), "lane_us": float(out[1]), "probe_launch_us": float(out[2]),
                "merge_us": float(out[3])}

    def last_counts(self) -> np.ndarray:
        n = self.world
        out = np.zeros(n * n, np.uint32)
        self._chk(self.lib.hsc_multi_last_counts(self.ctx, out.ctypes.data, n * n),
                  "hsc_multi_last_counts")
        return out.reshape(n, n)


class _Member(Validator):
    """A member context of a MultiValidator (not owned: close() is a no-op)."""

    def close(self) -> None:
        self.ctx = None


def bdb_osql_serial_check(v: Validator, arr: Optional[CurRangeArr], regop_only: int = 0) -> int:
    """bdb_osql_serial_check(bdb_state, ranges, &arr->file, &arr->offset, regop_only)
    (bdb/serializable.c:571): 0 = serializable, nonzero = not (or error)."""
    if arr is None:
        return 0
    f = C.c_uint(arr.file)
    o = C.c_uint(arr.offset)
    rc = v.lib.hip_bdb_osql_serial_check(v.ctx, C.cast(C.pointer(arr), _p), C.byref(f),
                                         C.byref(o), regop_only)
    arr.file, arr.offset = f.value, o.value
    return rc
