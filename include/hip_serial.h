/*
 * hip_serial.h -- C ABI of the MI355X serializable-isolation conflict validator.
 *
 * This library replaces the read-set check of comdb2's SERIALIZABLE isolation:
 *
 *   reference entry   int bdb_osql_serial_check(bdb_state_type *, void *ranges,
 *                         unsigned int *file, unsigned int *offset, int regop_only);
 *                     bdb/bdb_api.h:1824-1826, bdb/serializable.c:571-579
 *   reference plugin  SERIALCHECK serial_check_callback(char *tbname, int idxnum,
 *                         void *key, int keylen, void *ranges)
 *                     bdb/bdb_api.h:336-337, db/glue.c:2926-2963
 *   reference walk    osql_serial_check / serial_check_this_txn
 *                     bdb/serializable.c:341-569, 60-332
 *
 * Instead of re-walking the log once per transaction and scanning every read
 * range per logged write key, the library keeps the committed-write window
 * resident in HBM (sorted by (group, key), deduplicated to the max commit LSN
 * per key) and answers a whole batch of read sets with one range-overlap join
 * written as hand-written HIP kernels for gfx950.
 *
 * Every entry point is plain C: pointers and sizes, no torch or HIP types.
 * Return codes: 0 = success, negative = HSC_E* error.  For the check entry
 * points, rc_out[i] keeps the reference meaning: 0 = serializable, nonzero =
 * not serializable (callers never distinguish errors from conflicts,
 * db/toblock.c:4779-4805); on any device error every rc_out[i] is set to 1
 * (fail closed, as bdb/serializable.c:94-104,417-421 do for log errors).
 */
#ifndef HIP_SERIAL_H
#define HIP_SERIAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------
 * Read-set types.  Layout-identical mirrors of db/comdb2.h:1105-1124 so that a
 * comdb2 caller passes its own CurRangeArr* straight through (the `hash`
 * member built by currangearr_build_hash, db/sqlglue.c:312-351, is not read:
 * the library recomputes the same first-table / [begin,end] spans itself).
 * ------------------------------------------------------------------------ */
typedef struct hsc_currange {
    char *tbname;   /* NUL-terminated table name                              */
    int idxnum;     /* index number; -1 table scan; -2 default (currange_new) */
    void *lkey;     /* lower bound bytes (NULL or lkeylen bytes)              */
    void *rkey;     /* upper bound bytes                                      */
    int lflag;      /* 1: lower bound open (unbounded)                        */
    int lkeylen;
    int rflag;      /* 1: upper bound open                                    */
    int rkeylen;
    int islocked;   /* whole table read (full scan / both ends hit)           */
} hsc_currange;

typedef struct hsc_currangearr {
    int size;
    int cap;
    unsigned int file;   /* snapshot LSN (bdb_get_current_lsn at begin)       */
    unsigned int offset;
    void *hash;          /* ignored                                           */
    hsc_currange **ranges;
} hsc_currangearr;

/* ---------------------------------------------------------------------------
 * Log record stream, decoded to struct-of-arrays.  One row per log record, in
 * LSN order -- the view bdb/serializable.c gets from DB_LOGC->get plus the
 * generated llog_*_read decoders (bdb/llog.src:26-225).  Keys of undo_add_ix /
 * undo_del_ix[_lk] are the ones bdb_reconstruct_add/delete would recover
 * (bdb/rowlocks.c:428-617).
 * ------------------------------------------------------------------------ */
enum {
    HSC_REC_TXN_REGOP = 10,          /* berkdb/dbinc_auto/txn_auto.h:6        */
    HSC_REC_TXN_REGOP_ROWLOCKS = 15, /* txn_auto.h:59                         */
    HSC_REC_TXN_REGOP_GEN = 16,      /* txn_auto.h:76                         */
    HSC_REC_UNDO_ADD_DTA = 10003,    /* bdb/llog.src:26                       */
    HSC_REC_UNDO_ADD_IX = 10004,
    HSC_REC_LTRAN_COMMIT = 10005,
    HSC_REC_LTRAN_START = 10006,
    HSC_REC_LTRAN_COMPREC = 10007,
    HSC_REC_UNDO_DEL_DTA = 10008,
    HSC_REC_UNDO_DEL_IX = 10009,
    HSC_REC_UNDO_UPD_DTA = 10010,
    HSC_REC_UNDO_UPD_IX = 10011,
    HSC_REC_UNDO_ADD_DTA_LK = 10013,
    HSC_REC_UNDO_ADD_IX_LK = 10014,
    HSC_REC_UNDO_DEL_DTA_LK = 10015,
    HSC_REC_UNDO_DEL_IX_LK = 10016,
    HSC_REC_UNDO_UPD_DTA_LK = 10017,
    HSC_REC_UNDO_UPD_IX_LK = 10018,
    /* berkdb physical records the index-key reconstruction walks
     * (bdb/rowlocks.c:209-426; layouts berkdb/db/db.src) */
    HSC_REC_DB_ADDREM = 41,          /* db.src:47-57                          */
    HSC_REC_DB_BIG = 43,             /* db.src:73-83                          */
    HSC_REC_DB_DEBUG = 47,           /* db.src:131                            */
    HSC_REC_DB_PG_FREE = 50,         /* db.src:177-184                        */
    HSC_REC_DB_PG_FREEDATA = 52      /* db.src:206-214                        */
};

typedef struct hsc_llog {
    size_t nrec;
    const uint64_t *lsn;      /* (file << 32) | offset, strictly increasing   */
    const uint32_t *rectype;  /* HSC_REC_*                                    */
    const uint64_t *prev;     /* regop*: prev_lsn; llog records: prevllsn     */
    const int16_t *isabort;   /* ltran_commit: isabort                        */
    const int32_t *table;     /* llog undo records: index into tbnames        */
    const int16_t *ix;        /* undo_*_ix*: index number (short on disk)     */
    const uint64_t *key_off;  /* undo_*_ix*: key byte offset into keys        */
    const int32_t *keylen;    /* undo_*_ix*: key length                       */
    const uint8_t *keys;
    const char *const *tbnames;
    int ntbnames;
    uint64_t end_lsn;         /* __log_txn_lsn (berkdb/log/log_put.c:509)     */
} hsc_llog;

/* ---------------------------------------------------------------------------
 * Flat read sets: many CurRangeArr's as struct-of-arrays (the OSQL_SERIAL
 * payload of db/osqlcomm.c:909-993 after decode, without heap CurRange's).
 * Ranges of read set t are rows [txn_off[t], txn_off[t+1]) in array order.
 *
 * Key pointers: lkey_off / rkey_off == HSC_KEY_NULL stands for a NULL key
 * pointer (its length must be 0; currange_new leaves keys NULL,
 * db/sqlglue.c:163-175); any other offset is a present key, also with length
 * 0 (serial_readset_get malloc(0)s one, db/osqlcomm.c:974).  Only the
 * coalesce comparator tells them apart: currange_cmp compares the lower keys
 * only when both pointers are non-NULL (db/sqlglue.c:228-236), so a NULL one
 * ties with every range of its index while a present empty key sorts before
 * the longer ones.  The check itself reads at most min(len, keylen) bytes and
 * treats both alike (db/glue.c:2951-2958).
 * ------------------------------------------------------------------------ */
#define HSC_KEY_NULL UINT64_MAX
typedef struct hsc_readsets {
    int ntxn;
    const int64_t *txn_off;   /* [ntxn+1]                                     */
    const uint64_t *snap;     /* [ntxn] snapshot LSN (file << 32 | offset)    */
    const int32_t *table;     /* [nranges] index into tbnames                 */
    const int32_t *idxnum;
    const int32_t *lflag, *rflag, *islocked;
    const int32_t *lkeylen, *rkeylen;
    const uint64_t *lkey_off, *rkey_off; /* byte offsets into keys           */
    const uint8_t *keys;
    const char *const *tbnames;
    int ntbnames;
} hsc_readsets;

/* OSQL_SERIAL payloads (one read set each) as the master receives them:
 * message i = buf[off[i] .. off[i] + len[i]), starting at the osql_serial_t
 * header (buf_size, arr_size, file, offset; db/osqlcomm.c:748-753,809-826)
 * followed by the serial_readset_put ranges (db/osqlcomm.c:909-946).  Every
 * 2/4/8-byte item is byte-swapped on the wire (buf_put,
 * bbinc/endian_core.amd64.h:17-44) -- keys and table names of those lengths
 * included. */
typedef struct hsc_serial_msgs {
    size_t nmsg;
    const uint8_t *buf;
    const uint64_t *off;
    const uint64_t *len;
} hsc_serial_msgs;

/* Decoded committed write (what serial_check_this_txn hands the callback). */
typedef struct hsc_write {
    const char *tbname;
    int idxnum;          /* -2 for dta records (key == NULL)                  */
    const void *key;     /* NULL for dta records                              */
    int keylen;
    uint64_t commit_lsn; /* LSN of the txn's regop record                     */
} hsc_write;

/* Device-resident probe batch (what the check entry points lower to).  All
 * pointers are device pointers on the context's GPU.  Key words are the key
 * bytes in big-endian 8-byte words, zero padded, held as native uint64 so that
 * numeric order of the words equals memcmp order of the bytes. */
typedef struct hsc_probe_batch {
    size_t n;                 /* range probes                                  */
    const uint64_t *lo;       /* [words][n]                                    */
    const uint64_t *hi;       /* [words][n]                                    */
    const uint32_t *gid;      /* [n] key group (table, index, key length)      */
    const uint64_t *snap;     /* [n] snapshot LSN of the owning read set       */
    const uint32_t *txn;      /* [n] read-set (transaction) index              */
    size_t n_lock;            /* table-lock probes                             */
    const uint32_t *lock_table;
    const uint64_t *lock_snap;
    const uint32_t *lock_txn;
    size_t n_txn;
    uint8_t *verdict;         /* [n_txn] out: 1 = not serializable             */
    uint64_t *bitmap;         /* [ceil(n_txn/64)] out (may be NULL)            */
} hsc_probe_batch;

/* Per-kernel device time of the last probe / window build, in ms.  Wide
 * layout: locate, plan, scatter, join, pack kernels.  Narrow layout: locate =
 * verdict clear, join = the single probe kernel, pack; plan = scatter = 0. */
typedef struct hsc_timing {
    float locate_ms, plan_ms, scatter_ms, join_ms, pack_ms, probe_total_ms;
    float ingest_ms;
    uint64_t records;         /* join records emitted by the last probe         */
    uint64_t tiles;           /* tiles in the resident window                   */
} hsc_timing;

typedef struct hsc_ctx hsc_ctx;

enum {
    HSC_OK = 0,
    HSC_EINVAL = -1,
    HSC_EDEVICE = -2,
    HSC_ENOMEM = -3,
    HSC_ELOG = -4,     /* malformed log stream (unknown record, broken link)  */
    HSC_ESTATE = -5    /* window not built                                    */
};

/* ---- context ------------------------------------------------------------ */
/* device = -1 creates a host-only context: log decode, dictionaries and
 * marshalling work; every device operation returns HSC_EDEVICE. */
int hsc_ctx_create(int device, hsc_ctx **out);
void hsc_ctx_destroy(hsc_ctx *ctx);
/* Launch on this hipStream_t (NULL = the context's own stream).  Probes are
 * stream-ordered on the stream current at the call.  Each stream that probes
 * gets its own probe lane (scratch buffers, up to 4 lanes; a fifth stream
 * takes over the least recently used lane after waiting for that lane's last
 * batch), so batches probed on different streams may run concurrently.
 * Window builds wait for every lane's last batch; the caller orders a window
 * change against later probes on other streams.  A stream stays in use by the
 * context until the next hsc_set_stream (which records its lane's fence on
 * it) or hsc_ctx_destroy: keep it valid until then. */
int hsc_set_stream(hsc_ctx *ctx, void *hip_stream);
const char *hsc_last_error(hsc_ctx *ctx);
int hsc_device_count(void);

/* ---- write window (replaces the per-call log walk) ---------------------- */
/* Decode a log stream: every committed write txn (regop whose prev record is
 * an ltran_commit with isabort == 0 and prevllsn.file != 0,
 * bdb/serializable.c:426-534) contributes its logical records' (table, ix,
 * key) at the regop's LSN.  Replaces the window. */
int hsc_window_ingest_log(hsc_ctx *ctx, const hsc_llog *log);
/* Raw log records as a log cursor returns them (DB_LOGC->get data): the
 * bdb/llog.src:26-225 layouts, the txn regop records
 * (berkdb/dbinc_auto/txn_auto.h:6-86) and any berkdb physical records, in the
 * gen_rec_endian.awk on-disk encoding of a little-endian host: u32/short
 * fields and DB_LSNs big-endian, genid_t native, DBT = u32 BE size + bytes.
 * Record i is lsn[i] (strictly increasing), bytes buf[off[i] .. off[i] +
 * len[i]).  undo_add_ix / undo_del_ix / undo_del_ix_lk carry no key: the
 * reference rebuilds it from the physical log at undolsn = the record's header
 * prev_lsn (bdb/serializable.c:123-130,174-181), walking the header prev_lsn
 * chain over __db_addrem / __db_big / __db_pg_free[data] records
 * (bdb_reconstruct_add / _delete, bdb/rowlocks.c:209-617); the decoder runs
 * the same walk over the records of this log and, for appends, of every raw
 * log decoded since the last ingest.  A key the walk does not fully define
 * (the reference would read its uninitialised key buffer) is HSC_ELOG.
 * recon_* (optional, sorted by undolsn) supplies keys directly: an entry for
 * a record's undolsn takes precedence over the walk. */
typedef struct hsc_raw_log {
    size_t nrec;
    const uint64_t *lsn;
    const uint64_t *off;
    const uint32_t *len;
    const uint8_t *buf;
    uint64_t end_lsn;
    size_t nrecon;
    const uint64_t *recon_lsn;
    const uint64_t *recon_off;
    const int32_t *recon_len;
    const uint8_t *recon_keys;
} hsc_raw_log;
/* Decode + ingest (replaces the window), = hsc_window_ingest_log of the
 * decoded stream. */
int hsc_window_ingest_raw(hsc_ctx *ctx, const hsc_raw_log *log);
/* Decode only: *out points at a context-owned hsc_llog valid until the next
 * decode on this context. */
int hsc_decode_log(hsc_ctx *ctx, const hsc_raw_log *log, const hsc_llog **out);
/* Append decoded writes (commit_lsn non-decreasing across calls).  On a
 * built window (log, raw, staged or device ingest) the rows go to a sorted
 * delta run on the device (one merge launch per call; the reference sees
 * every commit up to the end of the log on every check, bdb/serializable.c:
 * 390-539, and commits keep appending, bdb/tran.c:1545-1560) that every probe
 * checks beside the main window; past 65536 delta rows, or on a key longer
 * than the window's words, the next check folds the delta into the main
 * window with one device rebuild.  Decoded writes carry no record LSNs, so
 * after one the DB_SET-on-a-non-record rule (bdb/serializable.c:417-421) is
 * off for the window.  The window's end LSN advances to at least
 * commit_lsn + 1 of every appended write (a snapshot at or past the old end
 * must still see it: fail closed); hsc_window_set_end sets the exact end of
 * the log (curlsn of full checks). */
int hsc_window_append(hsc_ctx *ctx, const hsc_write *w, size_t n);
/* Append log records: the continuation of the window's log (LSNs above every
 * record taken so far; log->end_lsn is the new end).  Every txn a new regop
 * commits contributes its writes, its logical chain walked back into records
 * of earlier ingests / appends when it reaches them (SURVEY.md §8(f) 1,
 * incremental decode); record LSNs, poison rules and the delta run follow. */
int hsc_window_append_log(hsc_ctx *ctx, const hsc_llog *log);
/* Raw-record form of hsc_window_append_log (hsc_raw_log as for ingest). */
int hsc_window_append_raw(hsc_ctx *ctx, const hsc_raw_log *log);
/* Rows in the delta run (appended since the last build of the main window). */
size_t hsc_window_delta_rows(hsc_ctx *ctx);
/* Delta folding.  Appended rows live in a sorted delta run beside the main
 * window; once it holds `rows` rows (0 = the default, half the run's
 * capacity of 65536) it is folded into the main window.  background = 1
 * (default): the run is frozen and the main window rebuilt with it on a
 * second stream and host thread while checks go on against the old window +
 * frozen run + a fresh run; the rebuilt window is swapped in by the first
 * call after it finished.  background = 0: the next check merges the run
 * inline (a full rebuild on the check's path). */
int hsc_set_fold(hsc_ctx *ctx, size_t rows, int background);
/* out[4]: background folds started, background folds swapped in, inline
 * merges, build time of the last background fold in microseconds. */
int hsc_fold_stats(hsc_ctx *ctx, uint64_t out[4]);
/* The pending tail (narrow windows whose keys fit 4 words): an append's rows
 * are mirrored into mapped host memory that the small-batch kernel scans
 * beside the delta runs, and merged into the live run once 256 rows wait or a
 * batch that is not small runs.  out[3]: appends kept in the tail, merges of
 * the tail into the run, rows waiting now. */
int hsc_append_stats(hsc_ctx *ctx, uint64_t out[3]);
/* Path restrictions of one context, for tests and A/B runs (0 = every path
 * the library picks by itself).  NO_SMALL: batches skip the small-batch
 * kernel (and appends its pending tail); NO_PACKED_SORT: window builds use
 * the whole-row radix sort; TILE_DIR: narrow / compact tile locates search
 * the 16-ary directory instead of the bucket table (set before the build);
 * CO_SERIAL: every coalesced read set takes the per-thread msort replay;
 * CO_RUN_THREAD: one thread per run in the coalesce merge scan;
 * NO_COMP_NARROW: composite keys whose varying bits total <= 62 but span
 * more keep the compact / wide layouts instead of the narrow index over
 * compressed codes (set before the build); NO_CT_POINTS: compact tiles build
 * no point index, so point probes take join records (set before the build). */
#define HSC_PATH_NO_SMALL 1u
#define HSC_PATH_NO_PACKED_SORT 2u
#define HSC_PATH_TILE_DIR 4u
#define HSC_PATH_CO_SERIAL 8u
#define HSC_PATH_CO_RUN_THREAD 16u
#define HSC_PATH_NO_COMP_NARROW 32u
#define HSC_PATH_NO_CT_POINTS 64u
#define HSC_PATH_ALL 127u
int hsc_set_paths(hsc_ctx *ctx, unsigned flags);
/* How the last window build sorted its rows: 0 whole-row radix sort, 1 the
 * packed 64-bit key sort, 2 the compact-code merge sort (wide keys). */
int hsc_window_sort_path(hsc_ctx *ctx);
int hsc_window_set_end(hsc_ctx *ctx, uint64_t end_lsn);
int hsc_window_reset(hsc_ctx *ctx);
/* Sort + dedupe + summaries on the device; implied by the check calls. */
int hsc_window_build(hsc_ctx *ctx);
/* Register a key group ahead of a device-side ingest; returns gid >= 0. */
int hsc_register_group(hsc_ctx *ctx, const char *tbname, int idxnum, int keylen);
/* Device-side ingest of pre-padded keys (bench / sharded driver path):
 * gid[n], words[words][n], lsn[n] are DEVICE pointers, keys already packed as
 * described for hsc_probe_batch; gid values come from hsc_register_group.
 * Rows are versions in log order: of equal (gid, key) rows the last one is
 * the key's newest version.  Replaces the window. */
int hsc_window_ingest_device(hsc_ctx *ctx, size_t n, int words,
                             const uint32_t *gid, const uint64_t *key_words,
                             const uint64_t *lsn, uint64_t end_lsn);
/* Window layout.  AUTO: the narrow layout -- every (group, key) as one
 * 62-bit code under a 16-ary index, each range answered by one probe kernel
 * without bucketing -- whenever the whole window fits it (any single int64
 * index, any single group of keys whose varying bits span < 62 bits), else
 * WIDE (every key as its big-endian words, ranges bucketed by window tile).
 * A narrow window answers a sparse batch (< 8 ranges per 2048-row tile) with
 * one direct probe kernel and a dense one with the tile pipeline over codes.
 * A dense batch runs on 8-byte tile rows (u32 key delta, u32 commit rank)
 * when every 4096-row tile spans < 2^32 codes, else on the codes as 16-byte
 * rows.  WIDE forces the wide layout; NARROW_DIRECT / NARROW_TILES /
 * NARROW_CODES keep AUTO's layout choice but force that probe path (tiles:
 * 8-byte rows where they fit; codes: always 16-byte code rows) -- testing.  Verdicts are
 * identical; a change between WIDE and the others applies at the next window
 * build (host-staged windows rebuild; a device-ingested window returns
 * HSC_ESTATE and must be re-ingested).  hsc_window_layout reports WIDE,
 * NARROW or COMPACT (AUTO on a window too wide for 62-bit codes: each
 * (table, index, key length) group's keys keep only the bits that vary inside
 * the group -- hsc_compact.hip -- when that shortens the rows; WIDE disables
 * it). */
enum {
    HSC_LAYOUT_AUTO = 0,
    HSC_LAYOUT_WIDE = 1,
    HSC_LAYOUT_NARROW = 2,
    HSC_LAYOUT_NARROW_DIRECT = 3,
    HSC_LAYOUT_NARROW_TILES = 4,
    HSC_LAYOUT_NARROW_CODES = 5,
    HSC_LAYOUT_COMPACT = 6, /* reported only: AUTO's wide window as per-group compact codes */
    HSC_LAYOUT_COMPACT_WIDE = 7 /* AUTO, but compact windows probe through the wide tile
                                   pipeline instead of the compact tiles -- testing */
};
int hsc_set_layout(hsc_ctx *ctx, int layout);
int hsc_window_layout(hsc_ctx *ctx);         /* HSC_LAYOUT_WIDE, _NARROW or _COMPACT */
int hsc_window_code_words(hsc_ctx *ctx);     /* words per probed row (compact: WC) */
/* Compact windows: words of the compact-tile keys gid || code (1..3) that
 * dense batches probe (hsc_ctiles.hip), 0 if the window has none. */
int hsc_window_tile_key_words(hsc_ctx *ctx);
int hsc_window_words(hsc_ctx *ctx);          /* key words per key (>= 1)     */
size_t hsc_window_keys(hsc_ctx *ctx);        /* distinct (group, key) rows   */
uint64_t hsc_window_end(hsc_ctx *ctx);
uint64_t hsc_window_max_commit(hsc_ctx *ctx);
/* Window snapshot (checkpoint of the resident state; the reference keeps
 * none -- its state is the log): the rows of the built window in (group, key)
 * order, after folding any delta run.  all_versions = 0: one row per (group,
 * key), its newest version; 1: every version.  gid[cap], key_words[words *
 * cap] (word j of row i at [j * cap + i], big-endian key order), lsn[cap];
 * all three NULL returns only the count.  Returns the row count (> cap:
 * nothing copied) or a negative HSC_E* code. */
long hsc_window_export(hsc_ctx *ctx, int all_versions, uint32_t *gid, uint64_t *key_words,
                       uint64_t *lsn, size_t cap);
int hsc_table_id(hsc_ctx *ctx, const char *tbname); /* -1 if never written   */
const char *hsc_table_name(hsc_ctx *ctx, int table_id); /* NULL if unknown   */
/* Key group gid -> (table id, index, key length); 0 or HSC_EINVAL. */
int hsc_group_info(hsc_ctx *ctx, int gid, int *table_id, int *idxnum, int *keylen);
/* Per-table max commit LSN (dta writes included): copies min(n, ntables)
 * entries, returns ntables. */
int hsc_table_max(hsc_ctx *ctx, uint64_t *out, int n);
/* Max-merge per-table LSNs from other shards (multi-GPU lock probes). */
int hsc_merge_table_max(hsc_ctx *ctx, const uint64_t *in, int n);

/* ---- drop-in checks ----------------------------------------------------- */
/* Exactly bdb_osql_serial_check (bdb/serializable.c:571-579) for one read set:
 * ranges == NULL -> 0; regop_only -> nonzero iff a committed write txn follows
 * (*file,*offset); otherwise (*file,*offset) := end LSN, then the full check.
 * Concurrent callers (one per committing transaction, db/toblock.c:4777-4800)
 * are batched by a collector the context owns (hsc_collector_check below):
 * a lone caller runs its own single-set pass, callers that arrive while a pass
 * runs form the next one -- none waits on another's context lock.
 * hsc_set_autocollect(ctx, 0) makes every call its own pass instead. */
int hip_bdb_osql_serial_check(void *ctx, void *ranges, unsigned int *file,
                              unsigned int *offset, int regop_only);
/* regop_only (here, in hip_serial_check_batch and hsc_collector_check) is
 * answered in the caller's thread from a snapshot (end LSN, max commit LSN,
 * unreadable-regop LSN, DB_SET rule) that every entry changing the window
 * republishes before it returns: no collector queue, no context lock, no
 * window build (db/toblock.c:4779-4785 probes under the commit_lock write
 * lock).  Only a snapshot the published values cannot decide -- no commit
 * after it, inside a log whose record LSNs must be searched -- takes the
 * locked path.  out[0] = probes answered from the snapshot, out[1] = locked. */
int hsc_regop_stats(hsc_ctx *ctx, uint64_t out[2]);
/* The drop-in entry through the context's own collector (1, the default) or
 * one pass per call (0).  0 or HSC_EINVAL. */
int hsc_set_autocollect(hsc_ctx *ctx, int on);
/* n read sets in one device pass.  ranges[i] is a CurRangeArr* (may be NULL);
 * file/offset are arrays of n in/out snapshot LSNs, or NULL to use (and
 * update) ranges[i]->file / ->offset in place.  Per element the semantics and
 * side effects of the single call.  Returns 0 or a negative HSC_E* code. */
int hip_serial_check_batch(void *ctx, void *const *ranges, unsigned int *file,
                           unsigned int *offset, int regop_only, int n,
                           int *rc_out);
/* Batching collector for concurrent callers (the reference calls
 * bdb_osql_serial_check from every block-processor thread, db/toblock.c:
 * 4779-4836).  hsc_collector_check has bdb_osql_serial_check's signature and
 * contract for one read set; calls that arrive together are run as one
 * hip_serial_check_batch by one of their callers (group-commit leader: it
 * takes every queued call, up to max_batch -- 0 = 65536 -- after waiting up to
 * max_wait_us for more to arrive; 0 = no wait, batches form while the previous
 * one runs).  Thread-safe; destroy only after every caller has returned. */
typedef struct hsc_collector hsc_collector;
typedef struct hsc_collector_stats {
    uint64_t calls;      /* hsc_collector_check calls that queued */
    uint64_t batches;    /* device passes run for them */
    uint64_t max_batch;  /* largest batch */
    uint64_t busy_ns;    /* wall time with at least one batch in flight (the union of
                            the passes' intervals: busy_ns / elapsed <= 1) */
    uint64_t gate_ns;    /* leaders waiting for a device pass to end (in-flight bound) */
    uint64_t handout_ns; /* leaders waking their batches' callers */
    uint64_t pass_ns;    /* sum of the passes' durations (> busy_ns when they overlap) */
} hsc_collector_stats;
/* Small-batch path (batches of <= 1024 read sets over a narrow window: one
 * k_small_narrow launch over fine-grained host memory) phase totals since
 * the context was created: host marshal, slot copy + launch, and the wait
 * for the kernel's done word (hip_serial_check_batch releases the context
 * lock while it waits, so concurrent callers overlap). */
typedef struct hsc_small_stats_t {
    uint64_t calls, marshal_ns, launch_ns, wait_ns;
    uint64_t slot_waits; /* launches that found every slot in flight */
    uint64_t lock_ns;    /* hip_serial_check_batch calls (any path) waiting for the context lock */
} hsc_small_stats_t;
int hsc_small_stats(hsc_ctx *ctx, hsc_small_stats_t *out);
/* Marshal and batch phase totals since the context was created: marshal
 * calls (one per pipeline chunk), read sets, range probes written; the
 * parallel walk of the read sets into per-worker parts (CurRange pointer
 * walk, dictionary lookups, bound padding), the staging allocation, the SoA
 * assembly; and for the staged path the upload + launch and the wait for a
 * chunk's verdicts (device time + transfers not hidden behind the next
 * chunk's marshal). */
typedef struct hsc_batch_stats_t {
    uint64_t marshals, read_sets, ranges;
    uint64_t parts_ns, alloc_ns, assemble_ns, launch_ns, wait_ns;
} hsc_batch_stats_t;
int hsc_batch_stats(hsc_ctx *ctx, hsc_batch_stats_t *out);

int hsc_collector_create(hsc_ctx *ctx, int max_batch, int max_wait_us, hsc_collector **out);
void hsc_collector_destroy(hsc_collector *col);
int hsc_collector_check(hsc_collector *col, void *ranges, unsigned int *file,
                        unsigned int *offset, int regop_only);
int hsc_collector_get_stats(hsc_collector *col, hsc_collector_stats *out);
/* Batches allowed on the device at once (1..8; default 4): their small-batch
 * kernels run side by side on streams of their own, and the next leader
 * marshals and launches while earlier batches' kernels run.  Full checks are
 * marshalled by their own callers before they queue. */
int hsc_collector_set_inflight(hsc_collector *col, int n);
/* Read/write conflict pairs before the OR-reduction:
 * every (read set t, writer commit LSN c) such that a write committed at c
 * (c > t's snapshot) has a key inside one of t's ranges -- all the pairs the
 * A0 join would find if serial_check_callback did not stop at the first hit
 * (db/glue.c:2926-2963), i.e. the rw-antidependency edges t -> writer.
 * Sorted by (t, c), unique.  Range probes only: table locks and the host-side
 * window rules (forced verdicts) yield a verdict but no pairs.  Output arrays
 * are owned by the context until its next call. */
int hsc_rw_edges(hsc_ctx *ctx, const hsc_readsets *rs, size_t *n_pairs, const uint32_t **txn,
                 const uint64_t **writer_lsn);

/* Replicant read-set coalesce on the device: currangearr_coalesce
 * (db/sqlglue.c:305-311) -- qsort by currange_cmp (:206-242, glibc's
 * top-down merge sort), currangearr_merge_neighbor (:247-304), twice -- of
 * every read set, with the reference's quirks (a right-key swap keeps the
 * surviving range's rkeylen; a range open at both ends becomes a table lock
 * that absorbs its table's other ranges).  Output arrays are owned by the
 * context until its next coalesce; key offsets point into rs->keys.  Every
 * range must name a table (the reference's strcmp would crash otherwise).
 * Sets of >= 256 ranges whose comparator is a consistent order (no unlocked
 * range with a present-but-empty lower key; locked ranges open at both ends)
 * sort and merge level-parallel with the same result; HSC_CO_SERIAL=1 in the
 * environment forces the per-set path (testing). */
typedef struct hsc_coalesced {
    int ntxn;
    const int64_t *txn_off;   /* [ntxn+1] */
    const int32_t *table, *idxnum, *lflag, *rflag, *islocked, *lkeylen, *rkeylen;
    const uint64_t *lkey_off, *rkey_off;
} hsc_coalesced;
int hsc_coalesce_readsets(hsc_ctx *ctx, const hsc_readsets *rs, hsc_coalesced *out);

/* Host threads that marshal a batch (0 = the box's CPUs: the affinity mask
 * capped by the cgroup CPU quota; HSC_THREADS overrides that default).  A
 * batch of >= 65536 read sets runs as a pipeline of 32768-set chunks over two
 * pinned staging sets: one chunk is marshalled while the previous one is
 * uploaded, joined and read back. */
int hsc_set_threads(hsc_ctx *ctx, int n);

/* Flat read sets (snapshots in rs->snap); rc_out[ntxn]; full checks only. */
int hsc_check_readsets(hsc_ctx *ctx, const hsc_readsets *rs, int *rc_out);

/* ---- marshalling + device probe (what the checks lower to) -------------- */
typedef struct hsc_marshalled {
    size_t n, n_lock, n_txn;
    int words;
    uint64_t *lo, *hi;        /* host [words][n] */
    uint32_t *gid;
    uint64_t *snap;
    uint32_t *txn;
    uint32_t *lock_table;
    uint64_t *lock_snap;
    uint32_t *lock_txn;
    uint8_t *forced;          /* [n_txn] verdicts decided on the host (1/0)   */
} hsc_marshalled;
/* Marshal flat read sets against the current window into probe SoA (host
 * memory owned by the library; valid until the next marshal / ctx destroy). */
int hsc_marshal_readsets(hsc_ctx *ctx, const hsc_readsets *rs,
                         const hsc_marshalled **out);
/* The host half of hip_serial_check_batch: CurRangeArr* ranges[n] (none
 * NULL) with snapshot LSNs snaps[n], marshalled as hsc_marshal_readsets does
 * (works on host-only contexts; the timing harness of the batch entry). */
int hsc_marshal_arrs(hsc_ctx *ctx, void *const *ranges, const uint64_t *snaps, int n,
                     const hsc_marshalled **out);
/* Run the join for a device-resident batch, asynchronously on the stream. */
int hsc_probe_device(hsc_ctx *ctx, const hsc_probe_batch *b);
/* verdict bytes -> bitmap (e.g. after a cross-GPU max all-reduce). */
int hsc_pack_verdicts(hsc_ctx *ctx, const uint8_t *verdict, size_t n_txn,
                      uint64_t *bitmap);
/* Multi-GPU verdict merge: out_dev[w] = OR over k < nparts of
 * parts_dev[k * words + w] -- the per-shard verdict bitmaps after an
 * all-gather (N x n_txn / 8 bytes per rank instead of a byte-wise max
 * all-reduce of N x n_txn).  Asynchronous on the context's stream. */
int hsc_or_bitmaps(hsc_ctx *ctx, const uint64_t *parts_dev, int nparts, size_t words,
                   uint64_t *out_dev);
int hsc_synchronize(hsc_ctx *ctx);
int hsc_get_timing(hsc_ctx *ctx, hsc_timing *t);
/* Enable per-kernel HIP event timing of probes (adds event records). */
int hsc_enable_timing(hsc_ctx *ctx, int on);

/* ---- multi-GPU context ---------------------------------
 * A multi context is an hsc_ctx: hip_serial_check_batch,
 * hip_bdb_osql_serial_check, hsc_collector_*, hsc_check_readsets /
 * _serial, hsc_window_ingest_log / _raw, hsc_window_append[_log|_raw],
 * hsc_register_group and the window accessors take it unchanged.  Its window
 * is cut into `world` contiguous pieces of the composite key space (gid, key
 * words) -- member d holds the keys K with sp[d-1] <= K < sp[d] -- one per
 * member context.  The context itself keeps the log decode, dictionaries and
 * window rules and marshals every batch on the host.  A range [g||lo, g||hi]
 * goes to the members whose pieces it overlaps (owner(g||lo) ..
 * owner(g||hi)), table locks to member 0 (it holds the global table maxima).
 * In one process the drop-in entries route while marshalling: each member
 * that holds any probe of the batch checks its share through its own one-GPU
 * path (the small-batch kernel for a lone call), and the verdicts are OR-ed.
 * Batches already resident on the GPUs are either routed there
 * (hsc_multi_probe_device: route kernels, then an exchange -- direct stores
 * between members of one process over xGMI peer access, RCCL grouped
 * ncclSend / ncclRecv between processes) or arrive routed
 * (hsc_multi_probe_routed); every member joins its probes against its piece
 * and the members' verdict bitmaps are OR-ed per read-set owner.  A per-rank
 * context (one process per GPU, hsc_multi_create_rank; librccl loaded at run
 * time) routes its drop-in batches on the devices.  Verdicts equal those of
 * one context holding the whole window.  Not on a multi
 * context: hsc_set_stream, hsc_probe_device, hsc_window_ingest_device (ingest
 * the members directly, then hsc_multi_adopt), hsc_rw_edges, the graph and
 * coalesce calls (use a member). */
/* n members on devices[0..n-1] (n <= 16; a device may repeat) in this
 * process.  Returns the context in *out (destroy with hsc_ctx_destroy). */
int hsc_multi_create(const int *devices, int n, hsc_ctx **out);
/* One member per process: this process is member `rank` of `world` on
 * `device`.  ids: the bytes hsc_multi_unique_ids wrote on one rank (every
 * rank passes the same ones; 2 x 128 bytes: one RCCL communicator per lane). */
int hsc_multi_unique_ids(void *out, size_t bytes);
int hsc_multi_create_rank(int device, int rank, int world, const void *ids, size_t bytes,
                          hsc_ctx **out);
int hsc_multi_world(hsc_ctx *ctx);   /* members of the partition */
int hsc_multi_rank(hsc_ctx *ctx);    /* global index of this process's first member */
int hsc_multi_local(hsc_ctx *ctx);   /* members in this process */
hsc_ctx *hsc_multi_member(hsc_ctx *ctx, int i);  /* i < hsc_multi_local */
/* The world - 1 ascending splitters (gid[S], words[W][S] big-endian key
 * words); default: equal-row quantiles of the ingested log's rows.  A
 * host-staged window is re-partitioned at the next check. */
int hsc_multi_set_splitters(hsc_ctx *ctx, size_t S, const uint32_t *gid, const uint64_t *words,
                            int W);
/* The members' windows, ingested directly (hsc_window_ingest_device on
 * hsc_multi_member, each holding exactly its piece's rows), become the
 * context's window; table maxima are max-merged over all members (an RCCL
 * all-reduce across ranks).  Collective on a per-rank context.  HSC_ESTATE
 * without splitters (world > 1); HSC_EINVAL when the members' key widths
 * differ or a member's first or last key lies outside its piece.  Appends
 * then go to the members (the context's append entries return HSC_ESTATE). */
int hsc_multi_adopt(hsc_ctx *ctx);
/* In-process contexts: HSC_MULTI_DIRECT (default: the device routing stores
 * into the other members' probe columns, the merge reads their bitmaps) or
 * HSC_MULTI_LOOPBACK (the per-rank form with peer copies in place of RCCL:
 * send blocks, k_route_unpack, owner slices gathered and OR-ed -- what a
 * per-rank context runs, on one process). */
#define HSC_MULTI_DIRECT 0
#define HSC_MULTI_LOOPBACK 1
int hsc_multi_set_transport(hsc_ctx *ctx, int transport);
/* Window placement.  HSC_MULTI_PIECES: each member holds its key-range piece
 * (the splitters); a batch's probes go to the pieces they overlap and the
 * verdicts are OR-ed.  HSC_MULTI_REPLICAS: every member holds the whole
 * window (builds and appends go to every member); a drop-in batch that fits
 * the small path goes whole to ONE member (the one with the fewest batches in
 * flight, round robin among equals: one member kernel per call), a larger
 * one is cut into per-member slices of its read sets, each checked by one
 * member against its replica -- no routing, no exchange, no OR across
 * members.  HSC_MULTI_AUTO (default): replicas when a host-staged window's
 * rows x (8 W + 16) bytes fit an eighth of the smallest member's device
 * memory, else pieces; an adopted window is pieces unless REPLICAS was set
 * (hsc_multi_adopt then needs every member to hold the same rows, no
 * splitters).  A host-staged window is re-placed at the next check.
 * hsc_multi_mode returns the placement in force (PIECES or REPLICAS). */
#define HSC_MULTI_AUTO 0
#define HSC_MULTI_PIECES 1
#define HSC_MULTI_REPLICAS 2
int hsc_multi_set_mode(hsc_ctx *ctx, int mode);
int hsc_multi_mode(hsc_ctx *ctx);
/* Device-resident batches, one per local member (pointers on its GPU), each
 * numbering its own read sets 0..b[i].n_txn-1: routed, probed and merged;
 * b[i].bitmap (ceil(n_txn / 64) words) receives the merged verdict bits of
 * member i's read sets.  lane (0 or 1): scratch set, so two batches can be in
 * flight; a lane is reused after its previous batch finished.  Returns once
 * the work is enqueued (the host waits for the routing counts only).
 * Collective on a per-rank context. */
int hsc_multi_probe_device(hsc_ctx *ctx, const hsc_probe_batch *b, int lane);
/* Device-resident batches routed when they were marshalled, one per local
 * member: b[i] holds exactly the probes whose [lo, hi] overlaps member i's
 * piece (hsc_multi_marshal_routed; table locks on member 0 only), read sets
 * numbered batch-wide: owner o owns [owner_base[o], owner_base[o + 1])
 * (world + 1 ascending multiples of 64 from 0), b[i].bitmap receives the
 * merged bits of member i's own read sets.  Every member probes its batch in
 * place; the bitmaps are OR-ed per owner (RCCL send / receive of the owners'
 * slices across ranks).  No routing and no probe exchange on the devices.
 * lane as for hsc_multi_probe_device; collective on a per-rank context. */
int hsc_multi_probe_routed(hsc_ctx *ctx, const hsc_probe_batch *b, const uint64_t *owner_base, int lane);
/* Marshal rs (hsc_marshal_readsets) and route it on the host: *out = the
 * columns of member `member` (read-set numbers + txn_base; table locks when
 * member == 0), host memory valid until the next marshal on ctx.  forced =
 * the whole batch's host-decided verdicts. */
int hsc_multi_marshal_routed(hsc_ctx *ctx, const hsc_readsets *rs, int member, uint32_t txn_base,
                             const hsc_marshalled **out);
/* member >= 0 above; member = -1 routes the batch to every member, *out =
 * member 0's columns and hsc_multi_routed_member the others' (same life). */
int hsc_multi_routed_member(hsc_ctx *ctx, int member, const hsc_marshalled **out);
/* Events around every member's probe of the routed pipelines (diagnostics,
 * per-member imbalance); out[i] = local member i's probe ms of the last batch
 * (waits for it). */
int hsc_multi_enable_timing(hsc_ctx *ctx, int on);
int hsc_multi_member_probe_ms(hsc_ctx *ctx, float *out, int n);
/* Host routing of the drop-in entries: out[8] = calls, member checks run,
 * probes routed, probe rows placed (> probes when ranges straddle pieces),
 * mean us routing per call, world, mean us launching the members, mean us
 * waiting for their verdicts. */
int hsc_multi_route_stats(hsc_ctx *ctx, double out[8]);
/* out[4]: routed batches, probes routed (sources), probe rows received
 * (destinations; > probes when ranges straddle pieces), local members. */
int hsc_multi_stats(hsc_ctx *ctx, uint64_t out[4]);
/* counts[s * world + d]: probes member s sent member d in the last batch. */
int hsc_multi_last_counts(hsc_ctx *ctx, uint32_t *counts, int n);
/* Host time per routed batch (diagnostics): out[0] device-routed batches,
 * then mean us enqueueing the lane waits, launching the route counts,
 * waiting for the counts the device publishes, enqueueing the rest of the
 * batch; out[5] hsc_multi_probe_routed batches, out[6] mean us enqueueing
 * one. */
int hsc_multi_phase_stats(hsc_ctx *ctx, double out[7]);
/* hsc_multi_probe_routed's host time per batch, split (us): out[0] batches,
 * out[1] lane_acquire (the members' cross-lane event waits), out[2] the
 * members' probe launches, out[3] the owners' merges and done events.  An
 * enqueue blocks when a hardware queue is full, so each phase holds that
 * wait too; bench.py times calls that start on an idle GPU for the pure
 * enqueue cost. */
int hsc_multi_routed_phase_stats(hsc_ctx *ctx, double out[4]);

/* ---- OSQL_SERIAL wire path --------------------------------------------
 * Decode only: *out points at context-owned read sets, valid until the next
 * decode on this context (HSC_EINVAL names the malformed message). */
int hsc_decode_serial(hsc_ctx *ctx, const hsc_serial_msgs *msgs, const hsc_readsets **out);
/* Decode + full check (regop_only = 0) of every message: rc_out[nmsg]. */
int hsc_check_serial(hsc_ctx *ctx, const hsc_serial_msgs *msgs, int *rc_out);

/* ---- dependency graph + SCC ------------------------
 * History of committed transactions as micro-ops (host pointers): txn ids
 * are commit order (a key's version order = its writers' commit order); a
 * read records the writer txn of the version it observed (-1 = initial), as
 * a Jepsen rw-register history with unique write values does.  Edges (Adya):
 * ww consecutive writers of a key, wr writer -> reader, rw reader -> next
 * writer after the observed version; self edges dropped, parallel edges
 * merged (type bits: 1 ww, 2 wr, 4 rw).  scc_out[v] = the largest txn id of
 * v's strongly connected component; a component with more than one txn is a
 * dependency cycle (G1c / G2 anomaly). */
typedef struct hsc_history {
    size_t nops;
    uint32_t ntxn;
    const uint32_t *txn;
    const uint64_t *key;
    const uint8_t *is_write;
    const int64_t *observed;
} hsc_history;

typedef struct hsc_graph_stats {
    uint64_t edges;
    uint64_t ww, wr, rw;          /* edges carrying each type bit              */
    uint32_t nontrivial_sccs;     /* components with >= 2 txns                 */
    uint32_t txns_in_cycles;
    uint32_t rounds, iterations;  /* colouring rounds / frontier steps         */
    float build_ms, scc_ms;       /* device time                               */
    uint32_t cut_nodes;           /* hsc_dep_graph_scc_cut: nodes of the cover */
} hsc_graph_stats;

int hsc_dep_graph_scc(hsc_ctx *ctx, const hsc_history *h, uint32_t *scc_out,
                      hsc_graph_stats *stats);
/* Edges of the last full build, sorted by (src, dst): copies min(cap, n)
 * (n = 0 after a raw build). */
int hsc_dep_graph_edges(hsc_ctx *ctx, uint32_t *src, uint32_t *dst, uint32_t *type,
                        size_t cap, size_t *n);

/* Sharded SCC (config 4 over N GPUs).  Every WW/WR/RW edge belongs to one
 * key, so a history split by key gives each shard an exact part of the edge
 * set.  Txn ids are commit order; a cycle always contains a backward edge
 * (src > dst) and all its nodes lie inside [dst, src] of its backward edges,
 * so components of >= 2 txns live in the graph induced on the "cover" (the
 * nodes inside some backward edge's interval).  Per shard: build, cover
 * (u8 per txn, merged over shards with a MAX all-reduce), cut (the shard's
 * edges between covered nodes, exchanged with an all-gather), then the SCC of
 * the union of the cuts -- the same scc[] as hsc_dep_graph_scc of the whole
 * history.  Pointers named *_dev are device memory of the context's GPU. */
/* flags: HSC_GRAPH_FULL = sorted unique edges with types and CSR / CSC (what
 * hsc_dep_graph_edges returns, stats.edges/ww/wr/rw filled); 0 = the raw edge
 * rows only (duplicates, no sort: all cover / cut need; stats.build_ms only). */
#define HSC_GRAPH_FULL 1
/* HSC_GRAPH_NO_RW: reads give their wr edge only; the rw edges come from
 * staged pairs (hsc_dep_graph_stage_rw_pairs). */
#define HSC_GRAPH_NO_RW 2
int hsc_dep_graph_build(hsc_ctx *ctx, const hsc_history *h, int flags, hsc_graph_stats *stats);
/* The same from device-resident ops (observed: writer txn, 0xFFFFFFFF =
 * initial version); ops naming a txn >= ntxn -> HSC_EINVAL. */
int hsc_dep_graph_build_device(hsc_ctx *ctx, size_t nops, uint32_t ntxn, const uint32_t *txn_dev,
                               const uint64_t *key_dev, const uint8_t *is_write_dev,
                               const uint32_t *observed_dev, int flags, hsc_graph_stats *stats);
/* The validator's rw pairs as graph edges: the pairs of
 * the last hsc_rw_edges call -- still on the device -- become rw edges
 * readset_txn[t] -> commit_txn[i] (commit_lsn[i] == the writer's commit LSN;
 * commit_lsn sorted ascending; host arrays) and join the next
 * hsc_dep_graph_build / _build_device (merged with its own edges, type bits
 * OR-ed; self edges dropped).  A pair whose read set or LSN is not mapped ->
 * HSC_EINVAL.  Pairs name every writer after the snapshot, not only the next
 * version: the extra edges t -> later writers follow the ww chain and leave
 * the components unchanged. */
int hsc_dep_graph_stage_rw_pairs(hsc_ctx *ctx, uint32_t nrs, const uint32_t *readset_txn,
                                 size_t ncommit, const uint64_t *commit_lsn,
                                 const uint32_t *commit_txn);
/* scc_out[ntxn] of the last HSC_GRAPH_FULL build (stats as hsc_dep_graph_scc,
 * build_ms 0). */
int hsc_dep_graph_scc_built(hsc_ctx *ctx, uint32_t *scc_out, hsc_graph_stats *stats);
/* cover_dev[ntxn of the last build] := 1 inside a backward edge's interval. */
int hsc_dep_graph_cover(hsc_ctx *ctx, uint8_t *cover_dev);
/* Edges of the last build with both ends covered, as rows src << 32 | dst
 * (sorted): *m of them, min(cap, *m) copied to rows_dev (NULL: count only). */
int hsc_dep_graph_cut(hsc_ctx *ctx, const uint8_t *cover_dev, uint64_t *rows_dev, size_t cap,
                      size_t *m);
/* scc_dev[ntxn] := largest txn of each txn's component in the graph whose
 * only edges between covered nodes are rows_dev[m] (~0 rows are padding);
 * uncovered txns are their own component.  HSC_EINVAL if a row leaves the
 * cover.  Leaves the last build's edges in place (own buffers). */
int hsc_dep_graph_scc_cut(hsc_ctx *ctx, uint32_t ntxn, const uint8_t *cover_dev,
                          const uint64_t *rows_dev, size_t m, uint32_t *scc_dev,
                          hsc_graph_stats *stats);

/* Sharded SCC on a multi context (config 4 over N GPUs behind the C ABI):
 * ops[i] = local member i's key shard of the history, device-resident on its
 * GPU (every WW/WR/RW edge belongs to one key).  Per member: raw build and
 * cover; covers OR-ed (RCCL MAX all-reduce across ranks, an OR over peer
 * buffers in one process); cuts; the union of the cuts (RCCL all-gather,
 * padded with ~0 rows, across ranks; peer copies to member 0 in one
 * process); its colouring SCC.  scc_dev[i] (ntxn u32 on member i's GPU;
 * scc_dev[0] required, others may be NULL) = the largest txn of each txn's
 * component, as hsc_dep_graph_scc of the whole history.  stats: member 0's
 * SCC stats, build_ms = the slowest local build, edges = rows of the cut
 * union.  Collective on a per-rank context. */
typedef struct hsc_ops_dev {
    size_t nops;
    const uint32_t *txn;       /* [nops] */
    const uint64_t *key;       /* [nops] */
    const uint8_t *is_write;   /* [nops] */
    const uint32_t *observed;  /* [nops] writer txn, 0xFFFFFFFF = initial version */
} hsc_ops_dev;
int hsc_multi_graph_scc(hsc_ctx *ctx, const hsc_ops_dev *ops, uint32_t ntxn, uint32_t *const *scc_dev,
                        hsc_graph_stats *stats);
/* Host ms of the last hsc_multi_graph_scc: build + cover, cover merge, cuts +
 * their union, SCC. */
int hsc_multi_graph_phase_ms(hsc_ctx *ctx, double out[4]);

/* ---- harness support (tests / bench; not on the check path) --------------
 * CurRangeArr objects as comdb2 holds a received read set (db/comdb2.h:1105-1124;
 * strdup'd table names, malloc'd keys, serial_readset_get db/osqlcomm.c:948-993),
 * one per read set of rs: *out = void *[ntxn] of hsc_currangearr *. */
int hsc_currangearrs_build(const hsc_readsets *rs, void ***out);
void hsc_currangearrs_free(void **arrs, int n);
/* nthreads caller threads, each checking read sets i = t, t + nthreads, ...
 * of arrs[n] `rounds` times with its own (file, offset) copies of the set's
 * snapshot -- through col (hsc_collector_check) when col != NULL, else one
 * hip_bdb_osql_serial_check per call.  rc_out[n] = last verdicts; per-call
 * latencies summarised in *res. */
typedef struct hsc_concurrent_result {
    double seconds;                             /* wall time of all threads */
    uint64_t calls;
    double lat_mean_us, lat_p50_us, lat_p99_us;  /* per call */
} hsc_concurrent_result;
int hsc_harness_concurrent(hsc_ctx *ctx, hsc_collector *col, void *const *arrs, int n,
                           int nthreads, int rounds, int regop_only, int *rc_out,
                           hsc_concurrent_result *res);
/* The master's commit protocol (db/toblock.c:4757-4836) replayed by nthreads
 * threads over a stream of events: events[k] >= 0 -- txn events[k] begins (its
 * CurRangeArr's snapshot := hsc_window_end); events[k] < 0 -- txn ~events[k]
 * commits.  Threads take events in order (a commit waits for its txn's begin).
 * A commit: commit_lock (a pthread rwlock) read-locked, released and
 * write-locked; while hip_bdb_osql_serial_check(regop_only = 1) on
 * &arr->file / &arr->offset says a newer commit exists: unlock, full check
 * (regop_only = 0; conflict -> abort, rc 1), write-lock again; then the txn's
 * writes are appended at commit LSN hsc_window_end + 1 (hsc_window_append)
 * and the lock released.  Per txn: rc_out (0 committed, 1 aborted),
 * commit_seq (its commit's index, -1 if aborted or without writes),
 * snap_out (the snapshot it began with), check_end_out (the end LSN its last
 * full check returned, 0 if none ran). */
typedef struct hsc_protocol_txn {
    void *arr;                /* CurRangeArr* (file / offset set at begin)   */
    const hsc_write *writes;  /* the txn's writes (commit_lsn ignored)       */
    int nwrites;
} hsc_protocol_txn;
typedef struct hsc_protocol_result {
    double seconds;           /* first event to last commit                  */
    uint64_t commits, aborts, regop_probes, full_checks;
    double regop_p50_us, regop_p99_us, regop_p999_us, regop_max_us;
    double full_p50_us, full_p99_us;
    double hold_p50_us, hold_p99_us;  /* commit_lock write-held per commit   */
    double commit_p50_us, commit_p99_us;  /* commit event: first lock to done */
} hsc_protocol_result;
int hsc_harness_commit_protocol(hsc_ctx *ctx, const hsc_protocol_txn *txns, int ntxn,
                                const int *events, int nevents, int nthreads, int *rc_out,
                                int64_t *commit_seq, uint64_t *snap_out, uint64_t *check_end_out,
                                hsc_protocol_result *res);

#ifdef __cplusplus
}
#endif
#endif /* HIP_SERIAL_H */
