// hsc_internal.h -- device data layout shared by the host driver (hsc_host.cpp)
// and the gfx950 kernels (hsc_kernels.hip).
//
// Resident write window (one per context / GPU), all struct-of-arrays in HBM:
//   words[j * cap + i]  key word j of row i (big-endian bytes 8j..8j+7 of the
//                       zero-padded key, as a native u64: numeric order of the
//                       words == memcmp order of the bytes)
//   lsn[i]              max commit (regop) LSN of that (group, key)
//   gid[i]              key group = (table, index, key length)
//   rows sorted by (gid, words[0..W-1]) and unique
//   gstart/gend[g]      row span of group g
//   tmax[l * ntiles + t] max lsn over tiles [t, t + 2^l)  (sparse table)
//   sp_g[t], sp_w[j * ntiles + t]  group / key words of tile t's first row
//   table_max[tid]      max commit LSN of any write to table tid (dta too)
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/hip_serial.h"

namespace hsc {

// Growable device buffer (reallocated only when a larger size is needed).
// growth headroom of a device buffer: want / dbuf_slack() more (default 2;
// HSC_DBUF_SLACK=8 the r05 eighth, an A/B)
inline size_t dbuf_slack()
{
    static const size_t k = [] {
        const char *v = getenv("HSC_DBUF_SLACK");
        const long x = v ? atol(v) : 2;
        return (size_t)(x >= 1 ? x : 2);
    }();
    return k;
}
struct DBuf {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t want)
    {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        // half again as much: a window that keeps growing (folds of a commit
        // stream) reallocates O(log n) times -- a hipFree synchronises the
        // device, which a fold's worker thread must not do on every fold
        size_t b = want + want / dbuf_slack() + 256;
        hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) bytes = b;
        return e;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return (T *)p; }
};

constexpr int kMaxWords = 64;       // MAXKEYLEN 512 B (bbinc/cdb2_constants.h:33)
constexpr int kTopCap = 6144;       // splitter prefixes held in LDS by the locate kernel
constexpr int kLocateThreads = 512;
constexpr int kMaxChunks = 512;     // probe chunks (locate / scatter workgroups)
constexpr int kHistCap = 8192;      // tiles whose bucket counters fit in LDS
constexpr int kDirectPerTile = 8;   // narrow: direct probe below 8 ranges per tile
constexpr int kJoinThreads = 512;
constexpr int kJoinChunk = 1024;    // join records per workgroup
constexpr uint32_t kTileCap = 1024; // narrow tiles: records per tile bucket before it spills
constexpr int kLdsJoinBudget = 65536;

// Probe codes written by the locate kernel: a | b << 31 | kind << 62.
constexpr uint64_t kKindFull = 1, kKindSplit = 2;
// Join record kinds (top two bits of the record meta word).
constexpr uint32_t kRecFull = 1, kRecHead = 2, kRecTail = 3;

struct WinView {
    const uint64_t *words;
    size_t stride;            // cap of the words array (row stride per word)
    const uint64_t *lsn;
    const uint32_t *gid;
    const uint32_t *gstart, *gend;
    const uint64_t *tmax;
    const uint64_t *table_max;
    const uint32_t *sp_g;     // [ntiles] group of each tile's first row
    const uint64_t *sp_w;     // [W][ntiles] key words of each tile's first row
    uint32_t n, ntiles, ntables;
    int W, log2T, levels;
    int gbits;                // bits of gid in a splitter prefix (key_prefix)
    int compact;              // words are per-group compact codes (hsc_compact.hip)
};

struct ProbeView {
    const uint64_t *lo, *hi;
    const uint32_t *gid;
    const uint64_t *snap;
    const uint32_t *txn;
    const uint32_t *lock_table;
    const uint64_t *lock_snap;
    const uint32_t *lock_txn;
    uint32_t n, n_lock;
};

// Join-record layout: rec_words u64 per record = lo[W] hi[W] snap meta,
// meta = txn | lb << 32 | ub << 44 | kind << 62 ([lb, ub) = the probe's
// group rows inside the tile).  2W+2 words -> 16-byte multiple.
__host__ __device__ inline int rec_words(int W) { return 2 * W + 2; }
#ifndef HSC_REC_PAD
#define HSC_REC_PAD 0
#endif
// Record stride in u64: with HSC_REC_PAD records start on 64-byte sectors,
// so a scattered record is written as whole sectors.
__host__ __device__ inline int rec_stride(int W)
{
    return HSC_REC_PAD ? (rec_words(W) + 7) & ~7 : rec_words(W);
}

constexpr int kMaxTileRows = 4096;  // window capacity is a multiple of this

// Tile size: largest power of two whose keys + lsn fit the LDS budget.
inline int tile_log2(int W)
{
    int l = 12;
    while (l > 6 && ((size_t)1 << l) * (size_t)(8 * W + 8) > (size_t)kLdsJoinBudget)
        --l;
    return l;
}

// ---- launchers (hsc_kernels.hip) -------------------------------------------
// Ingest.
hipError_t radix_sort_rows(int W, size_t n, uint32_t *gid, uint64_t *words, uint64_t *lsn,
                           size_t stride, uint32_t *gid_alt, uint64_t *words_alt,
                           uint64_t *lsn_alt, void *scratch, size_t scratch_bytes,
                           bool *result_in_alt, uint64_t *vary_mask, hipStream_t s);
size_t radix_scratch_bytes(size_t n, int W);
// vary[j] (host, j <= W): bits of word j / of the gid (j == W) that differ
// between rows, and with lsn_span the rows' min / max LSN (0, 0 if every LSN
// is 0) -- one kernel + readback; scratch >= 8 (W + 3) bytes
hipError_t vary_mask_rows(int W, size_t n, const uint32_t *gid, const uint64_t *words, size_t stride,
                          void *scratch, uint64_t *vary, hipStream_t s, const uint64_t *lsn = nullptr,
                          uint64_t *lsn_span = nullptr, uint64_t *lsn_vary = nullptr);
// radix_sort_rows with the vary masks already known
hipError_t radix_sort_known(int W, size_t n, uint32_t *gid, uint64_t *words, uint64_t *lsn,
                            size_t stride, uint32_t *gid_alt, uint64_t *words_alt,
                            uint64_t *lsn_alt, void *scratch, size_t scratch_bytes,
                            bool *result_in_alt, const uint64_t *vary, hipStream_t s);
hipError_t dedupe_rows(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                       const uint64_t *lsn, size_t stride_in, uint32_t *gid_out,
                       uint64_t *words_out, uint64_t *lsn_out, size_t stride_out,
                       uint32_t *flags, void *scratch, size_t scratch_bytes,
                       uint32_t *d_count, hipStream_t s);
// dedupe_rows with the last-of-key flags already in flags (scanned in place)
hipError_t dedupe_flagged(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                          const uint64_t *lsn, size_t stride_in, uint32_t *gid_out,
                          uint64_t *words_out, uint64_t *lsn_out, size_t stride_out,
                          uint32_t *flags, void *scratch, size_t scratch_bytes,
                          uint32_t *d_count, hipStream_t s);
// The packed writers' layout (hsc_graph.hip): every distinct writer is one
// u64 pk = compress(key) << tb | compress(txn), ascending; a directory of
// 2^D buckets over [pk[0], pk[nu - 1]]
struct PairPack {
    uint64_t km, tm;          // the writers' varying key / txn bits
    uint64_t kc, tc;          // their constant bits (the same in every writer)
    uint64_t kmv[6], tmv[6];  // compress moves
    uint64_t base, last;      // pk[0], pk[nu - 1]
    int tb, D, shift;         // txn bits, directory bits, bucket = (pk - base) >> shift
};
// Packed-key sort (hsc_ingest.hip): rows whose varying key bits plus a row
// index fit 64 bits sort as single words.
constexpr int kPackMaxWords = 8;
constexpr int kPackLimbs = kPackMaxWords + 1;
struct PackPlan {
    int W, I, B, nl;            // key words, index bits, packed key bits, varying limbs
    int limb[kPackLimbs];       // most significant first: W = the gid, j < W = word j
    int bits[kPackLimbs];
    uint64_t mask[kPackLimbs];  // the limb's varying bits
    uint64_t mv[kPackLimbs][6]; // their compress moves
    int skip = 0;               // low packed bits the rows are already ordered by (stable
                                // passes skip them: a txn-ordered writer list sorted by key)
    // the low I bits hold the row's LSN compressed by its varying bits instead
    // of the row index (the passes never sort them: equal keys keep input
    // order either way) -- the unpack expands it, no gather by row index
    bool lsn_packed = false;
    uint64_t lmask = 0, lconst = 0;  // the LSNs' varying / constant bits
    uint64_t lmv[6] = {};
};
// false: does not fit.  index = false: no row index (I = 0) -- the packed
// key is the whole row (no LSN to gather; equal rows are duplicates)
// lsn_bits (index only): {varying, constant} bits of the rows' LSNs -- when
// they fit beside the key bits they take the index's place (PackPlan::lsn_packed)
bool packed_plan(int W, size_t n, const uint64_t *vary, PackPlan *P, bool index = true,
                 const uint64_t *lsn_bits = nullptr);
size_t packed_scratch_bytes(size_t n);
// The packed sort with the dedupe fused into the unpack: every version to
// (gid_o, words_o, lsn_o) (gid_o null: not written; lsn null: LSNs 0, or with no index bits the
// packed keys themselves), the
// distinct rows to (gid_d, words_d) -- which may
// be the input gid / words; gid_d null: not written -- and to *lsn_d = whichever of k0 / k1 the sorted
// keys did not end in; d_count[0] = distinct rows
hipError_t packed_sort_dedupe(const PackPlan &P, size_t n, const uint32_t *gid, const uint64_t *words,
                              const uint64_t *lsn, size_t stride, uint64_t *k0, uint64_t *k1,
                              uint32_t *gid_o, uint64_t *words_o, uint64_t *lsn_o, size_t stride_o,
                              uint32_t *gid_d, uint64_t *words_d, size_t stride_d,
                              uint64_t **lsn_d, uint32_t *d_count, void *scratch,
                              size_t scratch_bytes, hipStream_t s, uint32_t *err = nullptr,
                              uint64_t *ww_rows = nullptr, const PairPack *ww_pp = nullptr);
// (ww_rows: for a key-only sort of packed (key, txn) writers -- no rows, no
// LSNs, no index -- also each distinct writer's ww row, decoded by ww_pp)
// (err != null: the one-sweep passes -- no count pass or scan per digit --
// with *err set if a tile's look-back stalled; the caller fails the build)
size_t scan_scratch_bytes(size_t n);
// (src != null: the tile-max sparse table derived from one over the same rows'
// LSNs with tiles 2^shift times shorter (shift 0 or 1, at least as many
// levels) instead of rebuilt -- the narrow tile view's, whose LSNs are the
// window's)
// (lsn16 != null: the same rows' LSN maxima per 16 rows -- the narrow
// index's level 1 -- read instead of every row's LSN for the tile maxima)
struct TmaxFrom {
    const uint64_t *src = nullptr;
    uint32_t ntiles = 0;
    int shift = 0;
    const uint64_t *lsn16 = nullptr;
};
hipError_t build_summaries(const WinView &w, uint32_t *gstart, uint32_t *gend, int ngroups,
                           uint64_t *tmax, const uint32_t *group_table,
                           uint64_t *table_max, uint32_t *sp_g, uint64_t *sp_w, hipStream_t s,
                           const TmaxFrom &from = TmaxFrom{});
// Probe.
struct ProbeWork {
    uint64_t *code;        // [n] a | b << 31 | kind << 62
    uint32_t *hist;        // [G][ntiles] per-chunk record counts -> offsets
    uint32_t *counts;      // [ntiles + 1] records per tile
    uint32_t *bucket_off;  // [ntiles + 1] (wide pipeline)
    uint32_t *cursor;      // [ntiles] (global-atomic mode, ntiles > kHistCap)
    uint32_t *item_off;    // [ntiles + 1]
    uint32_t *item_tile;   // [max items]
    uint4 *item_desc;      // [max items] {tile, first record, end record, 0}
    uint64_t *recs;        // join records
    uint32_t G, chunk;     // probe chunks (one workgroup each in locate/scatter)
    int lds_mode;          // ntiles <= kHistCap: LDS histograms, no global atomics
    uint64_t *stamps;      // diagnostic builds (HSC_STAMPS): [kernel][block][8] s_memtime
    // chunk-sorted records (narrow / compact tiles, no scatter pass): chunk g's records sit in
    // its own area of 2 * chunk records sorted by tile; cst[t][g] = where tile
    // t's run starts in it; join items are tile-local record ranges
    uint16_t *cst;
    uint32_t *cm;  // [G][round4(ntiles)] chunk-major (run start << 16 | count), the locate's rows
    // the batch's verdict bitmap, built in place of a pack pass (narrow and
    // compact tiles): k_plan_s writes the locate's flags as whole words, the
    // join ORs its hits in (null: verdict bytes only)
    uint64_t *bitmap;
};
// Diagnostic phase stamps (HSC_STAMPS builds only): thread 0 of a block
// records s_memtime at phase boundaries into a buffer of its own (never an
// output), read back and summarized by the host.
#ifdef HSC_STAMPS
#define HSC_STAMP(work, kern, k)                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0 && (work).stamps)                                            \
            (work).stamps[((size_t)(kern) * 8192 + blockIdx.x) * 8 + (k)] =               \
                __builtin_amdgcn_s_memtime();                                             \
    } while (0)
#else
#define HSC_STAMP(work, kern, k) \
    do {                         \
    } while (0)
#endif
hipError_t launch_locate(const WinView &w, const ProbeView &p, const ProbeWork &work,
                         uint8_t *verdict, hipStream_t s);
hipError_t launch_plan(const WinView &w, const ProbeWork &work, hipStream_t s);
hipError_t launch_scatter(const WinView &w, const ProbeView &p, const ProbeWork &work,
                          hipStream_t s);
hipError_t launch_join(const WinView &w, const ProbeWork &work, uint32_t max_items,
                       uint8_t *verdict, hipStream_t s);
// Narrow layout (hsc_narrow.hip): key64[i] = (K_i - K_0) >> s for the
// composite key K = gid || words (limb 0 = gid, limb j+1 = word j), s = tz
// bits of limb lw + every limb after lw; a 16-ary tree of key levels and a
// parallel tree of LSN maxima.
constexpr int kMaxLevels = 16;
struct NarrowView {
    const uint64_t *keys;      // key levels; level l at keys + off[l], len[l] entries
    const uint64_t *maxs;      // LSN max levels (level 0 = row LSNs), same offsets
    uint64_t off[kMaxLevels];
    uint32_t len[kMaxLevels];  // multiples of 16; the top level has 16 entries
    int levels;
    int lds_from;              // levels >= lds_from are staged in LDS
    uint32_t lds_entries;
    const uint64_t *base;      // [1 + W] limbs of K_0 (device)
    int W, lw, tz;
    uint32_t n;
    const uint64_t *table_max;
    uint32_t ntables;
    // compressed codes (comp != 0): the rows' varying bits of every limb
    // (gid, words) packed MSB first, minus row 0's -- for windows whose rows
    // differ in <= 62 bits spread beyond one 62-bit span (composite keys).
    // cmeta[8 l ..]: limb l's mask, pattern (row 0), 6 compress moves.
    int comp;
    const uint64_t *cmeta;
    uint64_t c0;               // compress(row 0)
};
bool narrow_span_fits(int W, int lw, int tz, const uint64_t *first, const uint64_t *last);
hipError_t narrow_end_rows(const WinView &w, const uint32_t *n_dev, uint64_t *out, hipStream_t s);
// (key32 != null: the narrow tiles' key32 -- and rank32 unless null, lsn32
// mode -- written by the same pass, *flag as narrow_tiles_build's)
bool narrow_level01_tiles(const NarrowView &nv);  // can narrow_build write key32 (levels 0 + 1 fused)
hipError_t narrow_build(const WinView &w, const NarrowView &nv, hipStream_t s, uint32_t *key32 = nullptr,
                        uint32_t *rank32 = nullptr, uint64_t rank_base = 0, uint32_t *flag = nullptr);
hipError_t launch_probe_narrow(const NarrowView &nv, const ProbeView &p, uint8_t *verdict,
                               hipStream_t s);
hipError_t narrow_codes(const NarrowView &nv, const ProbeView &p, uint64_t *lo64, uint64_t *hi64,
                        hipStream_t s);
// The small-batch form (one launch: ranges, delta run, locks; inputs and
// verdicts in host-mapped memory; the last block releases seq into *done).
struct DeltaView;
// The pending tail of appends (hsc_ctx.h h_pend): unsorted rows in mapped
// pinned memory, [gid: 4P][lsn: 8P][words: [W][P], W <= kPendMaxWords]
// [table ids: 4P][table maxima: 8P] with P = kPendRows.
constexpr uint32_t kPendRows = 256;
constexpr int kPendMaxWords = 4;
constexpr size_t kPendLsn = 4 * (size_t)kPendRows, kPendWords = kPendLsn + 8 * (size_t)kPendRows,
                 kPendTtid = kPendWords + 8 * (size_t)kPendMaxWords * kPendRows,
                 kPendTlsn = kPendTtid + 4 * (size_t)kPendRows, kPendBytes = kPendTlsn + 8 * (size_t)kPendRows;
struct PendView {
    const uint8_t *base;  // device address of the buffer (nullptr: none)
    uint32_t n, nt;       // rows, table entries
};
constexpr int kSmallMaxLevels = 8;  // key-tree levels k_small_narrow descends (16^8 = 2^32 rows)
// The done word: seq << 32, and with `pack` (at most kSmallPackTxns read sets)
// on a one-block grid the verdicts too: bit 31 set and bit t = read set t's
// verdict (no verdict bytes written: one store ends the call).
constexpr uint32_t kSmallPackTxns = 31, kSmallPacked = 1u << 31;
hipError_t launch_small_narrow(const NarrowView &nv, const DeltaView &d, const DeltaView &d2,
                               const PendView &pd, const ProbeView &p,
                               uint8_t *verdict, uint32_t *blocks_done, uint64_t *done,
                               uint32_t seq, bool pack, hipStream_t s);
// 16-ary directory over a sorted u64 array A (hsc_narrow.hip): level 0 = A
// padded with ~0 to a multiple of 16, level l+1 [i] = level l [16 i + 15]
// (the last entry of every 16-entry block), up to one block; levels >=
// lds_from are staged in LDS by the searching kernel (lds_n entries).
constexpr int kDirLevels = 12;
struct Dir16 {
    const uint64_t *v;          // all levels, level l at v + off[l]
    uint32_t off[kDirLevels];
    uint32_t len[kDirLevels];   // entries of level l (multiple of 16)
    int levels, lds_from;
    uint32_t lds_n;
    uint32_t n;                 // entries of A
};
// Builds d over src[0 .. n) into buf (resized); at most max_lds entries in LDS.
hipError_t dir16_build(const uint64_t *src, uint32_t n, struct DBuf &buf, Dir16 &d,
                       uint32_t max_lds, hipStream_t s);

// Narrow tiles (dense batches): 4096-row tiles of (u32 key delta, u32 commit rank).
struct NarrowTiles {
    const uint32_t *key32;     // [len0] key64 - first key64 of the tile
    const uint32_t *rank32;    // [len0] commit time of the row (see rank_lsn32)
    // rank_lsn32: the window's commit LSNs span < 2^32 - 2 (a window inside
    // one log file, or files that close together): rank32 = lsn - base + 1
    // and a snapshot S maps to clamp(S - base + 1) in O(1).  Otherwise
    // rank32 = 1 + the index of the row's LSN among the distinct commit LSNs
    // and S maps to #commits <= S through cdir.  Either way lsn > S <=>
    // rank32 > r(S).
    int rank_lsn32;
    uint64_t rank_base;        // lsn32 mode: the oldest commit LSN of the window
    Dir16 cdir;                // directory of the window's distinct commit LSNs
    Dir16 tdir;                // directory of the first code of every tile
    const uint32_t *trad;      // [trad_m + 2] bucket table over tile first codes
                               // (trad[k] = #first < k << shift; trad[m + 1] = shift),
                               // nullptr: search tdir instead
    uint32_t trad_m;           // buckets (power of two)
    uint4 *recs;               // chunk areas of 2 x chunk records {lo delta, hi delta, r(S), read set}
};
hipError_t check_sorted_u64(const uint64_t *v, size_t n, uint32_t *flag, hipStream_t s);
// rank32 by a search of cdir (the 16-ary directory over the commit LSNs C)
hipError_t narrow_tiles_build(const uint64_t *key64, const uint64_t *lsn, uint32_t n, uint32_t len,
                              const Dir16 &cdir, int rank_lsn32, uint64_t rank_base,
                              uint32_t *key32, uint32_t *rank32, uint32_t *flag, hipStream_t s);
// r(S) of lsn32 mode: lsn > S <=> lsn - base + 1 > r(S)
__host__ __device__ inline uint32_t lsn32_rank(uint64_t S, uint64_t base)
{
    if (S < base) return 0;
    const uint64_t d = S - base + 1;
    return d >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}
constexpr uint64_t kLsn32MaxSpan = 0xFFFFFFFDull;  // rows: lsn - base + 1 <= 0xFFFFFFFE
uint32_t narrow_tiles_chunk();
// Bucket table of the tiles' first codes (locate's tile search from LDS);
// returns the bucket count m (0: too many tiles, use the directory).
uint32_t narrow_trad_buckets(uint32_t ntiles, bool force_dir = false);
hipError_t narrow_trad_build(const uint64_t *first, uint32_t ntiles, uint32_t m, uint32_t *trad,
                             hipStream_t s, int logmode = 0);
// log-mode bucket of a code (see k_trad): exponent << sv | sv mantissa bits
constexpr uint32_t kTradLog = 1u << 16;
__host__ __device__ inline uint32_t trad_log_bucket(uint64_t x, int sv)
{
    if (x == 0) return 0;
    const int e = 63 - __builtin_clzll(x);
    const uint64_t mask = (1ull << sv) - 1;
    const uint64_t mant = e >= sv ? (x >> (e - sv)) & mask : (x << (sv - e)) & mask;
    return ((uint32_t)e << sv) | (uint32_t)mant;
}
uint32_t narrow_tiles_dir_lds();
// Read/write conflict pairs (hsc_edges.hip) over every window version: the
// build's key-sorted rows before dedupe.
struct EdgeView {
    const uint32_t *gid;
    const uint64_t *words;  // [W][stride]
    const uint64_t *lsn;
    size_t stride;
    uint32_t n;
    int W;
};
hipError_t edge_after(const EdgeView &w, uint64_t smin, uint32_t *flag, uint32_t *scratch,
                      EdgeView &o, uint32_t *n_out, hipStream_t s);
hipError_t launch_edge_count(const EdgeView &w, const ProbeView &p, uint2 *span, uint32_t *cnt,
                             hipStream_t s);
hipError_t launch_edge_emit(const EdgeView &w, const ProbeView &p, const uint2 *span,
                            const uint32_t *off, uint32_t *out_txn, uint64_t *out_lsn,
                            hipStream_t s);

// Incremental window (hsc_delta.hip): rows appended after a build, sorted by
// (gid, words), W words of stride `stride`; bmax = per-64-row LSN maxima.
struct DeltaView {
    const uint32_t *gid;
    const uint64_t *words;  // [W][stride]
    const uint64_t *lsn;
    const uint64_t *bmax;   // [ceil(n / 64)]
    size_t stride;
    uint32_t n;
    int W;
};
constexpr uint32_t kDeltaCap = 1u << 16;  // delta rows before a merge into the main window
// out (stride ostride) = merge of d and the sorted rows a; bmax of the result
hipError_t delta_merge(const DeltaView &d, const DeltaView &a, uint32_t *ogid, uint64_t *owords,
                       uint64_t *olsn, size_t ostride, uint64_t *bmax, hipStream_t s,
                       const uint64_t *tmax_src = nullptr, uint64_t *tmax_dst = nullptr,
                       uint32_t nt = 0, bool stage_a = false);
// stage_a: a (at most kDeltaStageRows rows) is read from mapped pinned host
// memory, each merge block copying it into LDS first (a commit's rows need no
// upload)
constexpr uint32_t kDeltaStageRows = 256;
// flags[txn] = 1 for every range probe with a delta row of its group in
// [lo, hi] committed after its snapshot (raw W-word bounds)
hipError_t launch_probe_delta(const DeltaView &d, const ProbeView &p, uint8_t *flags, hipStream_t s);

// Replicant coalesce (hsc_coalesce.hip): flat read sets in, per-set surviving
// rows (ord) + the four fields merge_neighbor rewrites (w_*) out.
struct CoView {
    int ntxn;
    const int64_t *off;                        // [ntxn + 1]
    const int32_t *table, *idxnum, *lflag, *rflag, *islocked, *lkeylen, *rkeylen;
    const uint64_t *lkey_off, *rkey_off;
    const uint8_t *keys;
    uint64_t nkeys;
    const int32_t *tbrank;                     // strcmp rank of each table name
    int32_t *w_rflag, *w_islocked, *w_rkeylen;  // [nranges] working copies
    uint64_t *w_rkey_off;
    uint32_t *ord, *tmp;                       // [nranges] coalesced order per set
    uint32_t *count;                           // [ntxn] ranges left per set
};
// isbig[t] != 0: set t (one of big_set[0 .. nbig), elements big_pre[k] ..
// big_pre[k + 1], at most big_maxn per set) takes the level-parallel sort.
constexpr uint32_t kCoBig = 256;
// tie_scratch (coalesce_tie_scratch_bytes(big_total), NULL if no big set has a
// NULL lower key): the big sets sort on glibc's exact merge tree instead.
// run_scratch (coalesce_run_scratch_bytes(big_total), or NULL for one thread
// per run): the merge scan of the big sets' runs in parallel chunks.
size_t coalesce_tie_scratch_bytes(uint32_t total);
size_t coalesce_run_scratch_bytes(uint32_t total);
hipError_t launch_coalesce(const CoView &v, const uint32_t *isbig, const uint32_t *big_set,
                           const uint32_t *big_pre, uint32_t nbig, uint32_t big_total,
                           uint32_t big_maxn, uint32_t *big_runpos, uint32_t *big_scratch,
                           void *tie_scratch, void *run_scratch, hipStream_t s);

// Narrow tiles keep the chunk histogram tile-major: hist[t * hist_stride(G) + g].
__host__ __device__ inline uint32_t hist_stride(uint32_t G) { return (G + 7) & ~7u; }
// XCD-contiguous chunk order: block b of a grid of 8 * per blocks runs on XCD
// b % 8 and takes chunk (b % 8) * per + b / 8.
__host__ __device__ inline uint32_t xcd_chunk(uint32_t b, uint32_t per) { return (b & 7) * per + (b >> 3); }
// The plan of chunk-sorted records (narrow and compact tiles): transposes the
// locate's chunk-major table into the tile-major offsets and run starts
// (ctl[1]: extra join items of hot tiles, zeroed by the locate).  It also
// writes the batch's verdict bytes from the locate's flags (clearing them),
// so the join and the delta probe mark the verdict directly and no pack pass
// is needed (pack folded into the plan)
hipError_t launch_plan_s(const ProbeWork &work, uint32_t ntiles, uint32_t *ctl, hipStream_t s,
                         uint8_t *flags, uint32_t n_txn, uint8_t *verdict);
// Verdict bytes + bitmap from the internal conflict flags; clears the flags.
hipError_t launch_pack_flags(uint8_t *flags, uint32_t n_txn, uint8_t *verdict, uint64_t *bitmap,
                             hipStream_t s);
hipError_t launch_locate_t(const NarrowView &nv, const WinView &wt, const ProbeView &p,
                           const ProbeWork &work, const NarrowTiles &nt, uint8_t *verdict,
                           hipStream_t s);
hipError_t launch_join_t(const ProbeWork &work, const NarrowTiles &nt, uint32_t n,
                         uint32_t ntiles, uint32_t max_items, uint8_t *verdict, hipStream_t s,
                         uint32_t extra_blocks = 512);
// Dependency graph + SCC (hsc_graph.hip).
constexpr uint64_t kDepWW = 1, kDepWR = 2, kDepRW = 4;
struct GraphInput {              // device pointers
    const uint32_t *txn;         // [nops] commit order of the op's txn
    const uint64_t *key;
    const uint8_t *is_write;
    const uint32_t *observed;    // reads: writer txn of the observed version, ~0 initial
    size_t nops;
    uint32_t ntxn;
    // staged extra edges (rows src << 32 | dst, type bits) merged into the build
    const uint64_t *x_rows = nullptr, *x_type = nullptr;
    size_t n_extra = 0;
    bool skip_rw = false;  // reads give wr edges only (rw come from x_rows)
    bool txn_sorted = false;  // ops in nondecreasing txn order (set by the check when it runs)
    bool check = false;       // graph_build checks the ops itself (GraphBufs::bad; an op
                              // out of range: hipErrorInvalidValue before any edge work)
};
constexpr uint32_t kBackCap = 1u << 20;  // GraphBufs::back rows
struct GraphBufs {
    DBuf flags, flags2, scratch, count;
    DBuf wg, ww, wl, wg2, ww2, wl2;            // writer rows
    DBuf ew, et, eg, ew2, et2, eg2, swap_rows;  // edge rows
    DBuf src, out_dst, type, in_src, in_dst, out_off, in_off;
    DBuf scc, active, color, mark, front, front2;
    DBuf h_txn, h_key, h_isw, h_obs;           // uploaded history
    DBuf diff, cut, cut_id, txn_of;            // sharded SCC: cover, cut rows, cut ids
    DBuf x_rows, x_type, x_map;                // staged extra edges (rw pairs)
    DBuf pk, pdir;                             // packed distinct writers + their directory
    DBuf ptab;                                 // the directory's buckets inline, one line each
    DBuf rp_cnt, rp_items;                     // partitioned read search: counts / cursors, items
    size_t n_extra = 0;
    size_t ne = 0;
    size_t ne_raw = 0;  // raw edge slots in ew
    bool raw = false;   // last build kept raw rows only (no sort / CSR)
    bool writer_packed = false;  // last build sorted its writers as packed (key, txn) words
    uint32_t diff_nn = 0;        // raw build: diff holds the cover's backward-edge diffs over diff_nn txns
    uint32_t cover_nn = 0;       // txns of the covers graph_cut tests (the build's ntxn)
    uint32_t bad = 0;            // the last checked build's input bits (GraphInput::check)
    uint32_t *edge_bad = nullptr;  // device word of the edge pass's observed-id check (graph_build_timed
                                   // reads it after the build), or null
    uint32_t *post = nullptr;      // device words read after a build: [-1] the packed writer sort's stall
                                   // flag, [0] backward rows listed, [1] = edge_bad's
    DBuf back;                     // a raw build's backward rows (graph_cover marks their intervals)
    bool ww_pk = false;            // the last build's ww rows came from its packed writers:
    PairPack pp{};                 // their layout, array (in the build's buffers) and count
    const uint64_t *ppk = nullptr;
    uint32_t pnu = 0;
    bool back_listed = false;
    uint32_t back_n = 0;           // listed rows (> back_cap: only counted -- graph_cover takes the diffs)
    uint32_t back_cap = kBackCap;
    DBuf cover_bits;             // graph_cut: the cover as a bitmap
    DBuf cover_list;             // graph_cut: the covered txns (the op-range cut)
    DBuf gvary;                  // k_gw_place's per-block OR / AND of the writers' key and txn
    // raw build over txn-sorted ops in the op-slot layout (ww rows [0, op_at),
    // op i's rows op_at + 2i, + 1, staged rows from x_at): graph_cut given the
    // ops' txn array visits the covered txns' ops only
    bool op_cut = false;
    size_t op_at = 0, op_n = 0, x_at = 0, x_n = 0;
    void release_all()
    {
        DBuf *all[] = {&flags, &flags2, &scratch, &count, &wg, &ww, &wl, &wg2, &ww2, &wl2,
                       &ew, &et, &eg, &ew2, &et2, &eg2, &swap_rows, &src, &out_dst, &type,
                       &in_src, &in_dst, &out_off, &in_off, &scc, &active, &color, &mark,
                       &front, &front2, &h_txn, &h_key, &h_isw, &h_obs, &diff, &cut,
                       &cut_id, &txn_of, &x_rows, &x_type, &x_map, &pk, &pdir, &ptab, &rp_cnt,
                       &rp_items, &cover_bits, &cover_list, &gvary, &back};
        for (DBuf *b : all) b->release();
    }
};
// full: sorted unique edges + CSR / CSC; else raw edge rows in g.ew only.
hipError_t graph_build(const GraphInput &in, GraphBufs &g, bool full, hipStream_t s);
hipError_t graph_type_counts(GraphBufs &g, uint64_t out[3], hipStream_t s);
// rw pairs (read set t, writer commit LSN c) -> edge rows t' -> c' of type rw:
// t' = rs_txn[t], c' = commit_txn[i] with commit_lsn[i] == c (sorted); a pair
// whose LSN is not listed sets *bad; self edges become ~0 rows.
hipError_t graph_pairs_rows(size_t n, const uint32_t *txn, const uint64_t *lsn, uint32_t nrs,
                            const uint32_t *rs_txn, size_t ncommit, const uint64_t *commit_lsn,
                            const uint32_t *commit_txn, uint64_t *rows, uint64_t *type,
                            uint32_t *bad, hipStream_t s);
hipError_t graph_scc(uint32_t nnodes, GraphBufs &g, uint32_t *rounds, uint32_t *iterations,
                     hipStream_t s);
// Compact codes of wide windows (hsc_compact.hip): per group the key bits
// that vary between its rows, most significant first, in WC words.
struct CompactTables {
    const uint64_t *mask, *pat, *mv;  // [ng][W] varying bits, first row, compress moves [ng][W][6]
    const uint32_t *bits;             // [ng] varying bits (0xFFFFFFFF: no rows)
    int W, WC;
    const uint32_t *wlen;             // [ng] words inside the group's key length (bounds
                                      // are zero past it, like its rows)
    int ng;                           // groups
};
constexpr int kMaxCompactWords = 6;
void compress_moves(uint64_t m, uint64_t mv[6]);
hipError_t compact_masks(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                         int W, int ng, const uint32_t *gstart, const uint32_t *gend,
                         uint64_t *mask, uint64_t *pat, hipStream_t s);
hipError_t compact_rows(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                        const CompactTables &t, uint64_t *cw, hipStream_t s);
// The code sort of wide rows (hsc_csort.hip): the compact tables of UNSORTED
// rows (each group's pattern = its lowest-index row; ng W <= kCsVaryLds / 16
// for the LDS accumulators), the (WC + 1)-word key of every row (gid ||
// code || row index), the keys' sort, and the sorted keys back to rows.
constexpr size_t kCsVaryLds = 64 * 1024;
hipError_t compact_masks_unsorted(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                                  int W, int ng, uint32_t *rep, uint64_t *mask, uint64_t *pat,
                                  hipStream_t s);
hipError_t compact_sort_keys(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                             const CompactTables &t, uint64_t *keys, hipStream_t s);
// split: code_sort_split_words(n) u32 of device scratch
size_t code_sort_split_words(size_t n);
hipError_t code_keys_sort(uint64_t *keys, uint64_t *tmp, uint32_t *split, size_t n, int KW, hipStream_t s,
                          uint64_t **sorted);
// sorted keys back to rows, with the dedupe fused in: every version to *_o, the last of
// each key to *_d (which may be the input gid / words -- only lsn_in is read
// by index), d_count[0] = distinct rows, and (codes_d set) the distinct rows'
// codes as [WC][stride_d] (what compact_rows computes); scratch >= n / 2048 + 16 +
// scan_scratch_bytes(n / 2048 + 1) / 4 words
hipError_t compact_unpack_dedupe(const uint64_t *keys, size_t n, const CompactTables &t,
                                 const uint64_t *lsn_in, uint32_t *gid_o, uint64_t *words_o,
                                 uint64_t *lsn_o, size_t stride_o, uint32_t *gid_d, uint64_t *words_d,
                                 uint64_t *lsn_d, size_t stride_d, uint32_t *d_count, uint32_t *scratch,
                                 uint64_t *codes_d, hipStream_t s);
hipError_t warm_csort();
// lo/hi bounds (W words) -> code bounds (WC words, SoA [WC][n]); ranges that
// miss their group's rows become (~0, 0)
struct PointHash;
hipError_t compact_probes(const ProbeView &p, const CompactTables &t, uint64_t *clo, uint64_t *chi,
                          hipStream_t s, const PointHash *ph = nullptr);
// Compact tiles (hsc_ctiles.hip): the compact window as one sorted array of
// WG-word keys gid || code (WG <= 3) with 32-bit commit times, 2048-row
// tiles, for dense batches.
constexpr int kCTLog2 = 11;
constexpr int kTBLog2 = 10, kTB = 1 << kTBLog2;  // word-0 buckets per tile
constexpr int kTBS = kTB + 4;                     // u32 per tile: kTB spans, tn | shift, pad
struct CTiles {
    const uint64_t *key;     // [WG][len] row keys, sorted (padding ~0)
    const uint32_t *rank;    // [len] lsn - rank_base + 1 in row order (padding 0)
    const uint32_t *tb;      // [ntiles][kTBS] per-tile word-0 bucket table (k_ct_tbuckets)
    const uint64_t *first;   // [WG][ntiles] first key of every tile
    const uint32_t *trad;    // [trad_m + 2] bucket table over first word 0 - base0
    uint32_t trad_m;
    uint64_t base0;          // word 0 of tile 0's first key
    uint64_t rank_base;      // oldest commit LSN of the window
    size_t len;              // row stride (n rounded up to whole tiles)
    uint32_t n, ntiles;
    int WG, WC, gb;          // key words, code words, group bits
    uint32_t np;             // probes of the batch
    uint32_t *recs;          // chunk areas of 2 x chunk 64-byte records (k_locate_c)
    int dbg;                 // diagnostics (HSC_CT_DBG): 1 join skips the searches, 2 also the gathers
};
// Exact-key index of the compact tiles' keys for point probes (lo == hi):
// open addressing over 128-byte buckets of four 32-byte entries {key words
// 0-2, rank} (rank 0 = empty; a row's rank is >= 1), linear probing by bucket.
// The bound kernel answers a point whose code bounds meet by one lookup --
// conflict iff the key is present with rank > r(S) -- sets the read set's flag
// and writes the probe an empty code range, so the locate makes no record for
// it and the join never searches it (the join's answer for a point record is
// the same: the row equal to the key, its rank against r(S)).
struct PointHash {
    const uint64_t *e;   // [nb][4][4]
    uint64_t nb;         // buckets (0: no index)
    int WG, gb;          // the tiles' key words and group bits
    uint64_t rank_base;  // CTiles::rank_base
    uint8_t *flags;      // the batch's conflict flags (the locate's)
    uint32_t ep;         // the build's epoch (bits 40..63 of a live entry's rank word)
};
uint64_t point_hash_buckets(uint32_t n);
// clear: the buffer is new (epochs restart at 1); else entries of older epochs read as empty
hipError_t point_hash_build(const CTiles &ct, uint64_t *e, uint64_t nb, uint32_t ep, bool clear, hipStream_t s);
hipError_t ctiles_build(const uint64_t *cw, size_t cs, int WC, const uint32_t *gid,
                        const uint64_t *lsn, const CTiles &ct, uint64_t *key, uint32_t *rank,
                        uint64_t *first, uint64_t *rel, uint32_t *trad, uint32_t *tb,
                        hipStream_t s);
size_t ctiles_locate_lds(const CTiles &ct);
uint32_t ctiles_chunk();
hipError_t launch_locate_c(const CTiles &ct, const WinView &wt, const ProbeView &p,
                           const uint64_t *clo, const uint64_t *chi, const ProbeWork &work,
                           uint8_t *flags, hipStream_t s);
hipError_t launch_join_c(const CTiles &ct, const ProbeWork &work, uint32_t max_items,
                         uint8_t *flags, hipStream_t s);
// Sharded SCC (hsc_graph.hip): cover[v] = 1 iff v lies inside [dst, src] of a
// backward edge of g; the edges of g between covered nodes -> g.cut rows
// (src << 32 | dst, *m of them); SCC of the graph induced on the cover by
// explicit rows (~0 = padding) into scc_out[nn] (device).
hipError_t graph_cover(GraphBufs &g, uint32_t nn, uint8_t *cover, hipStream_t s);
// op_txn: the last build's ops' txn array (still live), or null -- with it a
// raw build over txn-sorted ops tests the ww / staged rows and the covered
// txns' own op rows instead of every row (with op_key / op_isw too, the ww
// rows from the covered txns' write ops)
hipError_t graph_cut(GraphBufs &g, const uint8_t *cover, size_t *m, hipStream_t s,
                     const uint32_t *op_txn = nullptr, const uint64_t *op_key = nullptr,
                     const uint8_t *op_isw = nullptr, bool host_sort = true);
// (host_sort false: the cut rows in no particular order -- the SCC of a cut
// does not depend on it -- without the sort's two copies and syncs)
hipError_t graph_scc_rows(uint32_t nn, const uint8_t *cover, const uint64_t *rows, size_t m,
                          GraphBufs &g, uint32_t *scc_out, uint32_t *n_cut, uint32_t *rounds,
                          uint32_t *iterations, hipStream_t s);
hipError_t swap_edge_words(uint32_t m, const uint32_t *src, const uint32_t *dst, uint64_t *rows,
                           hipStream_t s);
hipError_t scan_exclusive_u32(uint32_t *a, size_t n, uint32_t *scratch, hipStream_t s);

// Raw log decoder (hsc_logdec.cpp): bytes -> the hsc_llog SoA it owns.
struct DecodedLog {
    std::vector<uint64_t> lsn, prev, key_off;
    std::vector<uint32_t> rectype;
    std::vector<int16_t> isabort, ix;
    std::vector<int32_t> table, keylen;
    std::vector<uint8_t> keys;
    std::vector<std::string> names;
    std::vector<const char *> name_ptrs;
    uint64_t end_lsn = 0;
    hsc_llog llog{};
    void view();  // point llog at the vectors
};
// Physical records (every record, header fields; whole bytes of __db_addrem
// and __db_big) that the index-key reconstruction walk may visit
// (bdb/rowlocks.c:209-617): the decoded raw logs since the last ingest, so a
// walk reaches records of earlier appends.  LSNs ascending.
struct PhysStore {
    std::vector<uint64_t> lsn, prev, off;
    std::vector<uint32_t> type, len;
    std::vector<uint8_t> bytes;
    void clear()
    {
        lsn.clear(), prev.clear(), off.clear(), type.clear(), len.clear(), bytes.clear();
    }
    long find(uint64_t l) const;
    void truncate(size_t n, size_t nbytes)
    {
        lsn.resize(n), prev.resize(n), off.resize(n), type.resize(n), len.resize(n);
        bytes.resize(nbytes);
    }
};
// reset: the raw log starts a new log (ingest), else it continues the stored
// records (append; a log whose first LSN is not above them starts anew).
int decode_raw_log(const hsc_raw_log *raw, DecodedLog &out, PhysStore &ps, bool reset,
                   std::string &err);

// OSQL_SERIAL wire decoder (hsc_wire.cpp): payloads -> hsc_readsets SoA.
struct DecodedReadSets {
    std::vector<int64_t> txn_off;
    std::vector<uint64_t> snap, lkey_off, rkey_off;
    std::vector<int32_t> table, idxnum, lflag, rflag, islocked, lkeylen, rkeylen;
    std::vector<uint8_t> keys;
    std::vector<std::string> names;
    std::vector<const char *> name_ptrs;
    hsc_readsets rs{};
    void view();
};
int decode_serial_msgs(const hsc_serial_msgs *m, DecodedReadSets &out, std::string &err);

hipError_t launch_pack(const uint8_t *verdict, uint32_t n_txn, uint64_t *bitmap,
                       hipStream_t s);
hipError_t launch_or_bitmaps(const uint64_t *parts, int nparts, size_t words, uint64_t *out,
                             hipStream_t s);

// Premarshal (hsc_collect.cpp): a caller marshals its own read set against
// the context's published dictionary snapshot before it queues; the batch
// (check_batch_pre = hip_serial_check_batch, full checks) takes those rows
// while the snapshot's epoch is current and marshals the rest itself.
struct PreMarshal;
PreMarshal *premarshal_new();
void premarshal_free(PreMarshal *pm);
bool premarshal(hsc_ctx *c, const hsc_currangearr *a, uint64_t S, PreMarshal *pm);
// bdb_osql_serial_check(..., regop_only = 1) on one read set: the context's
// published snapshot without its lock, or the locked path; errors -> 1
int ctx_regop_probe(hsc_ctx *c, void *ranges, unsigned int *file, unsigned int *offset);
int check_batch_pre(hsc_ctx *c, void *const *ranges, PreMarshal *const *pre, unsigned int *file,
                    unsigned int *offset, int n, int *rc_out);

// Multi-GPU routing (hsc_route.hip, hsc_multi.cpp): the window cut into
// world <= kMultiMax contiguous pieces of the composite key space (gid, key
// words) at world - 1 ascending splitters.
constexpr int kMultiMax = 16;
struct RouteSplit {
    const uint32_t *gid;  // [S]
    const uint64_t *w;    // [W][S]
    int S, W;
};
// Where a destination's rows go: probe columns with a row stride, and (member
// 0 only) the table-lock columns.
struct RouteTarget {
    uint64_t *lo, *hi, *snap;
    uint32_t *gid, *txn;
    size_t stride;
    uint64_t *lock_snap;
    uint32_t *lock_table, *lock_txn;
};
struct RouteArgs {
    RouteTarget t[kMultiMax];
    uint32_t base[kMultiMax];  // this source's first row in each target
    int N;
    uint32_t tbase;      // added to every read-set number (the batch-wide numbering)
    uint32_t lock_base;  // this source's first row in member 0's lock columns
};
// Received send blocks (RCCL): source s's block at byte boff[s], n[s] probes
// and nl[s] locks, numbered [roff[s], roff[s + 1]) / [loff[s], loff[s + 1])
// over the received blocks; they land at target rows dst[s] + k / lock rows
// ldst[s] + k (the receiver's own rows are stored there by its scatter).
struct RouteUnpack {
    uint64_t boff[kMultiMax];
    uint32_t n[kMultiMax], nl[kMultiMax], roff[kMultiMax + 1], loff[kMultiMax + 1];
    uint32_t dst[kMultiMax], ldst[kMultiMax];
    int N;
};
struct RouteParts {
    const uint64_t *p[kMultiMax];
    int n;
};
// bytes of one send block: probe columns lo[W] hi[W] snap, gid txn; locks
__host__ __device__ inline size_t route_block_bytes(int W, size_t n, size_t nl)
{
    return 8 * (size_t)(2 * W + 2) * n + 16 * nl;
}
uint32_t route_blocks(size_t n);  // chunks (hist rows) of a routed batch
// k_route_count's outputs (published by a one-workgroup k_route_total after
// it).  ctl (device): ctl[N + 1, 2N + 1) the scatter's cursors, zeroed for it.
// totals[0, N) = the counts, totals[N] = n_lock, totals[N + 1] = n_txn and,
// when host is set (fine-grained pinned memory mapped for the device), the
// same N + 2 words to host[] and then seq to host[N + 2] with a system-scope
// release -- the host spins on that word instead of a copy and an event.
struct RouteCountOut {
    uint32_t *ctl, *totals, *host;
    uint32_t seq, n_lock, n_txn;
};
hipError_t launch_route_count(const ProbeView &p, const RouteSplit &sp, int N, uint32_t *hist,
                              const RouteCountOut &o, hipStream_t s);
// words u32 of src to host[0, words), then seq to host[words] (system scope)
hipError_t launch_route_publish(const uint32_t *src, uint32_t words, uint32_t *host, uint32_t seq,
                                hipStream_t s);
// cursor: ctl + N + 1 of the count launch (zero)
hipError_t launch_route_scatter(const ProbeView &p, const RouteSplit &sp, const RouteArgs &a,
                                const uint32_t *hist, uint32_t *cursor, hipStream_t s);
hipError_t launch_route_unpack(const uint8_t *raw, const RouteUnpack &u, const RouteTarget &t, int W,
                               hipStream_t s);
hipError_t launch_or_slices(const RouteParts &parts, size_t words, uint64_t *out, hipStream_t s);
// verdict bytes (64 per output word, 8-byte aligned) of several members OR-ed into a bitmap
struct RouteBytes {
    const uint8_t *p[kMultiMax];
    int n;
};
hipError_t launch_or_bytes(const RouteBytes &parts, size_t words, uint64_t *out, hipStream_t s);

// per-file code-object warm-up (hsc_ctx_create)
hipError_t warm_kernels();
hipError_t warm_ingest();
hipError_t warm_narrow();
hipError_t warm_ctiles();
hipError_t warm_delta();
hipError_t warm_compact();
hipError_t warm_coalesce();
hipError_t warm_edges();
hipError_t warm_graph();
hipError_t warm_route();

}  // namespace hsc
