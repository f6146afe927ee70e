// hsc_ctiles.hip -- compact tiles: the dense-batch tile pipeline for wide
// windows whose compact codes (hsc_compact.hip) plus the group id fit in at
// most 3 words (config 3's composite keys: 184 varying bits + 5 group bits).
//
// Every row becomes one key of WG words, K = gid || code (the group id in the
// top gb bits, then the group's varying bits, most significant first).  Rows
// are sorted by (gid, key words) and the code keeps the words' order inside a
// group, so the keys are sorted, and a range [lo, hi] of group g maps exactly
// onto [g || lo', g || hi'] with lo', hi' the code bounds of compact_probes.
// The window is then ONE sorted array of WG-word keys with 32-bit commit
// times (lsn - oldest commit + 1; the window's commits span < 2^32 of log),
// cut into 2048-row tiles, and the narrow tile pipeline (hsc_narrow.hip)
// carries over with wide records:
//   locate  (4096 probes per workgroup): keys of lo / hi, their end tiles by a
//           bucket table over the tiles' first word 0 plus a full-key binary
//           search of the bucket (first keys in LDS), the whole tiles between
//           them from the tile-max sparse table, the chunk's tile histogram;
//           writes the probe's 64-byte entry {lo, hi, r(S), read set} once and
//           its one or two (tile, in-chunk rank) slots
//   plan    k_plan_t (fixed-capacity tile buckets, overflow runs for hot tiles)
//   scatter 4-byte bucket entries (probe index | record kind)
//   join    a workgroup per tile: its keys (Eytzinger order, every word) and
//           ranks in LDS (56 KiB), each record's probe entry gathered (one
//           64-byte line), #keys < lo and #keys <= hi by two lockstep
//           root-to-leaf walks, any rank > r(S) over [pa, pb) via 16- and
//           128-row maxima
//   pack    k_pack_flags
// Every key compare is exact (all WG words are in LDS), so unlike the wide
// pipeline's word-0 join a probe equal to a row never reads the window again.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <cstdlib>

namespace hsc {

namespace {

constexpr uint32_t kCTRows = 1u << kCTLog2;  // rows per tile
// 2048-probe chunks: config 3's ~600k ranges make ~290 locate workgroups,
// enough for every CU (4096-probe chunks left 110 of 256 idle; chunks sized
// to one workgroup per CU -- 2560 probes, 232 workgroups -- measured the same,
// 32.4 vs 32.9 us (r05): a workgroup's time is not its probes in series)
#ifndef HSC_CLOC_THREADS
#define HSC_CLOC_THREADS 512
#endif
#ifndef HSC_CLOC_P
#define HSC_CLOC_P 4
#endif
constexpr int kCLocThreads = HSC_CLOC_THREADS;
constexpr int kCLocP = HSC_CLOC_P;           // probes per locate thread
constexpr uint32_t kCChunk = kCLocThreads * kCLocP;
static_assert(kCChunk <= 4096, "in-chunk ranks are 12 bits");
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint32_t kSecondRec = 1u << 31, kPointRec = 1u << 30;
// record kinds (top two bits of a bucket entry): search lo and hi / lo only
// (the range runs past the tile) / hi only (it starts before the tile) / a
// point (lo == hi: one search, then an equality test)
constexpr uint32_t kCFull = 0, kCHead = 1, kCTail = 2, kCPoint = 3;

// K = g || code: the WC code words shifted right by gb bits under the group id
template <int WG>
__device__ __forceinline__ void compose(uint32_t g, int gb, const uint64_t (&c)[WG],
                                        uint64_t (&k)[WG])
{
    if (gb == 0) {
#pragma unroll
        for (int j = 0; j < WG; ++j) k[j] = c[j];
        return;
    }
    k[0] = ((uint64_t)g << (64 - gb)) | (c[0] >> gb);
#pragma unroll
    for (int j = 1; j < WG; ++j) k[j] = (c[j - 1] << (64 - gb)) | (c[j] >> gb);
}

template <int WG>
__device__ __forceinline__ bool key_lt(const uint64_t (&a)[WG], const uint64_t (&b)[WG])
{
#pragma unroll
    for (int j = 0; j < WG - 1; ++j)
        if (a[j] != b[j]) return a[j] < b[j];
    return a[WG - 1] < b[WG - 1];
}

// ---- build: row keys, ranks, tiles' first keys ----
template <int WG>
__global__ __launch_bounds__(256) void k_ct_rows(const uint64_t *cw, size_t cs, int WC,
                                                 const uint32_t *gid, const uint64_t *lsn,
                                                 CTiles ct, uint64_t *key, uint32_t *rank,
                                                 uint64_t *first)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ct.len) return;
    uint64_t k[WG];
    uint32_t r = 0;
    if (i < ct.n) {
        uint64_t c[WG];
#pragma unroll
        for (int j = 0; j < WG; ++j) c[j] = j < WC ? cw[(size_t)j * cs + i] : 0;
        compose<WG>(gid[i], ct.gb, c, k);
        r = (uint32_t)(lsn[i] - ct.rank_base) + 1;
    } else {
#pragma unroll
        for (int j = 0; j < WG; ++j) k[j] = ~0ull;  // padding: above every bound
    }
    const uint32_t t = i >> kCTLog2, o = i & (kCTRows - 1);
#pragma unroll
    for (int j = 0; j < WG; ++j) key[(size_t)j * ct.len + i] = k[j];
    rank[i] = r;
    if (o == 0 && t < ct.ntiles)
#pragma unroll
        for (int j = 0; j < WG; ++j) first[(size_t)j * ct.ntiles + t] = k[j];
}

// word 0 of every tile's first key relative to tile 0's (the bucket table's input)
__global__ void k_ct_rel(const uint64_t *first0, uint32_t ntiles, uint64_t *rel)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntiles) rel[t] = first0[t] - first0[0];
}

// Per tile: kTB buckets over word 0 of its rows relative to the first row's,
// shift = the least that puts the last row's below kTB << shift;
// tb[t * kTBS + k] = B(k) | B(k + 1) << 16 for k < kTB, B(k) = #rows of the
// tile whose bucket is < k (one LDS read gives a bucket's row span), then
// tn | shift << 16.  A join search starts inside one bucket (a few rows) instead of
// walking the tile's 11 levels.
__global__ __launch_bounds__(256) void k_ct_tbuckets(CTiles ct, const uint64_t *key0, uint32_t *tb)
{
    constexpr int PER = kTB / 256;  // buckets per thread
    __shared__ uint32_t cnt[kTB];
    __shared__ uint32_t scr[8];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    const size_t r0 = (size_t)t << kCTLog2;
    const uint32_t tn = min(kCTRows, ct.n - (uint32_t)r0);
    const uint64_t f0 = key0[r0], span = key0[r0 + tn - 1] - f0;
    const int bits = span ? 64 - __clzll(span) : 0;
    const int shift = bits > kTBLog2 ? bits - kTBLog2 : 0;
    for (int k = 0; k < PER; ++k) cnt[tid * PER + k] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < tn; i += 256) atomicAdd(&cnt[(uint32_t)((key0[r0 + i] - f0) >> shift)], 1u);
    __syncthreads();
    uint32_t mine[PER], sum = 0;
    for (int k = 0; k < PER; ++k) sum += mine[k] = cnt[tid * PER + k];
    uint32_t tot;
    uint32_t pre = block_excl_scan<256>(sum, scr, tot);
    uint32_t *o = tb + (size_t)t * kTBS;
    for (int k = 0; k < PER; ++k) {
        o[tid * PER + k] = pre | (pre + mine[k]) << 16;
        pre += mine[k];
    }
    if (tid == 0) o[kTB] = tn | (uint32_t)shift << 16;
}

// ---- locate ----
struct CLocLds {
    uint32_t first, trad, hist, wtot, bytes;
};
__host__ __device__ inline CLocLds cloc_lds(const CTiles &ct)
{
    CLocLds L{};
    uint32_t o = 0;
    L.first = o;
    o += 8 * ct.WG * ((ct.ntiles + 1) & ~1u);
    L.trad = o;
    o += 2 * ((ct.trad_m + 1 + 7) & ~7u);
    L.hist = o;
    o += 4 * ((ct.ntiles + 3) & ~3u);
    L.wtot = o;  // the tail's scan: one total per wave
    o += 4 * (kCLocThreads / 64);
    L.bytes = o;
    return L;
}

// #tiles whose first key is < x (LE: <= x): the bucket of x's word 0, then a
// binary search inside it with full-key compares (typically 0-2 steps)
template <int WG, bool LE>
__device__ __forceinline__ uint32_t ct_count(const uint64_t *lf, uint32_t nt, const uint16_t *T,
                                             uint32_t m, int shift, uint64_t base0,
                                             const uint64_t (&x)[WG])
{
    if (x[0] < base0) return 0;  // below tile 0's first word: below every first key
    const uint64_t b = (x[0] - base0) >> shift;
    uint32_t l = b < m ? T[b] : T[m], h = b < m ? T[b + 1] : nt;
    while (l < h) {
        const uint32_t mid = (l + h) >> 1;
        // word 0 decides unless equal; later words are read only on a tie
        uint64_t v = lf[mid];
        bool below = v < x[0], eq = v == x[0];
#pragma unroll
        for (int j = 1; j < WG; ++j)
            if (eq) {
                v = lf[(size_t)j * nt + mid];
                below = v < x[j];
                eq = v == x[j];
            }
        below = eq ? LE : below;
        l = below ? mid + 1 : l;
        h = below ? h : mid;
    }
    return l;
}

// No probe entries, slots or scatter: the chunk's records stay in registers until its tile histogram is complete, then each
// goes whole (64 bytes: {key x, r(S) | read set | kind << 62} + {hi key} for a
// full record; x = lo, or hi for a tail record) to its tile-sorted place in
// the chunk's own area, and row g of the chunk-major table gets (run start
// << 16 | count) per tile for k_plan_s (as the narrow locate)
template <int WG>
__global__ __launch_bounds__(kCLocThreads) void k_locate_c(CTiles ct, WinView wt, ProbeView p,
                                                           const uint64_t *clo,
                                                           const uint64_t *chi, ProbeWork work,
                                                           uint8_t *flags)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lds64[];
    const uint32_t nt = ct.ntiles;
    const CLocLds L = cloc_lds(ct);
    char *lb = (char *)lds64;
    uint64_t *lf = (uint64_t *)(lb + L.first);
    uint16_t *T = (uint16_t *)(lb + L.trad);
    uint32_t *hist = (uint32_t *)(lb + L.hist);
    const uint32_t g = xcd_chunk(blockIdx.x, (work.G + 7) / 8);
    if (g >= work.G) return;
    if (g == 0 && threadIdx.x < 3) work.item_off[threadIdx.x] = 0;  // the plan's / join's counters
    const uint32_t c0 = g * work.chunk, c1 = min(p.n, c0 + work.chunk);
    // every probe load of the chunk first (read-once inputs: non-temporal)
    uint64_t lo[kCLocP][WG], hi[kCLocP][WG], snap[kCLocP];
    uint32_t gg[kCLocP];
#pragma unroll
    for (int k = 0; k < kCLocP; ++k) {
        const uint32_t q0 = c0 + threadIdx.x + kCLocThreads * k;
        const uint32_t q = q0 < c1 ? q0 : 0;  // chunks past the ranges (lock probes only) read row 0
        const bool v = p.n != 0;
        gg[k] = v ? __builtin_nontemporal_load(p.gid + q) : 0;
        snap[k] = v ? __builtin_nontemporal_load(p.snap + q) : 0;
#pragma unroll
        for (int j = 0; j < WG; ++j) {
            const bool u = v && j < ct.WC;
            lo[k][j] = u ? __builtin_nontemporal_load(clo + (size_t)j * p.n + q) : 0;
            hi[k][j] = u ? __builtin_nontemporal_load(chi + (size_t)j * p.n + q) : 0;
        }
    }
    {  // first keys, bucket table, histogram into LDS
        const uint32_t nf = WG * nt;
        for (uint32_t i = threadIdx.x; i < nf; i += kCLocThreads) lf[i] = ct.first[i];
        for (uint32_t i = threadIdx.x; i <= ct.trad_m; i += kCLocThreads) T[i] = (uint16_t)ct.trad[i];
        for (uint32_t i = threadIdx.x; i < nt; i += kCLocThreads) hist[i] = 0;
    }
    const int shift = (int)ct.trad[ct.trad_m + 1];
    __syncthreads();
    uint64_t KA[kCLocP][WG], KB[kCLocP][WG], RT[kCLocP];
    uint2 SL[kCLocP];
#pragma unroll
    for (int k = 0; k < kCLocP; ++k) {
        const uint32_t q = c0 + threadIdx.x + kCLocThreads * k;
        SL[k] = make_uint2(kNoSlot, kNoSlot);
        if (q >= c1) continue;
        uint64_t a_[WG], b_[WG];
        compose<WG>(gg[k], ct.gb, lo[k], a_);
        compose<WG>(gg[k], ct.gb, hi[k], b_);
        uint2 sl = make_uint2(kNoSlot, kNoSlot);
        if (!key_lt<WG>(b_, a_)) {
            const uint32_t ca = ct_count<WG, false>(lf, nt, T, ct.trad_m, shift, ct.base0, a_);
            const uint32_t cb = ct_count<WG, true>(lf, nt, T, ct.trad_m, shift, ct.base0, b_);
            if (cb > 0) {
                const uint32_t a = ca ? ca - 1 : 0, bt = cb - 1;
                const uint32_t txn = p.txn[q];
                // tiles strictly between the end tiles lie inside the range
                if (bt > a + 1 && tiles_max(wt, a + 1, bt - 1) > snap[k]) flags[txn] = 1;
                sl.x = a << 12 | atomicAdd(&hist[a], 1u);
                bool point = true;
#pragma unroll
                for (int j = 0; j < WG; ++j) point &= a_[j] == b_[j];
                if (bt > a) {
                    sl.x |= kSecondRec;
                    sl.y = bt << 12 | atomicAdd(&hist[bt], 1u);
                } else if (point) {
                    sl.x |= kPointRec;
                }
                // entries {lo[0..2], r(S) | read set << 32}, {hi[0..2], ...} (words past WG zero)
                const uint64_t rt = (uint64_t)lsn32_rank(snap[k], ct.rank_base) | (uint64_t)txn << 32;
#pragma unroll
                for (int j = 0; j < WG; ++j) KA[k][j] = a_[j], KB[k][j] = b_[j];
                RT[k] = rt;
                SL[k] = sl;
            }
        }
    }
    // table locks: any write to a locked table after the snapshot
    for (uint32_t q = g * kCLocThreads + threadIdx.x; q < p.n_lock; q += work.G * kCLocThreads) {
        const uint32_t t = p.lock_table[q];
        if (t < wt.ntables && wt.table_max[t] > p.lock_snap[q]) flags[p.lock_txn[q]] = 1;
    }
    __syncthreads();
    {
        const int lane = threadIdx.x & 63;
        uint32_t *wtot = (uint32_t *)(lb + L.wtot);
        const uint32_t per = (nt + kCLocThreads - 1) / kCLocThreads;
        const uint32_t i0 = min(nt, threadIdx.x * per), i1 = min(nt, i0 + per);
        uint32_t sum = 0;
        for (uint32_t i = i0; i < i1; ++i) sum += hist[i];
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t run = x - sum;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) run += wtot[w];
        uint32_t *row = work.cm + (size_t)g * ((nt + 3) & ~3u);
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t c = hist[i];
            row[i] = run << 16 | c;
            hist[i] = run;
            run += c;
        }
        __syncthreads();
        u64x2 *area = (u64x2 *)ct.recs + (size_t)g * 2 * work.chunk * 4;
#pragma unroll
        for (int k = 0; k < kCLocP; ++k) {
            const uint2 sl = SL[k];
            if (sl.x == kNoSlot) continue;
            uint64_t a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
#pragma unroll
            for (int j = 0; j < WG; ++j) a[j] = KA[k][j], b[j] = KB[k][j];
            const bool two = (sl.x & kSecondRec) != 0;
            const uint32_t ta = (sl.x & ~(kSecondRec | kPointRec)) >> 12;
            const uint64_t kind = two ? kCHead : (sl.x & kPointRec) ? kCPoint : kCFull;
            u64x2 *r = area + 4 * (size_t)(hist[ta] + (sl.x & 0xFFFu));
            r[0] = u64x2{a[0], a[1]};
            r[1] = u64x2{a[2], RT[k] | kind << 62};
            if (kind == kCFull) {
                r[2] = u64x2{b[0], b[1]};
                r[3] = u64x2{b[2], 0};
            }
            if (two) {
                const uint32_t tb = sl.y >> 12;
                u64x2 *r2 = area + 4 * (size_t)(hist[tb] + (sl.y & 0xFFFu));
                r2[0] = u64x2{b[0], b[1]};
                r2[1] = u64x2{b[2], RT[k] | (uint64_t)kCTail << 62};
            }
        }
    }
}

// ---- join ----
// #rows < x (LE: <= x) of the tile: x's word-0 bucket, then a binary search
// of that bucket's rows (sorted order, full-key compares)
// WL: key words staged in LDS (kw, stride kCTRows); words WL .. WG - 1 are
// read from the window itself on a tie (kg: the tile's row 0 of word WL,
// stride glen)
template <int WG, bool LE, int WL = WG>
__device__ __forceinline__ uint32_t tile_count(const uint64_t *kw, const uint32_t *B, int shift,
                                               uint32_t tn, const uint64_t (&x)[WG], bool &found,
                                               const uint64_t *kg = nullptr, size_t glen = 0)
{
    constexpr uint32_t T = kCTRows;
    const uint64_t f0 = kw[0];
    if (x[0] < f0) return 0;
    const uint64_t d = (x[0] - f0) >> shift;
    if (d >= (uint64_t)kTB) return tn;
    const uint32_t span = B[d];
    uint32_t l = span & 0xFFFF, h = span >> 16;
    while (l < h) {
        const uint32_t mid = (l + h) >> 1;
        // word 0 decides unless equal; later words are read only on a tie
        uint64_t v = kw[mid];
        bool below = v < x[0], eq = v == x[0];
#pragma unroll
        for (int w = 1; w < WG; ++w)
            if (eq) {
                v = w < WL ? kw[(size_t)w * T + mid] : kg[(size_t)(w - WL) * glen + mid];
                below = v < x[w];
                eq = v == x[w];
            }
        found |= eq;  // a row equal to x was compared (lower bound: it is the result)
        below = eq ? LE : below;
        l = below ? mid + 1 : l;
        h = below ? h : mid;
    }
    return l;
}

// row r of the tile == x
template <int WG>
__device__ __forceinline__ bool row_eq(const uint64_t *kw, uint32_t r, const uint64_t (&x)[WG])
{
    bool eq = true;
#pragma unroll
    for (int w = 0; w < WG; ++w) eq &= kw[(size_t)w * kCTRows + r] == x[w];
    return eq;
}

// 1024 threads, one record and one row pair each: two 58 KiB workgroups per
// CU hold 32 waves (the CU's limit).  (r05: staging key words 0-1 only, word 2
// read from the window on a tie -- 16 KiB less, room for another stream's
// locate beside two join workgroups -- measured 82.4 vs 78.0 us per batch on
// two streams, the join 42.7 vs 39.0 us)
constexpr int kCJT = 1024;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// the searches of one record after its tile is staged
template <int WG, int WL = WG>
__device__ __forceinline__ void join_search(const ProbeWork &work, const CTiles &ct, uint8_t *flags,
                                            const uint64_t *kw, const uint32_t *rank,
                                            const uint32_t *b16, const uint32_t *b128,
                                            const uint32_t *B, uint32_t kind, const u64x2 (&pl)[2],
                                            const u64x2 ph0, const uint64_t ph1,
                                            const uint64_t *kg = nullptr)
{
    const uint32_t tn = B[kTB] & 0xFFFF;
    const int shift = (int)(B[kTB] >> 16);
    uint64_t lo[WG], hi[WG];
    const uint64_t fl[3] = {pl[0].x, pl[0].y, pl[1].x}, fh[3] = {ph0.x, ph0.y, ph1};
#pragma unroll
    for (int w = 0; w < WG; ++w) lo[w] = fl[w], hi[w] = fh[w];
    const uint64_t rt = pl[1].y;
    const uint32_t rs = (uint32_t)rt, txn = (uint32_t)(rt >> 32);
#ifdef HSC_STAMPS
    if (threadIdx.x == 0 && work.stamps && rs == 0x7FFFFFFF) flags[0] = 1;  // wait for the entry
#endif
    HSC_STAMP(work, 1, 3);
    uint32_t pa = 0, pb = tn;
    // a point: #rows <= lo = #rows < lo + (a row equals lo), and a lower-bound
    // search compares the equal row if there is one
    bool eqa = false, eqb = false;
    if (kind != kCTail) pa = tile_count<WG, false, WL>(kw, B, shift, tn, lo, eqa, kg, ct.len);
    if (kind == kCPoint)
        pb = pa + eqa;
    else if (kind != kCHead)
        pb = tile_count<WG, true, WL>(kw, B, shift, tn, hi, eqb, kg, ct.len);
#ifdef HSC_STAMPS
    if (threadIdx.x == 0 && work.stamps && pa + pb == 0x7FFFFFFF) flags[0] = 1;
#endif
    HSC_STAMP(work, 1, 4);
    // any rank > r(S) in [pa, pb) (a point reads its row); measured: tile
    // prefix / suffix rank maxima for head / tail records cost more in the
    // staging (scans, a barrier, registers) than they saved here
    const bool hit = kind == kCPoint ? pa < pb && rank[pa] > rs
                                     : pa < pb && any_after32(rank, b16, b128, pa, pb, rs);
    if (hit) {
        flags[txn] = 1;
        if (work.bitmap) atomicOr((unsigned long long *)&work.bitmap[txn >> 6], 1ull << (txn & 63));
    }
    HSC_STAMP(work, 1, 5);
}

// Chunk-sorted records: record j of the tile is in the run
// of the chunk whose offset inside the tile (k_plan_s's scan of the tile's
// column) is the last one <= j.  The column is loaded first, staged, each
// thread finds its record's chunk by a 9-step LDS search and loads the whole
// 64-byte record (no bucket entry, no gather) while the rows are in flight.
template <int WG, bool kTile, int WL = WG>
__device__ __forceinline__ void join_item_s(const ProbeWork &work, const CTiles &ct, uint8_t *flags,
                                            uint32_t xi, uint64_t *kw, uint32_t *rank,
                                            uint32_t *b16, uint32_t *b128, uint32_t *B,
                                            uint32_t *Es, uint16_t *Cs)
{
    constexpr uint32_t T = kCTRows;
    const uint32_t tid = threadIdx.x;
    uint32_t tile, j0, j1;
    if constexpr (kTile) {
        tile = xi, j0 = 0;
    } else {
        const uint32_t *d = (const uint32_t *)(work.item_desc + xi);
        tile = sload(d), j0 = sload(d + 1), j1 = sload(d + 2);
    }
    const uint32_t G = work.G;
    const size_t col = (size_t)tile * hist_stride(G);
    uint32_t e = 0, cs = 0;
    if (tid < G) e = work.hist[col + tid], cs = work.cst[col + tid];
    const size_t row = ((size_t)tile << kCTLog2) + 2 * tid;
    u64x2 kv[WL];
#pragma unroll
    for (int w = 0; w < WL; ++w) kv[w] = *(const u64x2 *)(ct.key + (size_t)w * ct.len + row);
    const u32x2 rr = *(const u32x2 *)(ct.rank + row);
    u32x2 bt = {0, 0};
    if (tid < kTBS / 2) bt = *(const u32x2 *)(ct.tb + (size_t)tile * kTBS + 2 * tid);
    if constexpr (kTile) j1 = min(kTileCap, sload(work.counts + tile));
    if (tid < G) Es[tid] = e, Cs[tid] = (uint16_t)cs;
    __syncthreads();
    const uint32_t j = j0 + tid;
    const bool live = j < j1;
    u64x2 A0 = {}, A1 = {}, B0 = {}, B1 = {};
    if (live) {
        uint32_t g = 0;  // Es[0] = 0 <= j
#pragma unroll
        for (int b = 8; b >= 0; --b) {
            const uint32_t c = g + (1u << b);
            if (c < G && Es[c] <= j) g = c;
        }
        const u64x2 *r = (const u64x2 *)ct.recs +
                         4 * ((size_t)g * 2 * work.chunk + Cs[g] + (j - Es[g]));
        A0 = r[0], A1 = r[1], B0 = r[2], B1 = r[3];
    }
#pragma unroll
    for (int w = 0; w < WL; ++w) *(u64x2 *)(kw + (size_t)w * T + 2 * tid) = kv[w];
    *(u32x2 *)(rank + 2 * tid) = rr;
    if (tid < kTBS / 2) *(u32x2 *)(B + 2 * tid) = bt;
    uint32_t m = max(rr.x, rr.y);
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
    if ((tid & 7) == 0) b16[tid >> 3] = m;
#pragma unroll
    for (int d = 8; d < 64; d <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
    if ((tid & 63) == 0) b128[tid >> 6] = m;
    __syncthreads();
    if (!live) return;
    const uint32_t kind = (uint32_t)(A1.y >> 62);
    const uint64_t rt = A1.y & ((1ull << 62) - 1);
    u64x2 pl[2] = {A0, u64x2{A1.x, rt}}, ph0 = B0;
    uint64_t ph1 = B1.x;
    if (kind == kCTail) ph0 = A0, ph1 = A1.x;  // a tail record carries hi in its first half
    // words past WL: read from the window on a tie (the tile's row 0 of word WL)
    const uint64_t *kg = WL < WG ? ct.key + (size_t)WL * ct.len + ((size_t)tile << kCTLog2) : nullptr;
    join_search<WG, WL>(work, ct, flags, kw, rank, b16, b128, B, kind, pl, ph0, ph1, kg);
}

// XCD-contiguous tiles (as the narrow join): measured neutral on config 3
// (1.100 vs 1.108 G checks/s, r02c), so off by default
#ifndef HSC_CJOIN_XCD
#define HSC_CJOIN_XCD 0
#endif
constexpr bool kCJoinXcd = HSC_CJOIN_XCD != 0;
__host__ __device__ inline uint32_t ct_tile_blocks(uint32_t ntiles)
{
    return kCJoinXcd ? 8 * ((ntiles + 7) / 8) : ntiles;
}

template <int WG, int WL = WG>
__global__ __launch_bounds__(kCJT) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_join_c(ProbeWork work, CTiles ct, uint8_t *flags)
{
    constexpr uint32_t T = kCTRows;
    static_assert(T == 2 * kCJT, "a row pair per thread");
    static_assert(kJoinChunk == kCJT && kTileCap == kCJT, "a record per thread");
    extern __shared__ __attribute__((aligned(16))) uint64_t jl[];
    uint64_t *kw = jl;                                   // [WL][T], sorted
    uint32_t *rank = (uint32_t *)(jl + (size_t)WL * T);  // [T], sorted order
    uint32_t *b16 = rank + T;                            // [T / 16]
    uint32_t *b128 = b16 + T / 16;                       // [T / 128]
    uint32_t *B = b128 + T / 128;                        // [kTBS] the tile's bucket table
    uint32_t *Es = B + kTBS;                              // the tile's column
    uint16_t *Cs = (uint16_t *)(Es + kMaxChunks);         // (run starts < 2 * kCChunk)
    // the first xb blocks take the hot tiles' overflow items in turn (dispatched
    // first: they are the fullest), then one block per tile
    const uint32_t xb = gridDim.x - ct_tile_blocks(ct.ntiles);
    if (blockIdx.x >= xb) {
        // neighbouring tiles on one XCD (they share lines of the chunk areas)
        const uint32_t b = blockIdx.x - xb, tb = gridDim.x - xb;
        const uint32_t tile = kCJoinXcd ? xcd_chunk(b, tb / 8) : b;
        if (tile < ct.ntiles) join_item_s<WG, true, WL>(work, ct, flags, tile, kw, rank, b16, b128, B, Es, Cs);
        return;
    }
    const uint32_t nextra = work.item_off[1];
    for (uint32_t xi = blockIdx.x; xi < nextra; xi += xb) {
        __syncthreads();  // the previous item's LDS reads are done
        join_item_s<WG, false, WL>(work, ct, flags, xi, kw, rank, b16, b128, B, Es, Cs);
    }
}

}  // namespace

hipError_t ctiles_build(const uint64_t *cw, size_t cs, int WC, const uint32_t *gid,
                        const uint64_t *lsn, const CTiles &ct, uint64_t *key, uint32_t *rank,
                        uint64_t *first, uint64_t *rel, uint32_t *trad, uint32_t *tb,
                        hipStream_t s)
{
    if (ct.len == 0 || ct.ntiles == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((ct.len + 255) / 256);
    switch (ct.WG) {
    case 1: k_ct_rows<1><<<blocks, 256, 0, s>>>(cw, cs, WC, gid, lsn, ct, key, rank, first); break;
    case 2: k_ct_rows<2><<<blocks, 256, 0, s>>>(cw, cs, WC, gid, lsn, ct, key, rank, first); break;
    case 3: k_ct_rows<3><<<blocks, 256, 0, s>>>(cw, cs, WC, gid, lsn, ct, key, rank, first); break;
    default: return hipErrorInvalidValue;
    }
    k_ct_rel<<<(ct.ntiles + 255) / 256, 256, 0, s>>>(first, ct.ntiles, rel);
    k_ct_tbuckets<<<ct.ntiles, 256, 0, s>>>(ct, key, tb);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return narrow_trad_build(rel, ct.ntiles, ct.trad_m, trad, s);
}

size_t ctiles_locate_lds(const CTiles &ct) { return cloc_lds(ct).bytes; }
uint32_t ctiles_chunk() { return kCChunk; }

hipError_t launch_locate_c(const CTiles &ct, const WinView &wt, const ProbeView &p,
                           const uint64_t *clo, const uint64_t *chi, const ProbeWork &work,
                           uint8_t *flags, hipStream_t s)
{
    if (p.n == 0 && p.n_lock == 0) return hipSuccess;
    const size_t lds = cloc_lds(ct).bytes;
    const uint32_t blocks = 8 * ((work.G + 7) / 8);
#define HSC_LOC_C(WG_) \
    k_locate_c<WG_><<<blocks, kCLocThreads, lds, s>>>(ct, wt, p, clo, chi, work, flags)
    switch (ct.WG) {
    case 1: HSC_LOC_C(1); break;
    case 2: HSC_LOC_C(2); break;
    case 3: HSC_LOC_C(3); break;
    default: return hipErrorInvalidValue;
    }
#undef HSC_LOC_C
    return hipGetLastError();
}

hipError_t launch_join_c(const CTiles &ct, const ProbeWork &work, uint32_t max_items,
                         uint8_t *flags, hipStream_t s)
{
    if (max_items == 0 || ct.n == 0 || ct.ntiles == 0) return hipSuccess;
    const uint32_t extra = max_items - ct.ntiles;
    const uint32_t blocks = ct_tile_blocks(ct.ntiles) + (extra < 512 ? extra : 512);
    // key words staged per tile (HSC_CJOIN_WL, A/B; default all): the rest
    // are read from the window on a tie
    static const int wl_env = getenv("HSC_CJOIN_WL") ? atoi(getenv("HSC_CJOIN_WL")) : 0;
    const int WL = wl_env >= 1 && wl_env < ct.WG ? wl_env : ct.WG;
    const size_t lds = 8 * (size_t)WL * kCTRows + 4 * (size_t)kCTRows + 4 * (kCTRows / 16) +
                       4 * (kCTRows / 128) + 4 * kTBS + 6 * (size_t)kMaxChunks;
#define HSC_JOIN_C(WG_, WL_) k_join_c<WG_, WL_><<<blocks, kCJT, lds, s>>>(work, ct, flags)
    switch (ct.WG * 4 + WL) {
    case 1 * 4 + 1: HSC_JOIN_C(1, 1); break;
    case 2 * 4 + 1: HSC_JOIN_C(2, 1); break;
    case 2 * 4 + 2: HSC_JOIN_C(2, 2); break;
    case 3 * 4 + 1: HSC_JOIN_C(3, 1); break;
    case 3 * 4 + 2: HSC_JOIN_C(3, 2); break;
    case 3 * 4 + 3: HSC_JOIN_C(3, 3); break;
    default: return hipErrorInvalidValue;
    }
#undef HSC_JOIN_C
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_ctiles()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_ct_rel);
}

}  // namespace hsc
