// hsc_narrow.hip -- the narrow window layout and its probe pipeline.
//
// The reference re-compares every logged write key against every read range
// of its index with min-length memcmp (db/glue.c:2937-2961).  The wide layout
// (hsc_kernels.hip) keeps every key as W big-endian u64 words; this one keeps
// a window tile of 4096 sorted rows as
//
//   key32[i] = (K_i - K_t) >> s         K = gid || word 0 || ... || word W-1,
//                                       K_t = the tile's first row,
//   lsn[i]   (u64, max commit LSN of the key)
//
// which is exact whenever every tile spans less than 2^32 << s: s counts the
// low bits of K that are the same in every row -- whole trailing words that
// never vary (zero padding of shorter key groups) plus tz low bits of the
// last word that does (a 9-byte int64 index key, 0x08 || BE(v ^ 2^63), has
// its last byte in the top of word 1: tz = 56).  A probe bound X maps into
// tile t exactly:
//
//   rows >= X  <=>  key32 >= ceil((X - K_t) / 2^s)   (0 if X <= K_t)
//   rows <= X  <=>  key32 <= floor((X - K_t) / 2^s)  (none if X < K_t)
//
// so the join stages 12 B per row instead of 8W + 8 B and its records carry
// two u32 bounds instead of 2W words.  Group boundaries need no row spans:
// gid is the most significant limb of K, so rows of other groups fall
// outside [g || lo, g || hi] by themselves.
//
//   locate  (one thread / range): splitter search in LDS -> end tiles; whole
//           middle tiles from the tile-max sparse table; per end tile the
//           tile-relative u32 bounds (a tile the range covers whole is
//           answered from its tile max); one returning atomic per record on
//           the tile's counter gives the record's rank in its bucket.
//   plan    (one workgroup): bucket offsets, join items; re-zeroes counters.
//   scatter (one thread / range): record -> bucket_off[tile] + rank.
//   join    (one workgroup / <= 1024 records of a tile): stages the tile's
//           key32 + lsn in LDS, two lockstep binary searches per record,
//           range max from 16/256-row block maxima.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace hsc {

constexpr uint32_t kNoTile = 0xFFFFFFFFu;
constexpr uint64_t kRelNone = 1ull << 33;  // saturated delta: beyond every row

// (X - B) >> shift for composite keys X = (xg, xw[j * xs]) and B = (bg,
// bw[j * bs]), limbs most significant first: limb 0 = gid, limb j + 1 = word
// j.  shift = tz bits of limb lw plus every limb after lw (the window's rows
// agree on all of those bits).  Returns false if X < B.  Otherwise v =
// min((X - B) >> shift, kRelNone) and rem = whether the shifted-out bits of
// X - B are nonzero.
__device__ __forceinline__ bool rel_diff(int W, int lw, int tz, uint32_t xg, const uint64_t *xw,
                                         size_t xs, uint32_t bg, const uint64_t *bw, size_t bs,
                                         uint64_t &v, bool &rem)
{
    uint64_t borrow = 0, d_last = 0, d_prev = 0, high = 0, below = 0;
    for (int i = W; i >= 0; --i) {
        const uint64_t x = i ? xw[(size_t)(i - 1) * xs] : (uint64_t)xg;
        const uint64_t b = i ? bw[(size_t)(i - 1) * bs] : (uint64_t)bg;
        const uint64_t d = x - b - borrow;
        borrow = (x < b) | ((x == b) & (borrow != 0));
        if (i > lw)
            below |= d;
        else if (i == lw)
            d_last = d;
        else if (i == lw - 1)
            d_prev = d;
        else
            high |= d;
    }
    if (borrow) return false;
    rem = (below != 0) | (tz ? (d_last & ((1ull << tz) - 1)) != 0 : false);
    const uint64_t top = tz ? d_prev >> tz : d_prev;
    const uint64_t low = tz ? (d_last >> tz) | (d_prev << (64 - tz)) : d_last;
    v = (high | top) ? kRelNone : (low < kRelNone ? low : kRelNone);
    return true;
}

// Tile-relative lower bound: smallest delta d with K_t + (d << s) >= X
// (> 0xFFFFFFFF: no row of the tile).
__device__ __forceinline__ uint64_t rel_lo(const WinView &w, uint32_t t, uint32_t g,
                                           const uint64_t *xw, size_t xs)
{
    uint64_t v;
    bool rem;
    if (!rel_diff(w.W, w.lw, w.tz, g, xw, xs, w.sp_g[t], w.sp_w + t, w.ntiles, v, rem)) return 0;
    return v + (rem ? 1 : 0);
}

// Tile-relative upper bound: largest delta d with K_t + (d << s) <= X
// (-1: no row of the tile).
__device__ __forceinline__ int64_t rel_hi(const WinView &w, uint32_t t, uint32_t g,
                                          const uint64_t *xw, size_t xs)
{
    uint64_t v;
    bool rem;
    if (!rel_diff(w.W, w.lw, w.tz, g, xw, xs, w.sp_g[t], w.sp_w + t, w.ntiles, v, rem)) return -1;
    return v < 0xFFFFFFFFull ? (int64_t)v : (int64_t)0xFFFFFFFFull;
}

// ============================================================================
// window build
// ============================================================================
// flag := 1 if some tile spans >= 2^32 << s (or its rows disagree on the
// s shifted-out bits).
__global__ void k_narrow_check(WinView w, uint32_t *flag)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.ntiles) return;
    const size_t f = (size_t)t << w.log2T;
    const size_t l = std::min<size_t>(w.n, f + ((size_t)1 << w.log2T)) - 1;
    uint64_t v;
    bool rem;
    const bool ge = rel_diff(w.W, w.lw, w.tz, w.gid[l], w.words + l, w.stride, w.gid[f],
                             w.words + f, w.stride, v, rem);
    if (!ge || rem || v > 0xFFFFFFFFull) atomicOr(flag, 1u);
}

__global__ void k_narrow_keys(WinView w, uint32_t *key32)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= w.n) return;
    const uint32_t t = (uint32_t)(i >> w.log2T);
    uint64_t v = 0;
    bool rem;
    rel_diff(w.W, w.lw, w.tz, w.gid[i], w.words + i, w.stride, w.sp_g[t], w.sp_w + t, w.ntiles,
             v, rem);
    key32[i] = (uint32_t)v;
}

hipError_t narrow_check(const WinView &w, uint32_t *flag, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || w.ntiles == 0) return e;
    k_narrow_check<<<(w.ntiles + 255) / 256, 256, 0, s>>>(w, flag);
    return hipGetLastError();
}

hipError_t narrow_keys(const WinView &w, uint32_t *key32, hipStream_t s)
{
    if (w.n == 0) return hipSuccess;
    k_narrow_keys<<<(w.n + 255) / 256, 256, 0, s>>>(w, key32);
    return hipGetLastError();
}

// ============================================================================
// probe
// ============================================================================
constexpr int kLocBatch = 2;  // probes per thread (one batch per thread)

// Record of probe q in tile t with bounds [lo, hi] (already non-empty):
// answered from the tile max when it covers the whole tile, else ranked.
__device__ __forceinline__ uint4 make_record(const WinView &w, const NarrowWork &nw, uint32_t t,
                                             uint32_t lo, uint32_t hi, uint64_t snap,
                                             uint8_t *verdict, uint32_t txn)
{
    if (lo == 0 && hi == 0xFFFFFFFFu) {
        if (w.tmax[t] > snap) verdict[txn] = 1;
        return make_uint4(kNoTile, 0, 0, 0);
    }
#ifdef HSC_AB_NOATOMIC  // A/B timing only: ranks collide, verdicts wrong
    const uint32_t r = 0;
#else
    const uint32_t r = atomicAdd(&nw.counts[(size_t)t * kCntStride], 1u);
#endif
    return make_uint4(t, r, lo, hi);
}

// Plan, run by the last locate workgroup to finish: bucket offsets, the
// overflow join items (chunks after a tile's first kJoinChunk records; the
// first chunk of tile t is join workgroup t), counters back to zero.
__device__ void plan_tiles(const NarrowWork &nw, uint32_t ntiles, uint32_t *lds)
{
    uint32_t carry_b = 0, carry_i = 0;
    for (uint32_t base = 0; base < ntiles; base += 4 * kLocateThreads) {
        const uint32_t t0 = base + 4 * threadIdx.x;
        uint32_t cv[4], ch[4], sb = 0, si = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            cv[k] = t0 + k < ntiles
                        ? __hip_atomic_load(&nw.counts[(size_t)(t0 + k) * kCntStride],
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (t0 + k < ntiles)
                __hip_atomic_store(&nw.counts[(size_t)(t0 + k) * kCntStride], 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            ch[k] = cv[k] > (uint32_t)kJoinChunk ? (cv[k] - 1) / kJoinChunk : 0;
            sb += cv[k];
            si += ch[k];
        }
        uint32_t tb, ti;
        uint32_t pb = block_excl_scan<kLocateThreads>(sb, lds, tb);
        uint32_t pi = block_excl_scan<kLocateThreads>(si, lds, ti);
        pb += carry_b;
        pi += carry_i;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = t0 + k;
            if (t < ntiles) {
                nw.bucket_off[t] = pb;
                for (uint32_t j = 0; j < ch[k]; ++j) {
                    nw.item_tile[pi + j] = t;
                    nw.item_chunk[pi + j] = j + 1;
                }
            }
            pb += cv[k];
            pi += ch[k];
        }
        carry_b += tb;
        carry_i += ti;
    }
    if (threadIdx.x == 0) {
        nw.bucket_off[ntiles] = carry_b;
        nw.n_extra[0] = carry_i;
    }
}

__global__ __launch_bounds__(kLocateThreads) void k_locate_n(WinView w, ProbeView p,
                                                             NarrowWork nw, uint8_t *verdict,
                                                             uint32_t ntop, uint32_t stride_t)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t scan_lds[16];
    __shared__ uint32_t last;
    uint64_t *top = (uint64_t *)smem;  // [ntop] splitter prefixes
    const size_t ks = p.n;
    const uint32_t c0 = blockIdx.x * nw.chunk;
    const uint32_t c1 = min(p.n, c0 + nw.chunk);
    // this thread's probes: every load issued before the splitter staging
    constexpr int NS = 2 * kLocBatch;
    uint32_t qq[kLocBatch];
    bool valid[kLocBatch];
    uint32_t gg[NS];
    uint64_t k0[NS];
    const uint64_t *km[NS];
    bool leq[NS];
    uint32_t cnt[NS];
    uint64_t sn[kLocBatch];
    uint32_t tx[kLocBatch];
#pragma unroll
    for (int b = 0; b < kLocBatch; ++b) {
        qq[b] = c0 + b * kLocateThreads + threadIdx.x;
        valid[b] = qq[b] < c1;
        const uint32_t q = valid[b] ? qq[b] : (c0 < p.n ? c0 : 0);
        const bool any = p.n > 0;
        const uint32_t g = any ? p.gid[q] : 0;
        gg[2 * b] = gg[2 * b + 1] = g;
        k0[2 * b] = any ? p.lo[q] : 0;
        k0[2 * b + 1] = any ? p.hi[q] : 0;
        km[2 * b] = p.lo + q;
        km[2 * b + 1] = p.hi + q;
        leq[2 * b] = false;
        leq[2 * b + 1] = true;
        sn[b] = any ? p.snap[q] : 0;
        tx[b] = any ? p.txn[q] : 0;
    }
    for (uint32_t base = 0; base < ntop; base += 8 * kLocateThreads) {
        uint64_t vw[8];
        uint32_t vg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = base + k * kLocateThreads + threadIdx.x;
#ifdef HSC_AB_NOSTAGE
            vw[k] = 0x0880000000000000ull + ((uint64_t)i << 32);
            vg[k] = 0;
#else
            if (i < ntop) {
                vw[k] = w.sp_w[(size_t)i * stride_t];
                vg[k] = w.sp_g[(size_t)i * stride_t];
            }
#endif
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = base + k * kLocateThreads + threadIdx.x;
            if (i < ntop) top[i] = key_prefix(w.gbits, vg[k], vw[k]);
        }
    }
    __syncthreads();

    if (c0 < c1) {
        count_splitters<NS>(w, top, ntop, stride_t, gg, k0, km, ks, leq, cnt);
        uint64_t mid[kLocBatch];
#pragma unroll
        for (int b = 0; b < kLocBatch; ++b) {
            const uint32_t c = cnt[2 * b], c2 = cnt[2 * b + 1];
            const uint32_t a = c ? c - 1 : 0, bt = c2 ? c2 - 1 : 0;
            const bool need = valid[b] && c2 > 0 && bt > a + 1;
            mid[b] = need ? tiles_max(w, a + 1, bt - 1) : 0;
        }
#pragma unroll
        for (int b = 0; b < kLocBatch; ++b) {
            if (!valid[b]) continue;
            const uint32_t q = qq[b];
            const uint32_t c = cnt[2 * b], c2 = cnt[2 * b + 1];
            uint4 ra = make_uint4(kNoTile, 0, 0, 0), rb = ra;
            const uint32_t a = c ? c - 1 : 0, bt = c2 ? c2 - 1 : 0;
            if (c2 > 0 && a <= bt) {
                if (mid[b] > sn[b]) {
                    verdict[tx[b]] = 1;
                } else if (a == bt) {
#ifdef HSC_AB_NOREL
                    const uint64_t lo = 1;
                    const int64_t hi = 2;
#else
                    const uint64_t lo = rel_lo(w, a, gg[2 * b], p.lo + q, ks);
                    const int64_t hi = rel_hi(w, a, gg[2 * b], p.hi + q, ks);
#endif
                    if (lo <= 0xFFFFFFFFull && hi >= 0 && (int64_t)lo <= hi)
                        ra = make_record(w, nw, a, (uint32_t)lo, (uint32_t)hi, sn[b], verdict, tx[b]);
                } else {
                    const uint64_t lo = rel_lo(w, a, gg[2 * b], p.lo + q, ks);
                    const int64_t hi = rel_hi(w, bt, gg[2 * b], p.hi + q, ks);
                    if (lo <= 0xFFFFFFFFull)
                        ra = make_record(w, nw, a, (uint32_t)lo, 0xFFFFFFFFu, sn[b], verdict, tx[b]);
                    if (hi >= 0)
                        rb = make_record(w, nw, bt, 0, (uint32_t)hi, sn[b], verdict, tx[b]);
                }
            }
            nw.code[2 * (size_t)q] = ra;
            nw.code[2 * (size_t)q + 1] = rb;
        }
    }
    // table locks: any write to a locked table after the snapshot
    for (uint32_t q = blockIdx.x * kLocateThreads + threadIdx.x; q < p.n_lock;
         q += gridDim.x * kLocateThreads) {
        const uint32_t t = p.lock_table[q];
        if (t < w.ntables && w.table_max[t] > p.lock_snap[q]) verdict[p.lock_txn[q]] = 1;
    }
    if (w.ntiles == 0 || p.n == 0) return;
    // The last workgroup to finish plans the buckets.  The plan reads only
    // the counters, and every access to them is a device-scope atomic or an
    // sc1 store (no L1/L2 copy can go stale): each counter add of this
    // workgroup has returned -- it was performed -- before the barrier, so no
    // release/acquire fence is needed around the arrival counter.
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = atomicAdd(nw.done, 1u);
        last = prev == gridDim.x - 1;
        if (last) __hip_atomic_store(nw.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
#ifdef HSC_AB_NOPLAN
    return;
#endif
    plan_tiles(nw, w.ntiles, scan_lds);
}

hipError_t launch_locate_n(const WinView &w, const ProbeView &p, const NarrowWork &nw,
                           uint8_t *verdict, hipStream_t s)
{
    if (p.n == 0 && p.n_lock == 0) return hipSuccess;
    uint32_t ntop = 0, stride_t = 1;
    if (w.n) {
        stride_t = (w.ntiles + kTopCap - 1) / kTopCap;
        ntop = (w.ntiles + stride_t - 1) / stride_t;
    }
    k_locate_n<<<nw.G, kLocateThreads, (size_t)ntop * 8 + 16, s>>>(w, p, nw, verdict, ntop,
                                                                   stride_t);
    return hipGetLastError();
}

constexpr int kScatThreads = 256;

__global__ __launch_bounds__(kScatThreads) void k_scatter_n(ProbeView p, NarrowWork nw)
{
    const uint32_t q = blockIdx.x * kScatThreads + threadIdx.x;
    if (q >= p.n) return;
    const uint4 a = nw.code[2 * (size_t)q], b = nw.code[2 * (size_t)q + 1];
    if (a.x == kNoTile && b.x == kNoTile) return;
    const uint64_t snap = p.snap[q];
    const uint32_t txn = p.txn[q];
    const uint32_t sa = a.x != kNoTile ? nw.bucket_off[a.x] + a.y : 0;
    const uint32_t sb = b.x != kNoTile ? nw.bucket_off[b.x] + b.y : 0;
    if (a.x != kNoTile) {
        nw.recs[sa] = make_uint4(a.z, a.w, (uint32_t)snap, (uint32_t)(snap >> 32));
        nw.rtxn[sa] = txn;
    }
    if (b.x != kNoTile) {
        nw.recs[sb] = make_uint4(b.z, b.w, (uint32_t)snap, (uint32_t)(snap >> 32));
        nw.rtxn[sb] = txn;
    }
}

hipError_t launch_scatter_n(const WinView &w, const ProbeView &p, const NarrowWork &nw,
                            hipStream_t s)
{
    (void)w;
    if (p.n == 0) return hipSuccess;
    k_scatter_n<<<(p.n + kScatThreads - 1) / kScatThreads, kScatThreads, 0, s>>>(p, nw);
    return hipGetLastError();
}

// Join workgroup b < ntiles: the first kJoinChunk records of tile b (its
// staging loads start at once: no item lookup in front of them); b >= ntiles:
// overflow item b - ntiles.  CHECK_FIRST: skip a tile without records before
// staging it (sparse batches); otherwise the record count is read while the
// tile's loads are in flight.
template <int LOG2T, bool CHECK_FIRST>
__global__ __launch_bounds__(kJoinThreads) void k_join_n(WinView w, NarrowWork nw,
                                                         uint8_t *verdict)
{
    constexpr uint32_t T = 1u << LOG2T;
    static_assert(T == 8 * kJoinThreads, "a thread stages 8 consecutive rows");
    __shared__ __attribute__((aligned(16))) uint32_t keys[T];
    __shared__ __attribute__((aligned(16))) uint64_t lsn[T];
    __shared__ uint64_t b16[T / 16];
    __shared__ uint64_t b256[T / 256];
    uint32_t tile, chunk = 0;
    if (blockIdx.x < w.ntiles) {
        tile = blockIdx.x;
    } else {
        const uint32_t e = blockIdx.x - w.ntiles;
        if (e >= nw.n_extra[0]) return;
        tile = nw.item_tile[e];
        chunk = nw.item_chunk[e];
    }
    const uint32_t rb = nw.bucket_off[tile] + chunk * kJoinChunk;
    uint32_t re = 0;
    if (CHECK_FIRST) {
        re = min(rb + (uint32_t)kJoinChunk, nw.bucket_off[tile + 1]);
        if (rb >= re) return;
    }
    const uint32_t ts = tile << LOG2T;
    const uint32_t tn = min(T, w.n - ts);
    // stage rows [8 tid, 8 tid + 8): keys (2 x 16 B) and lsn (4 x 16 B); the
    // window arrays are padded to whole tiles, rows >= tn are never searched
    const uint4 *ksrc = (const uint4 *)(w.key32 + ts) + 2 * threadIdx.x;
    const ulonglong2 *lsrc = (const ulonglong2 *)(w.lsn + ts) + 4 * threadIdx.x;
    const uint4 kv0 = ksrc[0], kv1 = ksrc[1];
    const ulonglong2 l0 = lsrc[0], l1 = lsrc[1], l2 = lsrc[2], l3 = lsrc[3];
    if (!CHECK_FIRST) {
        re = min(rb + (uint32_t)kJoinChunk, nw.bucket_off[tile + 1]);
        if (rb >= re) return;  // uniform across the workgroup
    }
    constexpr int kRec = kJoinChunk / kJoinThreads;
    uint4 rec[kRec];
    uint32_t rt[kRec];
#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t r = rb + k * kJoinThreads + threadIdx.x;
        if (r < re) {
            rec[k] = nw.recs[r];
            rt[k] = nw.rtxn[r];
        }
    }
    ((uint4 *)keys)[2 * threadIdx.x] = kv0;
    ((uint4 *)keys)[2 * threadIdx.x + 1] = kv1;
    ulonglong2 *ldst = (ulonglong2 *)lsn + 4 * threadIdx.x;
    ldst[0] = l0;
    ldst[1] = l1;
    ldst[2] = l2;
    ldst[3] = l3;
    // block maxima from registers: 8 rows here, 16 with the neighbour lane,
    // 256 over 32 lanes
    uint64_t m = l0.x > l0.y ? l0.x : l0.y;
    m = l1.x > m ? l1.x : m;
    m = l1.y > m ? l1.y : m;
    m = l2.x > m ? l2.x : m;
    m = l2.y > m ? l2.y : m;
    m = l3.x > m ? l3.x : m;
    m = l3.y > m ? l3.y : m;
    uint64_t o = __shfl_xor(m, 1, 64);
    m = o > m ? o : m;
    if ((threadIdx.x & 1) == 0) b16[threadIdx.x >> 1] = m;
#pragma unroll
    for (int d = 2; d < 32; d <<= 1) {
        o = __shfl_xor(m, d, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 31) == 0) b256[threadIdx.x >> 5] = m;
    __syncthreads();

#ifdef HSC_AB_NOSEARCH  // A/B timing only: staging without the searches
    if (rec[0].x == 0x12345678u && rt[0] == 7u) verdict[0] = keys[threadIdx.x] + lsn[threadIdx.x];
    return;
#endif
#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t r = rb + k * kJoinThreads + threadIdx.x;
        if (r >= re) continue;
        const uint32_t lo = rec[k].x, hi = rec[k].y;
        const uint64_t snap = (uint64_t)rec[k].z | ((uint64_t)rec[k].w << 32);
        // p = #keys < lo, q = #keys <= hi over rows [0, tn), in lockstep
        uint32_t pp = 0, qq = 0;
#pragma unroll
        for (uint32_t step = T; step > 0; step >>= 1) {
            if (pp + step <= tn && keys[pp + step - 1] < lo) pp += step;
            if (qq + step <= tn && keys[qq + step - 1] <= hi) qq += step;
        }
        if (pp < qq && lds_any_after<T / 256>(lsn, b16, b256, pp, qq, snap)) verdict[rt[k]] = 1;
    }
}

hipError_t launch_join_n(const WinView &w, const NarrowWork &nw, uint32_t max_extra,
                         bool sparse, uint8_t *verdict, hipStream_t s)
{
    if (w.n == 0 || w.ntiles == 0) return hipSuccess;
    if (w.log2T != kNarrowLog2T) return hipErrorInvalidValue;
    const uint32_t grid = w.ntiles + max_extra;
    if (sparse)
        k_join_n<kNarrowLog2T, true><<<grid, kJoinThreads, 0, s>>>(w, nw, verdict);
    else
        k_join_n<kNarrowLog2T, false><<<grid, kJoinThreads, 0, s>>>(w, nw, verdict);
    return hipGetLastError();
}

}  // namespace hsc
