// hsc_device.h -- device helpers shared by the probe kernels of the wide
// (hsc_kernels.hip) and narrow (hsc_narrow.hip) window layouts.
#pragma once
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

namespace hsc {

// Hacker's Delight compress / expand of the bits of x under mask m, with the
// moves of compress_moves(m) (the packed sorts, hsc_ingest.hip; the graph's
// packed writer search, hsc_graph.hip): compress keeps the order of values
// that agree outside m.
__device__ __forceinline__ uint64_t bits_compress(uint64_t x, uint64_t m, const uint64_t (&mv)[6])
{
    x &= m;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const uint64_t t = x & mv[i];
        x = (x ^ t) | (t >> (1 << i));
    }
    return x;
}

__device__ __forceinline__ uint64_t bits_expand(uint64_t x, uint64_t m, const uint64_t (&mv)[6])
{
#pragma unroll
    for (int i = 5; i >= 0; --i) x = (x & ~mv[i]) | ((x << (1 << i)) & mv[i]);
    return x & m;
}

// Native vectors: register arrays of these stay in VGPRs (arrays of the HIP
// uint4 / ulonglong2 structs can be demoted to scratch).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t y = __shfl_xor(v, o, 64);
        v = y > v ? y : v;
    }
    return v;
}

// Exclusive block scan of one u32 per thread; NT threads.
// 64-bit variant of block_excl_scan (two packed 32-bit sums that never carry).
template <int NT>
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *lds, uint64_t &total)
{
    constexpr int NW = NT / 64;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint64_t s = lane < NW ? lds[lane] : 0;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            const uint64_t y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < NW) lds[lane] = s;
    }
    __syncthreads();
    const uint64_t pre = wid ? lds[wid - 1] : 0;
    total = lds[NW - 1];
    __syncthreads();
    return pre + x - v;
}

template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds, uint32_t &total)
{
    constexpr int NW = NT / 64;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint32_t s = lane < NW ? lds[lane] : 0;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            uint32_t y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < NW) lds[lane] = s;
    }
    __syncthreads();
    uint32_t pre = wid ? lds[wid - 1] : 0;
    total = lds[NW - 1];
    __syncthreads();
    return pre + x - v;
}

// sign(A - B) for two keys of W words: A's word 0 is in a register, its word
// j >= 1 at a_mem[j * as]; B's word j at b0[j * bs].
__device__ __forceinline__ int cmp_words(int W, uint64_t a_w0, const uint64_t *a_mem, size_t as,
                                         const uint64_t *b0, size_t bs)
{
    uint64_t b = b0[0];
    if (a_w0 != b) return a_w0 < b ? -1 : 1;
    for (int j = 1; j < W; ++j) {
        const uint64_t a = a_mem[(size_t)j * as];
        b = b0[(size_t)j * bs];
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// 64-bit prefix of a composite key (gid, w0, ...): gid in the top gbits,
// then the top 64 - gbits bits of w0.  Prefix order agrees with composite
// order wherever two prefixes differ; equal prefixes need the full compare.
__device__ __forceinline__ uint64_t key_prefix(int gbits, uint32_t g, uint64_t w0)
{
    return gbits ? ((uint64_t)g << (64 - gbits)) | (w0 >> gbits) : w0;
}

// sign(full splitter of tile t - (g, key)), splitter read from sp_g / sp_w.
__device__ __forceinline__ int cmp_splitter_full(const WinView &w, uint32_t t, uint32_t g,
                                                 uint64_t k0, const uint64_t *kmem, size_t ks)
{
    const uint32_t sg = w.sp_g[t];
    if (sg != g) return sg < g ? -1 : 1;
    return -cmp_words(w.W, k0, kmem, ks, w.sp_w + t, w.ntiles);
}

// NS binary searches in lockstep over the splitters: out[i] = number of
// tiles whose first row compares < key i (leq[i]: <=).  LDS holds the 64-bit
// prefix of every stride_t-th splitter; ties and (stride_t > 1) the last
// step go to sp_g / sp_w.
template <int NS>
__device__ __forceinline__ void count_splitters(const WinView &w, const uint64_t *top,
                                                uint32_t ntop, uint32_t stride_t,
                                                const uint32_t (&g)[NS],
                                                const uint64_t (&k0)[NS],
                                                const uint64_t *const (&kmem)[NS], size_t ks,
                                                const bool (&leq)[NS], uint32_t (&out)[NS])
{
    uint32_t lo[NS], hi[NS];
    uint64_t pk[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        lo[i] = 0;
        hi[i] = ntop;
        pk[i] = key_prefix(w.gbits, g[i], k0[i]);
    }
    for (;;) {
        bool any = false;
        uint64_t sp[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) sp[i] = top[min((lo[i] + hi[i]) >> 1, ntop ? ntop - 1 : 0)];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (lo[i] < hi[i]) {
                any = true;
                const uint32_t m = (lo[i] + hi[i]) >> 1;
                const int c = sp[i] != pk[i] ? (sp[i] < pk[i] ? -1 : 1)
                                             : cmp_splitter_full(w, m * stride_t, g[i], k0[i], kmem[i], ks);
                if (leq[i] ? c <= 0 : c < 0)
                    lo[i] = m + 1;
                else
                    hi[i] = m;
            }
        }
        if (!any) break;
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const uint32_t t = lo[i];
        if (t == 0 || stride_t == 1) {
            out[i] = min(t * stride_t, w.ntiles);
            continue;
        }
        uint32_t L = (t - 1) * stride_t + 1, H = min(t * stride_t, w.ntiles);
        while (L < H) {
            const uint32_t m = (L + H) >> 1;
            const int c = cmp_splitter_full(w, m, g[i], k0[i], kmem[i], ks);
            if (leq[i] ? c <= 0 : c < 0)
                L = m + 1;
            else
                H = m;
        }
        out[i] = L;
    }
}

__device__ __forceinline__ uint64_t tiles_max(const WinView &w, uint32_t x, uint32_t y)
{
    uint32_t len = y - x + 1;
    int k = 31 - __clz(len);
    const uint64_t *lv = w.tmax + (size_t)k * w.ntiles;
    uint64_t a = lv[x], b = lv[y - (1u << k) + 1];
    return a > b ? a : b;
}

// Any lsn > snap in [from, to) of a[] (to - from <= N), N independent LDS
// reads (predicated), no dependent branch chain.
template <int N>
__device__ __forceinline__ bool any_gt(const uint64_t *a, uint32_t from, uint32_t to, uint64_t snap)
{
    bool r = false;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const uint32_t i = from + k;
        const uint64_t v = a[i < to ? i : from];
        r |= (i < to) & (v > snap);
    }
    return r;
}

// Any lsn > snap in rows [p, q) (non-empty) of the tile, with 16- and
// 256-row block maxima; NB256 = 256-row blocks per tile.
template <int NB256 = 8>
__device__ __forceinline__ bool lds_any_after(const uint64_t *lsn, const uint64_t *b16,
                                              const uint64_t *b256, uint32_t p, uint32_t q,
                                              uint64_t snap)
{
    if (q - p <= 2) return any_gt<2>(lsn, p, q, snap);
    if (q - p <= 16) return any_gt<16>(lsn, p, q, snap);
    const uint32_t p16 = (p + 15) & ~15u, q16 = q & ~15u;
    if (any_gt<15>(lsn, p, p16, snap) || any_gt<15>(lsn, q16, q, snap)) return true;
    const uint32_t bp = p16 >> 4, bq = q16 >> 4;  // 16-blocks [bp, bq)
    const uint32_t bp256 = (bp + 15) & ~15u, bq256 = bq & ~15u;
    if (bp256 > bq256) return any_gt<15>(b16, bp, bq, snap);  // no 256-boundary inside
    return any_gt<15>(b16, bp, bp256, snap) || any_gt<15>(b16, bq256, bq, snap) ||
           any_gt<NB256>(b256, bp256 >> 4, bq256 >> 4, snap);
}

// u32 variants over 32-bit commit times (narrow and compact tiles): any
// rank > s in [from, to) (to - from <= N), and in rows [p, q) of a tile with
// 16- and 128-row block maxima b16 / b128.
template <int N>
__device__ __forceinline__ bool any_gt32(const uint32_t *a, uint32_t from, uint32_t to, uint32_t s)
{
    bool r = false;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const uint32_t i = from + k;
        const uint32_t v = a[i < to ? i : from];
        r |= (i < to) & (v > s);
    }
    return r;
}

__device__ __forceinline__ bool any_after32(const uint32_t *rank, const uint32_t *b16,
                                            const uint32_t *b128, uint32_t p, uint32_t q,
                                            uint32_t s)
{
    const uint32_t q1 = q - 1;
    const bool hot_p = b16[p >> 4] > s, hot_q = b16[q1 >> 4] > s;
    if (!hot_p && !hot_q && (q1 >> 4) <= (p >> 4) + 1) return false;
    if (q - p <= 16) {  // short range: only its own rows (a wave runs its longest lane's count)
        bool r = false;
        for (uint32_t i = p; i < q; ++i) r |= rank[i] > s;
        return r;
    }
    const uint32_t p16 = (p + 15) & ~15u, q16 = q & ~15u;
    const uint32_t bp = p16 >> 4, bq = q16 >> 4;
    const uint32_t bp8 = min((bp + 7) & ~7u, bq), bq8 = max(bq & ~7u, bp8);
    bool r = false;
    if (hot_p) r |= any_gt32<15>(rank, p, p16, s);
    if (hot_q) r |= any_gt32<15>(rank, q16, q, s);
    r |= any_gt32<7>(b16, bp, bp8, s);
    r |= any_gt32<7>(b16, bq8, bq, s);
    if (bp8 < bq8) r |= any_gt32<32>(b128, bp8 >> 3, bq8 >> 3, s);
    return r;
}

// Block-uniform load through the constant address space: a scalar load,
// counted apart from the vector loads (waiting for it drains none of them).
template <class T>
__device__ __forceinline__ T sload(const T *p)
{
    return *(const __attribute__((address_space(4))) T *)p;
}

// ---- delta run (hsc_delta.hip) ---------------------------------------------
// sign of (gid, words) of row i of a [W][stride] SoA against (g, key words)
__device__ __forceinline__ int row_cmp(const uint32_t *gid, const uint64_t *words, size_t stride,
                                       int W, uint32_t i, uint32_t g, const uint64_t *key,
                                       size_t kstride)
{
    const uint32_t rg = gid[i];
    if (rg != g) return rg < g ? -1 : 1;
    for (int j = 0; j < W; ++j) {
        const uint64_t a = words[(size_t)j * stride + i], b = key[(size_t)j * kstride];
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// #rows of d < key (strict = true) or <= key (strict = false)
__device__ __forceinline__ uint32_t delta_count(const DeltaView &d, uint32_t g, const uint64_t *key,
                                                size_t kstride, bool strict)
{
    uint32_t lo = 0, hi = d.n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const int c = row_cmp(d.gid, d.words, d.stride, d.W, mid, g, key, kstride);
        if (c < 0 || (!strict && c == 0))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Range probe q of p against the delta: a row of its group inside [lo, hi]
// committed after its snapshot (64-row LSN maxima between the ends).
__device__ __forceinline__ bool delta_hit(const DeltaView &d, const ProbeView &p, uint32_t q)
{
    const uint32_t g = p.gid[q];
    const uint32_t pa = delta_count(d, g, p.lo + q, p.n, true);
    const uint32_t pb = delta_count(d, g, p.hi + q, p.n, false);
    if (pa >= pb) return false;
    const uint64_t s = p.snap[q];
    bool hit = false;
    uint32_t i = pa;
    for (; i < pb && (i & 63) && !hit; ++i) hit = d.lsn[i] > s;  // to a block boundary
    for (; i + 64 <= pb && !hit; i += 64) hit = d.bmax[i >> 6] > s;
    for (; i < pb && !hit; ++i) hit = d.lsn[i] > s;
    return hit;
}

}  // namespace hsc
