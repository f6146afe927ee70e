// hsc_kernels.hip -- gfx950 kernels of the serializable conflict validator.
//
// The reference answers one read set at a time by re-walking the log window
// and scanning every read range of the written index linearly per write key
// (bdb/serializable.c:390-539 -> db/glue.c:2937-2961).  Here the window is
// resident and sorted once; a batch of read ranges becomes a range-max join:
//
//   locate  (one thread / range): splitter search in LDS -> first and last
//           window tile the range can touch; whole tiles strictly inside the
//           range are answered from the tile-max sparse table; the two end
//           tiles get a join record (FULL, or HEAD + TAIL).  Also table locks.
//   plan    (one workgroup): bucket offsets and work items per tile.
//   scatter (one thread / range): LDS-aggregated slot reservation, writes the
//           join records grouped by tile.
//   join    (one workgroup / tile chunk): stages the tile's keys + LSNs in LDS
//           (each window byte is read from HBM once per batch), binary-searches
//           every record's bounds in LDS and tests max LSN > snapshot.
//   pack    (ballot): per-read-set verdict bytes -> bitmap.
//
// Wave size is 64 everywhere (ballots are 64-bit).
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <utility>

namespace hsc {

// ============================================================================
// ingest: LSD radix sort of (gid, words) rows carrying lsn, stable
// ============================================================================
constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortThreads * kSortItems;  // rows per block

// Digit d (0 = least significant byte of the composite key).
__device__ __forceinline__ uint32_t row_digit(int W, int d, size_t i, const uint32_t *gid,
                                              const uint64_t *words, size_t stride)
{
    if (d < 8 * W) {
        int j = W - 1 - (d >> 3);
        return (uint32_t)(words[(size_t)j * stride + i] >> (8 * (d & 7))) & 0xFFu;
    }
    return (gid[i] >> (8 * (d - 8 * W))) & 0xFFu;
}

// Bits that vary across rows: OR over rows of (row XOR row 0), per key word
// and for the gid (mask[W]); a radix digit whose byte is zero in the mask is
// the same in every row and its pass is skipped.
__global__ __launch_bounds__(256) void k_vary_mask(int W, size_t n, const uint32_t *gid,
                                                   const uint64_t *words, size_t stride,
                                                   const uint64_t *lsn, unsigned long long *mask)
{
    constexpr int U = 8;  // independent loads in flight per thread
    __shared__ uint64_t part[256 / 64];
    for (int j = 0; j <= W; ++j) {
        const uint64_t ref = j < W ? words[(size_t)j * stride] : gid[0];
        uint64_t m = 0;
        for (size_t i0 = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n;
             i0 += (size_t)gridDim.x * blockDim.x * U) {
            uint64_t v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = i0 + (size_t)u * blockDim.x;
                v[u] = i >= n ? ref : j < W ? words[(size_t)j * stride + i] : gid[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) m |= v[u] ^ ref;
        }
        for (int o = 32; o > 0; o >>= 1) m |= __shfl_xor(m, o, 64);
        // one atomic per block and word: all blocks OR into the same W + 1
        // words, so per-wave atomics would queue behind each other
        if (lane_id() == 0) part[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t b = part[0] | part[1] | part[2] | part[3];
            if (b) atomicOr(&mask[j], (unsigned long long)b);
        }
        __syncthreads();
    }
    if (!lsn) return;
    // the rows' LSN span: mask[W + 1] = min, mask[W + 2] = max; mask[W + 3] =
    // the LSN bits that vary (OR of lsn XOR lsn[0])
    const uint64_t lref = lsn[0];
    uint64_t lo = ~0ull, hi = 0, lv = 0;
    for (size_t i0 = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n;
         i0 += (size_t)gridDim.x * blockDim.x * U) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + (size_t)u * blockDim.x;
            v[u] = i < n ? lsn[i] : lsn[i0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            lo = v[u] < lo ? v[u] : lo;
            hi = v[u] > hi ? v[u] : hi;
            lv |= v[u] ^ lref;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
        lv |= __shfl_xor(lv, o, 64);
    }
    __shared__ uint64_t plo[256 / 64], phi[256 / 64], plv[256 / 64];
    if (lane_id() == 0) plo[threadIdx.x >> 6] = lo, phi[threadIdx.x >> 6] = hi, plv[threadIdx.x >> 6] = lv;
    __syncthreads();
    if (threadIdx.x == 0) {  // one atomic pair per block (same-address atomics serialise)
        for (int w = 1; w < 256 / 64; ++w) {
            lo = plo[w] < lo ? plo[w] : lo;
            hi = phi[w] > hi ? phi[w] : hi;
            lv |= plv[w];
        }
        if (hi) {
            atomicMin(&mask[W + 1], (unsigned long long)lo);
            atomicMax(&mask[W + 2], (unsigned long long)hi);
        }
        if (lv) atomicOr(&mask[W + 3], (unsigned long long)lv);
    }
}

// The same masks and LSN span in ONE pass for keys of WT <= 4 words: every
// row's words, gid and LSN are loaded together (U rows per thread, all loads
// in flight before the first OR).  k_vary_mask above walks the rows once per
// word: 100 us for config 2's 280 MB (2.8 TB/s).
template <int WT, int U = 8>
__global__ __launch_bounds__(256) void k_vary_mask_w(size_t n, const uint32_t *gid, const uint64_t *words,
                                                     size_t stride, const uint64_t *lsn,
                                                     unsigned long long *mask)
{
    __shared__ uint64_t part[256 / 64][WT + 4];
    uint64_t ref[WT + 1], m[WT + 1];
#pragma unroll
    for (int j = 0; j < WT; ++j) ref[j] = words[(size_t)j * stride], m[j] = 0;
    ref[WT] = gid[0], m[WT] = 0;
    const uint64_t lref = lsn ? lsn[0] : 0;
    uint64_t lo = ~0ull, hi = 0, lv = 0;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += (size_t)gridDim.x * 256 * U) {
        uint64_t v[U][WT + 1], l[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + (size_t)u * 256;
            const bool ok = i < n;
#pragma unroll
            for (int j = 0; j < WT; ++j) v[u][j] = ok ? words[(size_t)j * stride + i] : ref[j];
            v[u][WT] = ok ? gid[i] : ref[WT];
            l[u] = lsn ? lsn[ok ? i : i0] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int j = 0; j <= WT; ++j) m[j] |= v[u][j] ^ ref[j];
            lo = l[u] < lo ? l[u] : lo;
            hi = l[u] > hi ? l[u] : hi;
            lv |= l[u] ^ lref;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int j = 0; j <= WT; ++j) m[j] |= __shfl_xor(m[j], o, 64);
        const uint64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
        lv |= __shfl_xor(lv, o, 64);
    }
    if (lane_id() == 0) {
#pragma unroll
        for (int j = 0; j <= WT; ++j) part[threadIdx.x >> 6][j] = m[j];
        part[threadIdx.x >> 6][WT + 1] = lo;
        part[threadIdx.x >> 6][WT + 2] = hi;
        part[threadIdx.x >> 6][WT + 3] = lv;
    }
    __syncthreads();
    if (threadIdx.x <= WT) {  // one atomic per block and word
        const int j = threadIdx.x;
        const uint64_t b = part[0][j] | part[1][j] | part[2][j] | part[3][j];
        if (b) atomicOr(&mask[j], (unsigned long long)b);
    } else if (threadIdx.x == 64 && lsn) {  // (another wave: the min / max pair)
        uint64_t a = part[0][WT + 1], b = part[0][WT + 2];
#pragma unroll
        for (int w = 1; w < 256 / 64; ++w) {
            a = part[w][WT + 1] < a ? part[w][WT + 1] : a;
            b = part[w][WT + 2] > b ? part[w][WT + 2] : b;
        }
        if (b) {
            atomicMin(&mask[WT + 1], (unsigned long long)a);
            atomicMax(&mask[WT + 2], (unsigned long long)b);
        }
    } else if (threadIdx.x == 128 && lsn) {  // (a third wave: the LSN's varying bits)
        const uint64_t v = part[0][WT + 3] | part[1][WT + 3] | part[2][WT + 3] | part[3][WT + 3];
        if (v) atomicOr(&mask[WT + 3], (unsigned long long)v);
    }
}

// Per-block digit counts, digit-major: counts[digit * nblocks + block].
__global__ __launch_bounds__(kSortThreads) void k_rs_count(int W, int d, size_t n,
                                                           const uint32_t *gid,
                                                           const uint64_t *words, size_t stride,
                                                           uint32_t *counts, uint32_t nblocks)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortTile;
    for (int k = 0; k < kSortItems; ++k) {
        size_t i = base + (size_t)k * kSortThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[row_digit(W, d, i, gid, words, stride)], 1u);
    }
    __syncthreads();
    counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter.  Phase 1: wave w ranks rows [1024 w, 1024 w + 1024) of the
// block in index order (16 rounds of 64 lanes; 8 ballots per round for the
// wave match) against wave-private digit counters in LDS, so the rounds need
// no block barrier; the per-wave counts then become per-(wave, digit) offsets
// and the block's sorted permutation is written to LDS.  Phase 2 walks the
// block in sorted order, so consecutive threads write consecutive addresses
// of each digit's run (coalesced stores); the rows it gathers were read by
// phase 1 and are served from L1/L2.
template <int WT>  // key words if 1..3 (phase 2 holds rows in registers), 0 = any
__global__ __launch_bounds__(kSortThreads) void k_rs_scatter(
    int Wrt, int d, size_t n, const uint32_t *gid, const uint64_t *words, const uint64_t *lsn,
    size_t stride, uint32_t *gid_o, uint64_t *words_o, uint64_t *lsn_o,
    const uint32_t *offsets, uint32_t nblocks)
{
    constexpr int kWaves = kSortThreads / 64;
    constexpr uint32_t kWaveRows = kSortTile / kWaves;
    const int W = WT > 0 ? WT : Wrt;
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t loff[256];
    __shared__ uint32_t wcnt[kWaves][256];
    __shared__ uint16_t perm[kSortTile];
    __shared__ uint32_t lds16[16];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const uint32_t dg = threadIdx.x;  // one digit per thread
    const size_t at = (size_t)dg * nblocks + blockIdx.x;
    const uint32_t mine = offsets[at];
    const size_t nxt_at = at + 1;
    const uint32_t total_rows = (uint32_t)n;
    // block's count of digit dg = next offset - this offset
    const uint32_t nxt = nxt_at < (size_t)256 * nblocks ? offsets[nxt_at] : total_rows;
    const uint32_t cnt = nxt - mine;
    gbase[dg] = mine;
    uint32_t tot;
    loff[dg] = block_excl_scan<kSortThreads>(cnt, lds16, tot);
#pragma unroll
    for (int w = 0; w < kWaves; ++w) wcnt[w][dg] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortTile;
    const uint64_t lt_mask = (lane ? (~0ull >> (64 - lane)) : 0ull);
    const uint32_t wbase = wid * kWaveRows;
    uint32_t *wc = wcnt[wid];
    uint32_t dig[kSortItems], lp[kSortItems];
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {  // every digit load in flight before the ranking
        const size_t i = base + wbase + k * 64 + lane;
        dig[k] = i < n ? row_digit(W, d, i, gid, words, stride) : 0;
    }
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const size_t i = base + wbase + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t dk = dig[k];
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((dk >> b) & 1u);
            peers &= ((dk >> b) & 1u) ? m : ~m;
        }
        const uint32_t before = wc[dk];
        lp[k] = before + __popcll(peers & lt_mask);
        dig[k] = valid ? dk : 0xFFFFFFFFu;
        // every lane has read the counter before the group's first lane bumps it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && (peers & lt_mask) == 0) wc[dk] = before + __popcll(peers);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    {  // per-(wave, digit) start inside the block's sorted order
        uint32_t acc = loff[dg];
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t t = wcnt[w][dg];
            wcnt[w][dg] = acc;
            acc += t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortItems; ++k)
        if (dig[k] != 0xFFFFFFFFu) perm[wc[dig[k]] + lp[k]] = (uint16_t)(wbase + k * 64 + lane);
    __syncthreads();
    // phase 2: sorted order -> contiguous runs per digit
    const uint32_t nrows = (uint32_t)min((size_t)kSortTile, n - base);
    if constexpr (WT == 0) {
        for (uint32_t j = threadIdx.x; j < nrows; j += kSortThreads) {
            const size_t i = base + perm[j];
            const uint32_t dj = row_digit(W, d, i, gid, words, stride);
            const uint32_t pos = gbase[dj] + (j - loff[dj]);
            gid_o[pos] = gid[i];
            for (int jw = 0; jw < W; ++jw) words_o[(size_t)jw * stride + pos] = words[(size_t)jw * stride + i];
            lsn_o[pos] = lsn[i];
        }
        return;
    } else {
    // kGather rows per thread at a time, all their loads before any store
    // (the row's digit is recomputed from the loaded words)
    constexpr int kGather = 4;
    for (uint32_t j0 = threadIdx.x; j0 < nrows; j0 += kGather * kSortThreads) {
        size_t ii[kGather];
        uint32_t gv[kGather];
        uint64_t lv[kGather], wv[kGather][WT];
#pragma unroll
        for (int u = 0; u < kGather; ++u) {
            const uint32_t j = j0 + u * kSortThreads;
            ii[u] = base + perm[j < nrows ? j : j0];
        }
#pragma unroll
        for (int u = 0; u < kGather; ++u) {
            gv[u] = gid[ii[u]];
            lv[u] = lsn[ii[u]];
#pragma unroll
            for (int jw = 0; jw < WT; ++jw)
                if (jw < W) wv[u][jw] = words[(size_t)jw * stride + ii[u]];
        }
#pragma unroll
        for (int u = 0; u < kGather; ++u) {
            const uint32_t j = j0 + u * kSortThreads;
            if (j >= nrows) break;
            uint32_t dj;
            if (d < 8 * W) {
                const int jw = W - 1 - (d >> 3);
                uint64_t x = 0;
#pragma unroll
                for (int q = 0; q < WT; ++q)
                    if (q == jw) x = wv[u][q];
                dj = (uint32_t)(x >> (8 * (d & 7))) & 0xFFu;
            } else {
                dj = (gv[u] >> (8 * (d - 8 * W))) & 0xFFu;
            }
            const uint32_t pos = gbase[dj] + (j - loff[dj]);
            gid_o[pos] = gv[u];
#pragma unroll
            for (int jw = 0; jw < WT; ++jw)
                if (jw < W) words_o[(size_t)jw * stride + pos] = wv[u][jw];
            lsn_o[pos] = lv[u];
        }
    }
    }
}

// ---- generic exclusive scan of u32 (in place), block sums recursively -----
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__global__ __launch_bounds__(kScanThreads) void k_scan_tile(uint32_t *a, size_t n, uint32_t *sums)
{
    __shared__ uint32_t lds[kScanThreads / 64];
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = (base + k < n) ? a[base + k] : 0;
        s += v[k];
    }
    uint32_t total;
    uint32_t pre = block_excl_scan<kScanThreads>(s, lds, total);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) a[base + k] = pre;
        pre += v[k];
    }
    if (threadIdx.x == 0 && sums) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_add(uint32_t *a, size_t n, const uint32_t *sums)
{
    const uint32_t add = sums[blockIdx.x];
    const size_t base = (size_t)blockIdx.x * kScanTile;
    for (int k = threadIdx.x; k < kScanTile; k += kScanThreads)
        if (base + k < n) a[base + k] += add;
}

size_t scan_scratch_bytes(size_t n)
{
    size_t total = 0;
    while (n > (size_t)kScanTile) {
        n = (n + kScanTile - 1) / kScanTile;
        total += n * sizeof(uint32_t);
    }
    return total + 256;
}

static hipError_t scan_u32(uint32_t *a, size_t n, uint32_t *scratch, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    size_t nb = (n + kScanTile - 1) / kScanTile;
    if (nb == 1) {
        k_scan_tile<<<1, kScanThreads, 0, s>>>(a, n, nullptr);
        return hipGetLastError();
    }
    uint32_t *sums = scratch;
    k_scan_tile<<<(unsigned)nb, kScanThreads, 0, s>>>(a, n, sums);
    hipError_t e = scan_u32(sums, nb, scratch + nb, s);
    if (e != hipSuccess) return e;
    k_scan_add<<<(unsigned)nb, kScanThreads, 0, s>>>(a, n, sums);
    return hipGetLastError();
}

hipError_t scan_exclusive_u32(uint32_t *a, size_t n, uint32_t *scratch, hipStream_t s)
{
    return scan_u32(a, n, scratch, s);
}

size_t radix_scratch_bytes(size_t n, int W)
{
    size_t nblocks = (n + kSortTile - 1) / kSortTile;
    size_t ndig = 8 * (size_t)W + 4;
    return ndig * 256 * sizeof(uint32_t) + 256 * nblocks * sizeof(uint32_t) +
           scan_scratch_bytes(256 * nblocks) + 1024;
}

hipError_t vary_mask_rows(int W, size_t n, const uint32_t *gid, const uint64_t *words, size_t stride,
                          void *scratch, uint64_t *vary, hipStream_t s, const uint64_t *lsn,
                          uint64_t *lsn_span, uint64_t *lsn_vary)
{
    for (int j = 0; j <= W; ++j) vary[j] = 0;
    if (lsn_span) lsn_span[0] = lsn_span[1] = 0;
    if (lsn_vary) *lsn_vary = 0;
    if (n == 0) return hipSuccess;
    unsigned long long *dmask = (unsigned long long *)scratch;  // [W + 1] masks, min, max, LSN vary
    hipError_t e = hipMemsetAsync(dmask, 0, 8 * ((size_t)W + 4), s);
    if (e == hipSuccess) e = hipMemsetAsync(dmask + W + 1, 0xFF, 8, s);
    if (e != hipSuccess) return e;
    const uint64_t *ls = lsn_span ? lsn : nullptr;
    // 512 workgroups of 8 rows x (W + 2) loads in flight per thread: all
    // workgroups OR into the same W + 3 words, one atomic each per word (2048
    // workgroups of 4 rows measured 109 us on config 2, the per-word kernel
    // 100 us)
    static const size_t vary_wg = getenv("HSC_VARY_WG") ? (size_t)atoi(getenv("HSC_VARY_WG")) : 512;  // (A/B)
    static const int vary_u = getenv("HSC_VARY_U") ? atoi(getenv("HSC_VARY_U")) : 8;  // rows per thread (A/B: 16)
    const unsigned wgrid = (unsigned)std::min<size_t>((n + 2047) / 2048, std::max<size_t>(vary_wg, 1));
    switch (W) {
    case 1: k_vary_mask_w<1><<<wgrid, 256, 0, s>>>(n, gid, words, stride, ls, dmask); break;
    case 2:
        if (vary_u == 16)
            k_vary_mask_w<2, 16><<<wgrid, 256, 0, s>>>(n, gid, words, stride, ls, dmask);
        else
            k_vary_mask_w<2><<<wgrid, 256, 0, s>>>(n, gid, words, stride, ls, dmask);
        break;
    case 3: k_vary_mask_w<3><<<wgrid, 256, 0, s>>>(n, gid, words, stride, ls, dmask); break;
    case 4: k_vary_mask_w<4><<<wgrid, 256, 0, s>>>(n, gid, words, stride, ls, dmask); break;
    default: {
        const unsigned hgrid = (unsigned)std::min<size_t>((n + 2047) / 2048, 512);
        k_vary_mask<<<hgrid, 256, 0, s>>>(W, n, gid, words, stride, ls, dmask);
    }
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    uint64_t hm[kMaxWords + 4];
    e = hipMemcpyAsync(hm, dmask, 8 * ((size_t)W + 4), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    for (int j = 0; j <= W; ++j) vary[j] = hm[j];
    if (lsn_span) {
        lsn_span[0] = hm[W + 2] ? hm[W + 1] : 0;
        lsn_span[1] = hm[W + 2];
        if (lsn_vary) *lsn_vary = hm[W + 3];
    }
    return hipSuccess;
}

hipError_t radix_sort_rows(int W, size_t n, uint32_t *gid, uint64_t *words, uint64_t *lsn,
                           size_t stride, uint32_t *gid_alt, uint64_t *words_alt,
                           uint64_t *lsn_alt, void *scratch, size_t scratch_bytes,
                           bool *result_in_alt, uint64_t *vary_mask, hipStream_t s)
{
    uint64_t hm[kMaxWords + 1];
    *result_in_alt = false;
    if (scratch_bytes < radix_scratch_bytes(n, W)) return hipErrorInvalidValue;
    hipError_t e = vary_mask_rows(W, n, gid, words, stride, scratch, hm, s);
    if (e != hipSuccess) return e;
    if (vary_mask)
        for (int j = 0; j <= W; ++j) vary_mask[j] = hm[j];
    return radix_sort_known(W, n, gid, words, lsn, stride, gid_alt, words_alt, lsn_alt, scratch,
                            scratch_bytes, result_in_alt, hm, s);
}

hipError_t radix_sort_known(int W, size_t n, uint32_t *gid, uint64_t *words, uint64_t *lsn,
                            size_t stride, uint32_t *gid_alt, uint64_t *words_alt,
                            uint64_t *lsn_alt, void *scratch, size_t scratch_bytes,
                            bool *result_in_alt, const uint64_t *hm, hipStream_t s)
{
    *result_in_alt = false;
    if (n <= 1) return hipSuccess;
    if (scratch_bytes < radix_scratch_bytes(n, W)) return hipErrorInvalidValue;
    const int ndig = 8 * W + 4;
    const uint32_t nblocks = (uint32_t)((n + kSortTile - 1) / kSortTile);
    uint32_t *counts = (uint32_t *)scratch + (size_t)ndig * 256;
    uint32_t *scan_tmp = counts + (size_t)256 * nblocks;
    hipError_t e = hipSuccess;
    bool alt = false;
    uint32_t *g0 = gid, *g1 = gid_alt;
    uint64_t *w0 = words, *w1 = words_alt, *l0 = lsn, *l1 = lsn_alt;
    for (int d = 0; d < ndig; ++d) {
        const int j = d < 8 * W ? W - 1 - (d >> 3) : W;
        const int byte = d < 8 * W ? (d & 7) : d - 8 * W;
        if (((hm[j] >> (8 * byte)) & 0xFFu) == 0) continue;  // digit constant across rows
        k_rs_count<<<nblocks, kSortThreads, 0, s>>>(W, d, n, g0, w0, stride, counts, nblocks);
        e = scan_u32(counts, (size_t)256 * nblocks, scan_tmp, s);
        if (e != hipSuccess) break;
#define HSC_RS(WT_) k_rs_scatter<WT_><<<nblocks, kSortThreads, 0, s>>>(W, d, n, g0, w0, l0, stride, \
                                                                   g1, w1, l1, counts, nblocks)
        if (W == 1)
            HSC_RS(1);
        else if (W == 2)
            HSC_RS(2);
        else if (W == 3)
            HSC_RS(3);
        else
            HSC_RS(0);
#undef HSC_RS
        e = hipGetLastError();
        if (e != hipSuccess) break;
        std::swap(g0, g1);
        std::swap(w0, w1);
        std::swap(l0, l1);
        alt = !alt;
    }
    *result_in_alt = alt;
    return e;
}

// ---- dedupe: keep the last row of every run of equal (gid, key) ----------
__global__ void k_flag_last(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                            size_t stride, uint32_t *flags)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t f = 1;
    if (i + 1 < n && gid[i] == gid[i + 1]) {
        f = 0;
        for (int j = 0; j < W; ++j)
            if (words[(size_t)j * stride + i] != words[(size_t)j * stride + i + 1]) {
                f = 1;
                break;
            }
    }
    flags[i] = f;
}

__global__ void k_compact(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                          const uint64_t *lsn, size_t stride_in, const uint32_t *pos,
                          const uint32_t *flags_last, uint32_t *gid_o, uint64_t *words_o,
                          uint64_t *lsn_o, size_t stride_out, uint32_t *d_count)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // flags were scanned in place into pos; recover "is last" from neighbours
    uint32_t p = pos[i];
    uint32_t nxt = (i + 1 < n) ? pos[i + 1] : flags_last[0] + p;
    if (nxt == p) return;
    gid_o[p] = gid[i];
    for (int j = 0; j < W; ++j) words_o[(size_t)j * stride_out + p] = words[(size_t)j * stride_in + i];
    lsn_o[p] = lsn[i];
    if (i + 1 == n) *d_count = p + 1;
}

__global__ void k_copy_last_flag(const uint32_t *flags, size_t n, uint32_t *out)
{
    out[0] = flags[n - 1];
}

hipError_t dedupe_flagged(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                          const uint64_t *lsn, size_t stride_in, uint32_t *gid_out,
                          uint64_t *words_out, uint64_t *lsn_out, size_t stride_out,
                          uint32_t *flags, void *scratch, size_t scratch_bytes,
                          uint32_t *d_count, hipStream_t s)
{
    if (n == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
    if (scratch_bytes < scan_scratch_bytes(n) + 16) return hipErrorInvalidValue;
    uint32_t *last = (uint32_t *)scratch;
    uint32_t *tmp = last + 4;
    const unsigned g = (unsigned)((n + 255) / 256);
    k_copy_last_flag<<<1, 1, 0, s>>>(flags, n, last);
    hipError_t e = scan_u32(flags, n, tmp, s);
    if (e != hipSuccess) return e;
    k_compact<<<g, 256, 0, s>>>(W, n, gid, words, lsn, stride_in, flags, last, gid_out, words_out,
                                lsn_out, stride_out, d_count);
    return hipGetLastError();
}

hipError_t dedupe_rows(int W, size_t n, const uint32_t *gid, const uint64_t *words,
                       const uint64_t *lsn, size_t stride_in, uint32_t *gid_out,
                       uint64_t *words_out, uint64_t *lsn_out, size_t stride_out,
                       uint32_t *flags, void *scratch, size_t scratch_bytes,
                       uint32_t *d_count, hipStream_t s)
{
    if (n) k_flag_last<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(W, n, gid, words, stride_in, flags);
    return dedupe_flagged(W, n, gid, words, lsn, stride_in, gid_out, words_out, lsn_out, stride_out,
                          flags, scratch, scratch_bytes, d_count, s);
}

// ---- summaries: group spans, tile maxima, sparse table, table maxima ------
// Rows are sorted by gid: group g's span is [#gid < g, #gid <= g), two binary
// searches per group (a group with no rows gets an empty span) instead of a
// pass over every row's gid.  gid == nullptr: one group holding every row.
__global__ void k_group_bounds(uint32_t n, const uint32_t *gid, int ngroups, uint32_t *gstart,
                               uint32_t *gend)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint32_t)ngroups) return;
    if (!gid) {
        gstart[g] = 0;
        gend[g] = n;
        return;
    }
    uint32_t lo = 0, hi = n;  // #gid < g
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gid[mid] < g) lo = mid + 1; else hi = mid;
    }
    const uint32_t a = lo;
    hi = n;  // #gid <= g
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gid[mid] <= g) lo = mid + 1; else hi = mid;
    }
    gstart[g] = a;
    gend[g] = lo;
}

__global__ __launch_bounds__(256) void k_tile_max(uint32_t n, int log2T, const uint64_t *lsn,
                                                  uint64_t *tmax0)
{
    __shared__ uint64_t part[4];
    const uint32_t t0 = blockIdx.x << log2T;
    const uint32_t t1 = min(n, t0 + (1u << log2T));
    uint64_t m = 0;
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += 256) m = lsn[i] > m ? lsn[i] : m;
    m = wave_max_u64(m);
    if (lane_id() == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t r = part[0];
        for (int k = 1; k < 4; ++k) r = part[k] > r ? part[k] : r;
        tmax0[blockIdx.x] = r;
    }
}

__global__ void k_sparse_level(uint32_t ntiles, int level, uint64_t *tmax)
{
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const uint64_t *prev = tmax + (size_t)(level - 1) * ntiles;
    uint32_t u = t + (1u << (level - 1));
    uint64_t a = prev[t], b = u < ntiles ? prev[u] : 0;
    tmax[(size_t)level * ntiles + t] = a > b ? a : b;
}

// Every level l >= 1 of the sparse table in one workgroup (windows of up to
// kSparseLdsTiles tiles): level l - 1 lives in LDS, each thread takes its
// pairs into registers, a barrier, then the level is written over it (and out).
// One launch instead of one ~4.6 us launch per level.
constexpr uint32_t kSparseLdsTiles = 8192;
constexpr int kSparseThreads = 1024;
__global__ __launch_bounds__(kSparseThreads) void k_sparse_all(uint32_t ntiles, int levels,
                                                               uint64_t *tmax)
{
    extern __shared__ uint64_t lv[];
    constexpr int R = kSparseLdsTiles / kSparseThreads;
    for (uint32_t t = threadIdx.x; t < ntiles; t += kSparseThreads) lv[t] = tmax[t];
    __syncthreads();
    for (int l = 1; l < levels; ++l) {
        const uint32_t h = 1u << (l - 1);
        uint64_t m[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = threadIdx.x + r * kSparseThreads;
            const uint64_t a = t < ntiles ? lv[t] : 0, b = t + h < ntiles ? lv[t + h] : 0;
            m[r] = a > b ? a : b;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = threadIdx.x + r * kSparseThreads;
            if (t < ntiles) {
                lv[t] = m[r];
                tmax[(size_t)l * ntiles + t] = m[r];
            }
        }
        __syncthreads();
    }
}

// Per-table max commit LSN over the key rows: one workgroup per group, whole
// tiles of its row span from the tile-max sparse table, the partial tiles at
// both ends scanned; one atomic per group (rows of a group are contiguous).
__global__ __launch_bounds__(256) void k_group_table_max(WinView w, const uint32_t *gstart,
                                                         const uint32_t *gend,
                                                         const uint32_t *group_table,
                                                         uint64_t *table_max)
{
    __shared__ uint64_t part[4];
    const uint32_t g = blockIdx.x;
    const uint32_t a = gstart[g], b = gend[g];
    if (a >= b) return;
    const uint32_t T = 1u << w.log2T;
    const uint32_t ta = (a + T - 1) >> w.log2T, tb = b >> w.log2T;  // whole tiles [ta, tb)
    uint64_t m = 0;
    if (ta < tb) {
        if (threadIdx.x == 0) m = tiles_max(w, ta, tb - 1);
        const uint32_t e0 = ta << w.log2T, s1 = tb << w.log2T;
        for (uint32_t i = a + threadIdx.x; i < e0; i += 256) m = w.lsn[i] > m ? w.lsn[i] : m;
        for (uint32_t i = s1 + threadIdx.x; i < b; i += 256) m = w.lsn[i] > m ? w.lsn[i] : m;
    } else {
        for (uint32_t i = a + threadIdx.x; i < b; i += 256) m = w.lsn[i] > m ? w.lsn[i] : m;
    }
    m = wave_max_u64(m);
    if (lane_id() == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t r = part[0];
        for (int k = 1; k < 4; ++k) r = part[k] > r ? part[k] : r;
        atomicMax((unsigned long long *)&table_max[group_table[g]], (unsigned long long)r);
    }
}

// Compact splitter arrays: first row of every tile.
__global__ void k_splitters(WinView w, uint32_t *sp_g, uint64_t *sp_w)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= w.ntiles) return;
    const size_t pos = (size_t)t << w.log2T;
    sp_g[t] = w.gid[pos];
    for (int j = 0; j < w.W; ++j) sp_w[(size_t)j * w.ntiles + t] = w.words[(size_t)j * w.stride + pos];
}

// Level l of a sparse table over tiles twice as long (shift 1) or as long
// (shift 0) as the source's, from the source's level l: entry t covers source
// tiles [t << shift, (t << shift) + 2^(l + shift)), i.e. one source entry or two
// (the second when it starts inside the source).
__global__ __launch_bounds__(256) void k_tmax_from(const uint64_t *src, uint32_t ns, int shift, uint64_t *dst,
                                                   uint32_t nt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y;
    if (t >= nt) return;
    const uint32_t a = t << shift;
    uint64_t m = src[(size_t)l * ns + a];
    if (shift) {
        const uint32_t b = a + (1u << l);
        if (b < ns) {
            const uint64_t y = src[(size_t)l * ns + b];
            m = y > m ? y : m;
        }
    }
    dst[(size_t)l * nt + t] = m;
}

hipError_t build_summaries(const WinView &w, uint32_t *gstart, uint32_t *gend, int ngroups,
                           uint64_t *tmax, const uint32_t *group_table, uint64_t *table_max,
                           uint32_t *sp_g, uint64_t *sp_w, hipStream_t s, const TmaxFrom &from)
{
    if (w.n == 0) {
        hipError_t e = hipMemsetAsync(gstart, 0, sizeof(uint32_t) * (size_t)ngroups, s);
        if (e == hipSuccess) e = hipMemsetAsync(gend, 0, sizeof(uint32_t) * (size_t)ngroups, s);
        return e;
    }
    if (ngroups > 0)
        k_group_bounds<<<(ngroups + 255) / 256, 256, 0, s>>>(w.n, ngroups == 1 ? nullptr : w.gid,
                                                             ngroups, gstart, gend);
    if (from.src && w.levels >= 1) {
        k_tmax_from<<<dim3((w.ntiles + 255) / 256, (unsigned)w.levels), 256, 0, s>>>(from.src, from.ntiles, from.shift,
                                                                                   tmax, w.ntiles);
    } else {
        if (from.lsn16 && w.log2T >= 4)
            k_tile_max<<<w.ntiles, 256, 0, s>>>((w.n + 15) / 16, w.log2T - 4, from.lsn16, tmax);
        else
            k_tile_max<<<w.ntiles, 256, 0, s>>>(w.n, w.log2T, w.lsn, tmax);
        if (w.levels > 1 && w.ntiles <= kSparseLdsTiles)
            k_sparse_all<<<1, kSparseThreads, 8 * (size_t)w.ntiles, s>>>(w.ntiles, w.levels, tmax);
        else
            for (int l = 1; l < w.levels; ++l)
                k_sparse_level<<<(w.ntiles + 255) / 256, 256, 0, s>>>(w.ntiles, l, tmax);
    }
    if (ngroups > 0 && table_max) {
        WinView wt = w;
        wt.tmax = tmax;
        k_group_table_max<<<ngroups, 256, 0, s>>>(wt, gstart, gend, group_table, table_max);
    }
    k_splitters<<<(w.ntiles + 255) / 256, 256, 0, s>>>(w, sp_g, sp_w);
    return hipGetLastError();
}

// ============================================================================
// probe
// ============================================================================
//
// Probes are split into G contiguous chunks; chunk g is handled by workgroup g
// of both k_locate and k_scatter.  k_locate counts the join records of its
// chunk per tile in LDS and stores the row hist[g][*]; k_colscan turns every
// column into chunk offsets inside the tile's bucket; k_plan scans the tile
// totals.  k_scatter then seeds its LDS counters with bucket_off[t] +
// hist[g][t], so every record slot comes from an LDS atomic: no global
// atomics, no contention across XCDs.

constexpr int kLocateBatch = 2;  // probes per thread advanced together

__global__ __launch_bounds__(kLocateThreads) void k_locate(WinView w, ProbeView p,
                                                           ProbeWork work, uint8_t *verdict,
                                                           uint32_t ntop, uint32_t stride_t)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *top = (uint64_t *)smem;              // [ntop] splitter prefixes
    uint32_t *hist = (uint32_t *)(top + ntop);     // [ntiles]
    // stage the splitters: loads in batches of 8 per thread before the stores
    for (uint32_t base = 0; base < ntop; base += 8 * kLocateThreads) {
        uint64_t vw[8];
        uint32_t vg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = base + k * kLocateThreads + threadIdx.x;
            if (i < ntop) {
                vw[k] = w.sp_w[(size_t)i * stride_t];
                vg[k] = w.sp_g[(size_t)i * stride_t];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = base + k * kLocateThreads + threadIdx.x;
            if (i < ntop) top[i] = key_prefix(w.gbits, vg[k], vw[k]);
        }
    }
    if (work.lds_mode)
        for (uint32_t i = threadIdx.x; i < w.ntiles; i += kLocateThreads) hist[i] = 0;
    __syncthreads();

    const size_t ks = p.n;
    const uint32_t c0 = blockIdx.x * work.chunk;
    const uint32_t c1 = min(p.n, c0 + work.chunk);
    for (uint32_t base = c0; base < c1; base += kLocateBatch * kLocateThreads) {
        constexpr int NS = 2 * kLocateBatch;
        uint32_t qq[kLocateBatch];
        bool valid[kLocateBatch];
        uint32_t gg[NS];
        uint64_t k0[NS];
        const uint64_t *km[NS];
        bool leq[NS];
        uint32_t cnt[NS];
#pragma unroll
        for (int b = 0; b < kLocateBatch; ++b) {
            qq[b] = base + b * kLocateThreads + threadIdx.x;
            valid[b] = qq[b] < c1;
            const uint32_t q = valid[b] ? qq[b] : c0;
            const uint32_t g = p.gid[q];
            gg[2 * b] = gg[2 * b + 1] = g;
            k0[2 * b] = p.lo[q];
            k0[2 * b + 1] = p.hi[q];
            km[2 * b] = p.lo + q;
            km[2 * b + 1] = p.hi + q;
            leq[2 * b] = false;
            leq[2 * b + 1] = true;
        }
        count_splitters<NS>(w, top, ntop, stride_t, gg, k0, km, ks, leq, cnt);
        // middle tiles of split ranges: sparse-table maxima and snapshots are
        // loaded for every probe of the batch before any is used
        uint64_t mid[kLocateBatch], sn[kLocateBatch];
#pragma unroll
        for (int b = 0; b < kLocateBatch; ++b) {
            const uint32_t c = cnt[2 * b], c2 = cnt[2 * b + 1];
            const uint32_t a = c ? c - 1 : 0, bt = c2 ? c2 - 1 : 0;
            const bool need = valid[b] && c2 > 0 && bt > a + 1;
            mid[b] = tiles_max(w, need ? a + 1 : 0, need ? bt - 1 : 0);
            sn[b] = p.snap[valid[b] ? qq[b] : c0];
            if (!need) mid[b] = 0;
        }
#pragma unroll
        for (int b = 0; b < kLocateBatch; ++b) {
            if (!valid[b]) continue;
            const uint32_t q = qq[b];
            const uint32_t c = cnt[2 * b], c2 = cnt[2 * b + 1];
            uint64_t cd = 0;
            if (c2 > 0) {
                const uint32_t a = c ? c - 1 : 0, bt = c2 - 1;
                if (a == bt) {
                    cd = (uint64_t)a | ((uint64_t)a << 31) | (kKindFull << 62);
                } else if (a < bt) {
                    if (mid[b] > sn[b])
                        verdict[p.txn[q]] = 1;
                    else
                        cd = (uint64_t)a | ((uint64_t)bt << 31) | (kKindSplit << 62);
                }
            }
            work.code[q] = cd;
            if (cd) {
                const uint32_t a = (uint32_t)(cd & 0x7FFFFFFFu);
                const uint32_t bt = (uint32_t)((cd >> 31) & 0x7FFFFFFFu);
                if (work.lds_mode) {
                    atomicAdd(&hist[a], 1u);
                    if (bt != a) atomicAdd(&hist[bt], 1u);
                } else {
                    atomicAdd(&work.counts[a], 1u);
                    if (bt != a) atomicAdd(&work.counts[bt], 1u);
                }
            }
        }
    }
    // table locks: any write to a locked table after the snapshot
    for (uint32_t q = blockIdx.x * kLocateThreads + threadIdx.x; q < p.n_lock;
         q += gridDim.x * kLocateThreads) {
        const uint32_t t = p.lock_table[q];
        if (t < w.ntables && w.table_max[t] > p.lock_snap[q]) verdict[p.lock_txn[q]] = 1;
    }
    if (work.lds_mode) {
        __syncthreads();
        uint32_t *row = work.hist + (size_t)blockIdx.x * w.ntiles;
        for (uint32_t i = threadIdx.x; i < w.ntiles; i += kLocateThreads) row[i] = hist[i];
    }
}

hipError_t launch_locate(const WinView &w, const ProbeView &p, const ProbeWork &work,
                         uint8_t *verdict, hipStream_t s)
{
    if (p.n == 0 && p.n_lock == 0) return hipSuccess;
    uint32_t ntop = 0, stride_t = 1;
    if (w.n) {
        stride_t = (w.ntiles + kTopCap - 1) / kTopCap;
        ntop = (w.ntiles + stride_t - 1) / stride_t;
    }
    size_t lds = (size_t)ntop * 8 + (work.lds_mode ? (size_t)w.ntiles * 4 : 0);
    k_locate<<<work.G, kLocateThreads, lds, s>>>(w, p, work, verdict, ntop, stride_t);
    return hipGetLastError();
}

// ---- plan ------------------------------------------------------------------
// Column scan of hist[G][ntiles]: hist[g][t] := sum over g' < g; counts[t] :=
// total.  A workgroup owns 16 tiles (16 lanes read 64 contiguous bytes of a
// row) and splits the G rows into 64 segments (4 per wave); each thread holds
// its segment's values in registers, so the scan is one pass with every load
// in flight.  ceil(ntiles / 16) workgroups keep every CU busy.
constexpr int kColTiles = 16, kColSegs = 64;
constexpr int kColSegRows = kMaxChunks / kColSegs;
__global__ __launch_bounds__(1024) void k_colscan(ProbeWork work, uint32_t ntiles)
{
    __shared__ uint32_t segtot[kColSegs][kColTiles];
    const int col = threadIdx.x % kColTiles, seg = threadIdx.x / kColTiles;
    const uint32_t t = blockIdx.x * kColTiles + col;
    const uint32_t per = (work.G + kColSegs - 1) / kColSegs;
    const uint32_t g0 = seg * per;
    uint32_t v[kColSegRows];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kColSegRows; ++k) {
        const uint32_t g = g0 + k;
        v[k] = (k < (int)per && g < work.G && t < ntiles) ? work.hist[(size_t)g * ntiles + t] : 0;
        sum += v[k];
    }
    segtot[seg][col] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int j = 0; j < seg; ++j) run += segtot[j][col];
    if (t < ntiles) {
#pragma unroll
        for (int k = 0; k < kColSegRows; ++k) {
            const uint32_t g = g0 + k;
            if (k < (int)per && g < work.G) work.hist[(size_t)g * ntiles + t] = run;
            run += v[k];
        }
        if (seg == kColSegs - 1) work.counts[t] = run;
    }
}

// One workgroup: bucket offsets, per-tile chunk counts, item -> tile table.
// Each thread owns 8 consecutive tiles per 8192-tile round.
__global__ __launch_bounds__(1024) void k_plan(ProbeWork work, uint32_t ntiles)
{
    __shared__ uint32_t lds[16];
    uint32_t carry_b = 0, carry_i = 0;
    for (uint32_t base = 0; base < ntiles; base += 8 * 1024) {
        const uint32_t t0 = base + 8 * threadIdx.x;
        uint32_t cv[8], ch[8], sb = 0, si = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) cv[k] = t0 + k < ntiles ? work.counts[t0 + k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            ch[k] = (cv[k] + kJoinChunk - 1) / kJoinChunk;
            sb += cv[k];
            si += ch[k];
        }
        uint32_t tb, ti;
        uint32_t pb = block_excl_scan<1024>(sb, lds, tb);
        uint32_t pi = block_excl_scan<1024>(si, lds, ti);
        pb += carry_b;
        pi += carry_i;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t t = t0 + k;
            if (t < ntiles) {
                work.bucket_off[t] = pb;
                work.cursor[t] = pb;
                work.item_off[t] = pi;
                for (uint32_t j = 0; j < ch[k]; ++j) {
                    work.item_tile[pi + j] = t;
                    const uint32_t r0 = pb + j * kJoinChunk;
                    work.item_desc[pi + j] = make_uint4(t, r0, min(r0 + kJoinChunk, pb + cv[k]), 0);
                }
            }
            pb += cv[k];
            pi += ch[k];
        }
        carry_b += tb;
        carry_i += ti;
    }
    if (threadIdx.x == 0) {
        work.bucket_off[ntiles] = carry_b;
        work.item_off[ntiles] = carry_i;
    }
}

hipError_t launch_plan(const WinView &w, const ProbeWork &work, hipStream_t s)
{
    if (work.lds_mode) k_colscan<<<(w.ntiles + kColTiles - 1) / kColTiles, 1024, 0, s>>>(work, w.ntiles);
    k_plan<<<1, 1024, 0, s>>>(work, w.ntiles);
    return hipGetLastError();
}

// ---- scatter: join records grouped by tile ---------------------------------
// One join record = rec_words(W) u64: lo[W] hi[W] snap meta, with
// meta = txn | lb << 32 | ub << 45 | kind << 62, [lb, ub) = the rows of the
// probe's group inside the tile (so the join needs no group lookup).
__device__ __forceinline__ void write_record(const WinView &w, uint64_t *recs, uint32_t slot,
                                             const ProbeView &p, uint32_t q, uint32_t tile,
                                             uint64_t kind)
{
    const int W = w.W, rw = rec_words(W);
    const uint32_t T = 1u << w.log2T;
    const uint32_t ts = tile << w.log2T;
    const uint32_t tn = min(T, w.n - ts);
    const uint32_t g = p.gid[q];
    const uint32_t gs = w.gstart[g], ge = w.gend[g];
    const uint64_t lb = gs > ts ? min(gs - ts, tn) : 0;
    const uint64_t ub = ge > ts ? min(ge - ts, tn) : 0;
    const uint64_t meta = (uint64_t)p.txn[q] | (lb << 32) | (ub << 45) | (kind << 62);
    ulonglong2 *r = (ulonglong2 *)(recs + (size_t)slot * rec_stride(W));
    const size_t ks = p.n;
    auto word = [&](int k) -> uint64_t {
        if (k < W) return p.lo[(size_t)k * ks + q];
        if (k < 2 * W) return p.hi[(size_t)(k - W) * ks + q];
        if (k == 2 * W) return p.snap[q];
        return meta;
    };
    for (int k = 0; k < rw; k += 2) r[k >> 1] = make_ulonglong2(word(k), word(k + 1));
}

// Seed the LDS slot counters of chunk blockIdx.x: bucket_off[t] + hist[g][t].
__device__ __forceinline__ void seed_slots(const WinView &w, const ProbeWork &work,
                                           uint32_t *base_t)
{
    const uint32_t *row = work.hist + (size_t)blockIdx.x * w.ntiles;
    for (uint32_t b = 0; b < w.ntiles; b += 8 * kLocateThreads) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = b + k * kLocateThreads + threadIdx.x;
            v[k] = i < w.ntiles ? work.bucket_off[i] + row[i] : 0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t i = b + k * kLocateThreads + threadIdx.x;
            if (i < w.ntiles) base_t[i] = v[k];
        }
    }
    __syncthreads();
}

// Generic key width: one record at a time.
__global__ __launch_bounds__(kLocateThreads) void k_scatter_any(WinView w, ProbeView p,
                                                                ProbeWork work)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *base_t = (uint32_t *)smem;  // [ntiles] next free slot of this chunk
    if (work.lds_mode) seed_slots(w, work, base_t);
    const uint32_t c0 = blockIdx.x * work.chunk;
    const uint32_t c1 = min(p.n, c0 + work.chunk);
    for (uint32_t q = c0 + threadIdx.x; q < c1; q += kLocateThreads) {
        const uint64_t cd = work.code[q];
        if (!cd) continue;
        const uint32_t a = (uint32_t)(cd & 0x7FFFFFFFu);
        const uint32_t b = (uint32_t)((cd >> 31) & 0x7FFFFFFFu);
        const bool full = (cd >> 62) == kKindFull;
        const uint32_t sa = work.lds_mode ? atomicAdd(&base_t[a], 1u) : atomicAdd(&work.cursor[a], 1u);
        write_record(w, work.recs, sa, p, q, a, full ? kRecFull : kRecHead);
        if (!full) {
            const uint32_t sb = work.lds_mode ? atomicAdd(&base_t[b], 1u) : atomicAdd(&work.cursor[b], 1u);
            write_record(w, work.recs, sb, p, q, b, kRecTail);
        }
    }
}

// W <= 3: every global load of a batch of kScatB probes is issued before the
// first dependent use (probe words, then group bounds), then the LDS slot
// atomics, then the 16-byte record stores.
constexpr int kScatB = 4;
template <int WT>
__global__ __launch_bounds__(kLocateThreads) void k_scatter(WinView w, ProbeView p,
                                                            ProbeWork work)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *base_t = (uint32_t *)smem;
    if (work.lds_mode) seed_slots(w, work, base_t);
    const uint32_t c0 = blockIdx.x * work.chunk;
    const uint32_t c1 = min(p.n, c0 + work.chunk);
    const size_t ks = p.n;
    const uint32_t T = 1u << w.log2T;
    constexpr int rs = HSC_REC_PAD ? 8 : 2 * WT + 2;
    for (uint32_t base = c0; base < c1; base += kScatB * kLocateThreads) {
        constexpr int WA = WT > 2 ? WT : 2;
        uint64_t cd[kScatB], lo[kScatB][WA], hi[kScatB][WA], snap[kScatB];
        uint32_t g[kScatB], txn[kScatB], gs[kScatB], ge[kScatB];
#pragma unroll
        for (int k = 0; k < kScatB; ++k) {
            const uint32_t q0 = base + k * kLocateThreads + threadIdx.x;
            const uint32_t q = q0 < c1 ? q0 : c0;
            cd[k] = q0 < c1 ? work.code[q] : 0;
            g[k] = p.gid[q];
            txn[k] = p.txn[q];
            snap[k] = p.snap[q];
#pragma unroll
            for (int j = 0; j < WT; ++j) {
                lo[k][j] = p.lo[(size_t)j * ks + q];
                hi[k][j] = p.hi[(size_t)j * ks + q];
            }
        }
#pragma unroll
        for (int k = 0; k < kScatB; ++k) {
            gs[k] = w.gstart[g[k]];
            ge[k] = w.gend[g[k]];
        }
        uint32_t slot[kScatB][2];
#pragma unroll
        for (int k = 0; k < kScatB; ++k) {
            slot[k][0] = slot[k][1] = 0;
            if (!cd[k]) continue;
            const uint32_t a = (uint32_t)(cd[k] & 0x7FFFFFFFu);
            const uint32_t b = (uint32_t)((cd[k] >> 31) & 0x7FFFFFFFu);
            slot[k][0] = work.lds_mode ? atomicAdd(&base_t[a], 1u) : atomicAdd(&work.cursor[a], 1u);
            if ((cd[k] >> 62) != kKindFull)
                slot[k][1] = work.lds_mode ? atomicAdd(&base_t[b], 1u) : atomicAdd(&work.cursor[b], 1u);
        }
#pragma unroll
        for (int k = 0; k < kScatB; ++k) {
            if (!cd[k]) continue;
            const bool full = (cd[k] >> 62) == kKindFull;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && full) break;
                const uint32_t tile = h == 0 ? (uint32_t)(cd[k] & 0x7FFFFFFFu)
                                             : (uint32_t)((cd[k] >> 31) & 0x7FFFFFFFu);
                const uint64_t kind = full ? kRecFull : (h == 0 ? kRecHead : kRecTail);
                const uint32_t ts = tile << w.log2T;
                const uint32_t tn = min(T, w.n - ts);
                const uint64_t lb = gs[k] > ts ? min(gs[k] - ts, tn) : 0;
                const uint64_t ub = ge[k] > ts ? min(ge[k] - ts, tn) : 0;
                const uint64_t meta = (uint64_t)txn[k] | (lb << 32) | (ub << 45) | (kind << 62);
                ulonglong2 *r = (ulonglong2 *)(work.recs + (size_t)slot[k][h] * rs);
                uint64_t rv[2 * WT + 2];  // lo[WT] hi[WT] snap meta
#pragma unroll
                for (int j = 0; j < WT; ++j) {
                    rv[j] = lo[k][j];
                    rv[WT + j] = hi[k][j];
                }
                rv[2 * WT] = snap[k];
                rv[2 * WT + 1] = meta;
#pragma unroll
                for (int i = 0; i <= WT; ++i) r[i] = make_ulonglong2(rv[2 * i], rv[2 * i + 1]);
            }
        }
    }
}

hipError_t launch_scatter(const WinView &w, const ProbeView &p, const ProbeWork &work,
                          hipStream_t s)
{
    if (p.n == 0) return hipSuccess;
    size_t lds = work.lds_mode ? (size_t)w.ntiles * 4 : 16;
    if (w.W == 1)
        k_scatter<1><<<work.G, kLocateThreads, lds, s>>>(w, p, work);
    else if (w.W == 2)
        k_scatter<2><<<work.G, kLocateThreads, lds, s>>>(w, p, work);
    else if (w.W == 3)
        k_scatter<3><<<work.G, kLocateThreads, lds, s>>>(w, p, work);
    else
        k_scatter_any<<<work.G, kLocateThreads, lds, s>>>(w, p, work);
    return hipGetLastError();
}

// ---- join: one workgroup per (tile, chunk of records) ----------------------
// Key compare of a probe key (words 0,1 in registers, later words at
// kmem[j]) with tile row `row` (LDS, word j at kw[j * T + row]):
// sign(key - row).
__device__ __forceinline__ int cmp_row(int W, const uint64_t *kw, uint32_t T, uint32_t row,
                                       uint64_t k0, uint64_t k1, const uint64_t *kmem)
{
    const uint64_t r0 = kw[row];
    if (k0 != r0) return k0 < r0 ? -1 : 1;
    if (W == 1) return 0;
    const uint64_t r1 = kw[T + row];
    if (k1 != r1) return k1 < r1 ? -1 : 1;
    for (int j = 2; j < W; ++j) {
        const uint64_t a = kmem[j], b = kw[(size_t)j * T + row];
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// Word 0 of the row in LDS, later words (only on a tie of word 0) from the
// window in global memory.  Used for compact codes, whose first word holds
// the group's 64 most significant varying bits, so ties are rare.
__device__ __forceinline__ int cmp_row_w0(int W, const uint64_t *kw, const WinView &w, uint32_t ts,
                                          uint32_t row, uint64_t k0, uint64_t k1,
                                          const uint64_t *kmem)
{
    const uint64_t r0 = kw[row];
    if (k0 != r0) return k0 < r0 ? -1 : 1;
    for (int j = 1; j < W; ++j) {
        const uint64_t a = j == 1 ? k1 : kmem[j], b = w.words[(size_t)j * w.stride + ts + row];
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// WT: key words if 1..3 (fast staging path, tiles of 2^LOG2T rows), 0 = any.
// W0: stage only key word 0 (and the LSNs) of the tile.
template <int WT, int LOG2T, bool W0 = false>
__global__ __launch_bounds__(kJoinThreads) void k_join(WinView w, ProbeWork work,
                                                       uint8_t *verdict)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t item = blockIdx.x;
    if (item >= work.item_off[w.ntiles]) return;
    const uint32_t tile = work.item_tile[item];
    const uint32_t rb = work.bucket_off[tile] + (item - work.item_off[tile]) * kJoinChunk;
    const uint32_t re = min(rb + (uint32_t)kJoinChunk, work.bucket_off[tile + 1]);
    const int W = WT > 0 ? WT : w.W;
    const int rw = rec_stride(W);
    const uint32_t T = 1u << w.log2T;
    const uint32_t ts = tile << w.log2T;

    constexpr int WS = W0 ? 1 : WT;                // key words staged (WT > 0)
    uint64_t *kw = (uint64_t *)smem;               // [W][T] (W0: [1][T])
    uint64_t *lsn = kw + (size_t)(W0 ? 1 : W) * T; // [T]
    uint64_t *b16 = lsn + T;                       // [T / 16]
    uint64_t *b256 = b16 + T / 16;                 // [T / 256]

    // records of this thread (kJoinChunk / kJoinThreads of them), fetched
    // before the tile so their latency overlaps the staging
    constexpr int kRec = kJoinChunk / kJoinThreads;
    ulonglong2 tail[kRec];
    ulonglong2 bnd[kRec][2];
#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t r = rb + k * kJoinThreads + threadIdx.x;
        if (r < re) {
            const uint64_t *rec = work.recs + (size_t)r * rw;
            tail[k] = *(const ulonglong2 *)(rec + 2 * W);
            if constexpr (WT == 2) {
                bnd[k][0] = *(const ulonglong2 *)rec;
                bnd[k][1] = *(const ulonglong2 *)(rec + 2);
            } else if constexpr (WT >= 3) {  // words 0, 1 of lo and hi; later words from rec
                bnd[k][0] = *(const ulonglong2 *)rec;
                bnd[k][1] = make_ulonglong2(rec[W], rec[W + 1]);
            } else if constexpr (WT == 1) {
                bnd[k][0] = *(const ulonglong2 *)rec;  // lo0, hi0
            }
        }
    }

    // stage the tile: every thread issues all of its 16-byte loads first and
    // only then writes LDS, so its loads are in flight together.  The window
    // arrays are padded to a whole number of tiles, so the loads need no
    // bounds checks (rows >= tn are never searched).
    if constexpr (WT > 0) {
        constexpr int kIt = (1 << LOG2T) / (2 * kJoinThreads);
        ulonglong2 v[kIt][WS + 1];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const uint32_t pr = threadIdx.x + it * kJoinThreads;
#pragma unroll
            for (int j = 0; j < WS; ++j)
                v[it][j] = *(const ulonglong2 *)(w.words + (size_t)j * w.stride + ts + 2 * pr);
            v[it][WS] = *(const ulonglong2 *)(w.lsn + ts + 2 * pr);
        }
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const uint32_t pr = threadIdx.x + it * kJoinThreads;
#pragma unroll
            for (int j = 0; j < WS; ++j) *(ulonglong2 *)(kw + (size_t)j * T + 2 * pr) = v[it][j];
            *(ulonglong2 *)(lsn + 2 * pr) = v[it][WS];
        }
    } else {
        for (int j = 0; j <= W; ++j) {
            const uint64_t *src = j < W ? w.words + (size_t)j * w.stride + ts : w.lsn + ts;
            uint64_t *dst = j < W ? kw + (size_t)j * T : lsn;
            for (uint32_t pr = threadIdx.x; pr < T / 2; pr += kJoinThreads)
                *(ulonglong2 *)(dst + 2 * pr) = *(const ulonglong2 *)(src + 2 * pr);
        }
    }
    __syncthreads();
    // block maxima: 16-row blocks, then 256-row blocks
    if (threadIdx.x < T / 16) {
        const ulonglong2 *src = (const ulonglong2 *)(lsn + 16 * threadIdx.x);
        uint64_t m = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const ulonglong2 v = src[k];
            m = v.x > m ? v.x : m;
            m = v.y > m ? v.y : m;
        }
        b16[threadIdx.x] = m;
    }
    __syncthreads();
    if (threadIdx.x < T / 256) {
        uint64_t m = 0;
        for (int k = 0; k < 16; ++k) m = b16[16 * threadIdx.x + k] > m ? b16[16 * threadIdx.x + k] : m;
        b256[threadIdx.x] = m;
    }
    __syncthreads();

#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t r = rb + k * kJoinThreads + threadIdx.x;
        if (r >= re) continue;
        const uint64_t *rec = work.recs + (size_t)r * rw;
        const uint64_t snap = tail[k].x, meta = tail[k].y;
        const uint32_t txn = (uint32_t)meta;
        const uint32_t lb = (uint32_t)(meta >> 32) & 0x1FFFu;
        const uint32_t ub = (uint32_t)(meta >> 45) & 0x1FFFu;
        const uint32_t kind = (uint32_t)(meta >> 62);
        if (lb >= ub) continue;
        uint64_t l0, l1, h0, h1;
        if constexpr (WT >= 2) {
            l0 = bnd[k][0].x;
            l1 = bnd[k][0].y;
            h0 = bnd[k][1].x;
            h1 = bnd[k][1].y;
        } else if constexpr (WT == 1) {
            l0 = bnd[k][0].x;
            h0 = bnd[k][0].y;
            l1 = h1 = 0;
        } else {
            l0 = rec[0];
            l1 = W > 1 ? rec[1] : 0;
            h0 = rec[W];
            h1 = W > 1 ? rec[W + 1] : 0;
        }
        // lower bound of lo and upper bound of hi in [lb, ub), in lockstep
        uint32_t alo = lb, ahi = kind == kRecTail ? lb : ub;
        uint32_t blo = kind == kRecHead ? ub : lb, bhi = ub;
        while (alo < ahi || blo < bhi) {
            const uint32_t am = (alo + ahi) >> 1, bm = (blo + bhi) >> 1;
            if (alo < ahi) {
                const int c = W0 ? cmp_row_w0(W, kw, w, ts, am, l0, l1, rec)
                                 : cmp_row(W, kw, T, am, l0, l1, rec);
                if (c > 0) alo = am + 1; else ahi = am;
            }
            if (blo < bhi) {
                const int c = W0 ? cmp_row_w0(W, kw, w, ts, bm, h0, h1, rec + W)
                                 : cmp_row(W, kw, T, bm, h0, h1, rec + W);
                if (c >= 0) blo = bm + 1; else bhi = bm;
            }
        }
        const uint32_t pp = alo, qq = blo;
        if (pp >= qq) continue;
        const bool hit = WT > 0 ? lds_any_after<(1 << LOG2T) / 256>(lsn, b16, b256, pp, qq, snap)
                                : lds_any_after<16>(lsn, b16, b256, pp, qq, snap);
        if (hit) verdict[txn] = 1;
    }
}

hipError_t launch_join(const WinView &w, const ProbeWork &work, uint32_t max_items,
                       uint8_t *verdict, hipStream_t s)
{
    if (max_items == 0 || w.n == 0) return hipSuccess;
    const size_t T = (size_t)1 << w.log2T;
    // compact 3-word codes: only word 0 staged, later words read on a tie
    const bool w0 = w.W == 3 && w.log2T == 11 && w.compact;
    const size_t lds = T * 8 * (size_t)(w0 ? 1 : w.W) + T * 8 + (T / 16) * 8 +
                       std::max<size_t>(T / 256, 16) * 8;
    if (w.W == 1 && w.log2T == 12)
        k_join<1, 12><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    else if (w.W == 1 && w.log2T == 11)
        k_join<1, 11><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    else if (w.W == 2 && w.log2T == 11)
        k_join<2, 11><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    else if (w0)
        k_join<3, 11, true><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    else if (w.W == 3 && w.log2T == 11)
        k_join<3, 11><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    else
        k_join<0, 0><<<max_items, kJoinThreads, lds, s>>>(w, work, verdict);
    return hipGetLastError();
}

// ---- pack: verdict bytes -> bitmap ----------------------------------------
__global__ void k_pack(const uint8_t *verdict, uint32_t n, uint64_t *bitmap)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool v = t < n && verdict[t] != 0;
    const uint64_t m = __ballot(v);
    if (lane_id() == 0 && t < n) bitmap[t >> 6] = m;
}

hipError_t launch_pack(const uint8_t *verdict, uint32_t n_txn, uint64_t *bitmap, hipStream_t s)
{
    if (n_txn == 0 || bitmap == nullptr) return hipSuccess;
    k_pack<<<(n_txn + 255) / 256, 256, 0, s>>>(verdict, n_txn, bitmap);
    return hipGetLastError();
}

// ---- OR of per-shard verdict bitmaps (after an all-gather) -----------------
__global__ void k_or_bitmaps(const uint64_t *parts, int nparts, size_t words, uint64_t *out)
{
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint64_t m = 0;
    for (int k = 0; k < nparts; ++k) m |= parts[(size_t)k * words + w];
    out[w] = m;
}

hipError_t launch_or_bitmaps(const uint64_t *parts, int nparts, size_t words, uint64_t *out,
                             hipStream_t s)
{
    if (words == 0) return hipSuccess;
    k_or_bitmaps<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(parts, nparts, words, out);
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_kernels()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_compact);
}

}  // namespace hsc
