// hsc_csort.hip -- sort of wide window rows by their compact codes (gfx950).
//
// A window whose key bits that vary do not fit the packed 64-bit sort of
// hsc_ingest.hip (config 3: 189 varying bits over 8-word keys) used to take
// the whole-row LSD radix sort: one pass per varying key byte (23 for config
// 3), each moving gid + 8 words + LSN = 76 bytes per row -- 10.5 ms of the
// 11.4 ms build.  Its rows sort instead by their compact codes
// (hsc_compact.hip: a group's varying bits, memcmp order kept): each row
// becomes one key of KW = WC + 1 words
//     gid (32 bits) || code (64 WC bits) || row index (32 bits),
// unique (the index breaks ties, so the sort is stable by construction and
// the last version of a key is the last of its run), sorted here by
//   block sort   1024 keys per workgroup: 4-key networks in registers, then
//                merge levels in LDS;
//   merges       runs of 1024, 2048, ... merged pairwise by merge path: the
//                splits of every 1024-output tile first (k_cs_splits, all
//                tiles at once), then a workgroup per tile stages its keys
//                of the two runs in LDS, and
//                every thread merges 4 outputs from its own split into an
//                LDS permutation that the tile then writes out in order,
// i.e. log2(n / 1024) passes of 2 x 8 KW bytes per row, then unpacked back
// to rows (hsc_compact.hip compact_unpack: words = pattern | expanded code,
// the LSN gathered by index).
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace hsc {
namespace {

constexpr int kCsThreads = 256;
constexpr int kCsBlock = 1024;                  // keys per block sort / merge tile
constexpr int kCsPer = kCsBlock / kCsThreads;  // outputs per thread

template <int KW>
__device__ __forceinline__ bool key_lt(const uint64_t *a, const uint64_t *b)
{
#pragma unroll
    for (int k = 0; k < KW; ++k)
        if (a[k] != b[k]) return a[k] < b[k];
    return false;
}

// Sort keys [b * 1024, b * 1024 + 1024) of src into dst (the tail block
// padded with all-ones keys, which sort last and are not stored): every
// thread sorts its 4 consecutive keys in registers, then 8 merge levels in
// LDS (runs of 4, 8, ... 512 merged pairwise; each thread finds its 4
// outputs' split of its pair by a binary search and merges them) -- 16
// barriers instead of a bitonic network's 55.  LDS holds the keys word-major
// (K[k][i]): lanes reading consecutive keys read consecutive words.
template <int KW>
__device__ __forceinline__ bool lds_lt(const uint64_t (*K)[kCsBlock], uint32_t i, uint32_t j)
{
#pragma unroll
    for (int k = 0; k < KW; ++k)
        if (K[k][i] != K[k][j]) return K[k][i] < K[k][j];
    return false;
}

template <int KW>
__device__ __forceinline__ bool reg_lt(const uint64_t (&a)[KW], const uint64_t (&b)[KW])
{
#pragma unroll
    for (int k = 0; k < KW; ++k)
        if (a[k] != b[k]) return a[k] < b[k];
    return false;
}

template <int KW>
__device__ __forceinline__ void reg_cx(uint64_t (&a)[KW], uint64_t (&b)[KW])
{
    if (reg_lt<KW>(b, a)) {
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const uint64_t x = a[k];
            a[k] = b[k];
            b[k] = x;
        }
    }
}

template <int KW>
__global__ __launch_bounds__(kCsThreads) void k_cs_block_sort(const uint64_t *src, uint64_t *dst, size_t n)
{
    static_assert(kCsPer == 4, "4 keys per thread");
    __shared__ uint64_t K[KW][kCsBlock];
    const size_t base = (size_t)blockIdx.x * kCsBlock;
    for (int e = threadIdx.x; e < kCsBlock * KW; e += kCsThreads) {
        const int i = e / KW, k = e - i * KW;
        K[k][i] = base + i < n ? src[base * KW + e] : ~0ull;
    }
    __syncthreads();
    const uint32_t t0 = threadIdx.x * kCsPer;
    uint64_t r[kCsPer][KW];
#pragma unroll
    for (int q = 0; q < kCsPer; ++q)
#pragma unroll
        for (int k = 0; k < KW; ++k) r[q][k] = K[k][t0 + q];
    // 4-key sorting network
    reg_cx<KW>(r[0], r[1]);
    reg_cx<KW>(r[2], r[3]);
    reg_cx<KW>(r[0], r[2]);
    reg_cx<KW>(r[1], r[3]);
    reg_cx<KW>(r[1], r[2]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kCsPer; ++q)
#pragma unroll
        for (int k = 0; k < KW; ++k) K[k][t0 + q] = r[q][k];
    __syncthreads();
    for (uint32_t run = kCsPer; run < (uint32_t)kCsBlock; run *= 2) {
        const uint32_t p0 = t0 / (2 * run) * (2 * run), d = t0 - p0;  // this thread's pair, diagonal
        const uint32_t a0 = p0, b0 = p0 + run;
        uint32_t lo = d > run ? d - run : 0, hi = min(d, run);
        while (lo < hi) {  // outputs [d, d + 4) of merging runs [a0, +run) and [b0, +run)
            const uint32_t mid = (lo + hi) >> 1;
            if (lds_lt<KW>(K, a0 + mid, b0 + d - 1 - mid))
                lo = mid + 1;
            else
                hi = mid;
        }
        uint32_t a = lo, b = d - lo;
#pragma unroll
        for (int q = 0; q < kCsPer; ++q) {
            const bool ta = b >= run || (a < run && lds_lt<KW>(K, a0 + a, b0 + b));
            const uint32_t from = ta ? a0 + a : b0 + b;
#pragma unroll
            for (int k = 0; k < KW; ++k) r[q][k] = K[k][from];
            a += ta;
            b += !ta;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kCsPer; ++q)
#pragma unroll
            for (int k = 0; k < KW; ++k) K[k][t0 + q] = r[q][k];
        __syncthreads();
    }
    for (int e = threadIdx.x; e < kCsBlock * KW; e += kCsThreads) {
        const int i = e / KW, k = e - i * KW;
        if (base + i < n) dst[base * KW + e] = K[k][i];
    }
}

// #elements of A among the first d outputs of merging A (la) and B (lb):
// keys are distinct, so the merge is unique.
template <int KW>
__device__ __forceinline__ uint32_t merge_split(const uint64_t *A, uint32_t la, const uint64_t *B,
                                                uint32_t lb, uint32_t d)
{
    uint32_t lo = d > lb ? d - lb : 0, hi = min(d, la);
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key_lt<KW>(A + (size_t)mid * KW, B + (size_t)(d - 1 - mid) * KW))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// merge_split for diagonal d by a 16-lane group (sub of the wave): 16-ary
// rounds -- every lane tests one sample split, a ballot counts the splits
// still taking A -- so a tile's split costs ~log16 dependent global reads
// instead of log2.  Every lane of the wave runs the same rounds.
template <int KW>
__device__ __forceinline__ uint32_t merge_split16(const uint64_t *A, uint32_t la, const uint64_t *B,
                                                  uint32_t lb, uint32_t d, bool act, int l16, int sub)
{
    uint32_t lo = act ? (d > lb ? d - lb : 0) : 0, hi = act ? min(d, la) : 0;
    // answer in [lo, hi]: the least i with !(A[i] < B[d - 1 - i])
    uint32_t len = hi - lo;
    while (__any(len != 0)) {
        const uint32_t st = (len + 15) >> 4, s = (uint32_t)(l16 + 1) * st;
        // sample lo + s - 1 still takes A: A[i] < B[d - 1 - i]
        const bool t = len && s <= len &&
                       key_lt<KW>(A + (size_t)(lo + s - 1) * KW, B + (size_t)(d - lo - s) * KW);
        const uint32_t m = __popc((uint32_t)(__ballot(t) >> (16 * sub)) & 0xFFFFu);
        if (len) {
            const uint32_t n0 = lo + m * st;
            len = min(st - 1, lo + len - n0), lo = n0;
        }
    }
    return lo;
}

// The split of every merge tile's first output (one 16-lane group per tile,
// all tiles at once): the merge's workgroups then start from a load instead
// of a chain of dependent global reads each (which left the pass latency-
// bound: 4 rounds of workgroups per CU, each waiting ~6 search rounds).
template <int KW>
__global__ __launch_bounds__(kCsThreads) void k_cs_splits(const uint64_t *src, size_t n, size_t L,
                                                          uint32_t ntiles, uint32_t *split)
{
    const int lane = threadIdx.x & 63, sub = lane >> 4, l16 = lane & 15;
    const uint32_t t = (blockIdx.x * kCsThreads + threadIdx.x) >> 4;
    const bool act = t < ntiles;
    const size_t o0 = act ? (size_t)t * kCsBlock : 0;
    const size_t p0 = o0 / (2 * L) * (2 * L);
    const uint32_t la = (uint32_t)min(L, n - p0);
    const uint32_t lb = (uint32_t)min(L, n - min(n, p0 + L));
    const uint64_t *A = src + p0 * KW, *B = A + (size_t)la * KW;
    const uint32_t sp = merge_split16<KW>(A, la, B, lb, (uint32_t)(o0 - p0), act, l16, sub);
    if (act && l16 == 0) split[t] = sp;
}

// One merge pass: runs of L keys of src merged pairwise into dst, 1024
// outputs per workgroup, from the splits k_cs_splits left.
template <int KW>
__global__ __launch_bounds__(kCsThreads) void k_cs_merge(const uint64_t *src, uint64_t *dst, size_t n,
                                                         size_t L, const uint32_t *split)
{
    __shared__ uint64_t S[kCsBlock * KW];
    __shared__ uint16_t pos[kCsBlock];  // output r of the tile = staged key pos[r]
    const size_t o0 = (size_t)blockIdx.x * kCsBlock;
    if (o0 >= n) return;
    const size_t p0 = o0 / (2 * L) * (2 * L);  // the pair's first key
    const uint32_t la = (uint32_t)min(L, n - p0);
    const uint32_t lb = (uint32_t)min(L, n - min(n, p0 + L));
    const uint64_t *A = src + p0 * KW, *B = A + (size_t)la * KW;
    const uint32_t d0 = (uint32_t)(o0 - p0), d1 = min(d0 + (uint32_t)kCsBlock, la + lb);
    // the pair's last tile ends with every key of A taken
    const uint32_t i0 = split[blockIdx.x], i1 = d1 == la + lb ? la : split[blockIdx.x + 1];
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t na = i1 - i0, nb = j1 - j0;
    // stage A[i0, i1) then B[j0, j1)
    for (uint32_t e = threadIdx.x; e < (na + nb) * KW; e += kCsThreads) {
        const uint32_t r = e / KW, k = e - r * KW;
        S[e] = r < na ? A[(size_t)(i0 + r) * KW + k] : B[(size_t)(j0 + r - na) * KW + k];
    }
    __syncthreads();
    const uint64_t *SA = S, *SB = S + (size_t)na * KW;
    const uint32_t dt = min((uint32_t)(threadIdx.x * kCsPer), na + nb);
    uint32_t a = merge_split<KW>(SA, na, SB, nb, dt), b = dt - a;
    for (int r = 0; r < kCsPer && a + b < na + nb; ++r) {
        const bool take_a = b >= nb || (a < na && key_lt<KW>(SA + (size_t)a * KW, SB + (size_t)b * KW));
        pos[dt + r] = (uint16_t)(take_a ? a : na + b);
        a += take_a;
        b += !take_a;
    }
    __syncthreads();
    // the tile's outputs leave in order: consecutive threads, consecutive words
    uint64_t *out = dst + o0 * KW;
    for (uint32_t e = threadIdx.x; e < (na + nb) * KW; e += kCsThreads) {
        const uint32_t r = e / KW, k = e - r * KW;
        out[e] = S[(size_t)pos[r] * KW + k];
    }
}

template <int KW>
hipError_t sort_kw(uint64_t *keys, uint64_t *tmp, uint32_t *split, size_t n, hipStream_t s,
                   uint64_t **sorted)
{
    const uint32_t blocks = (uint32_t)((n + kCsBlock - 1) / kCsBlock);
    k_cs_block_sort<KW><<<blocks, kCsThreads, 0, s>>>(keys, tmp, n);
    uint64_t *src = tmp, *dst = keys;
    const uint32_t sb = (blocks + kCsThreads / 16 - 1) / (kCsThreads / 16);
    for (size_t L = kCsBlock; L < n; L *= 2) {
        k_cs_splits<KW><<<sb, kCsThreads, 0, s>>>(src, n, L, blocks, split);
        k_cs_merge<KW><<<blocks, kCsThreads, 0, s>>>(src, dst, n, L, split);
        std::swap(src, dst);
    }
    *sorted = src;
    return hipGetLastError();
}

}  // namespace

size_t code_sort_split_words(size_t n) { return (n + kCsBlock - 1) / kCsBlock + 1; }

hipError_t code_keys_sort(uint64_t *keys, uint64_t *tmp, uint32_t *split, size_t n, int KW, hipStream_t s,
                          uint64_t **sorted)
{
    *sorted = keys;
    if (n == 0) return hipSuccess;
    switch (KW) {
    case 2: return sort_kw<2>(keys, tmp, split, n, s, sorted);
    case 3: return sort_kw<3>(keys, tmp, split, n, s, sorted);
    case 4: return sort_kw<4>(keys, tmp, split, n, s, sorted);
    default: return hipErrorInvalidValue;
    }
}

hipError_t warm_csort()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_cs_merge<4>);
}

}  // namespace hsc
