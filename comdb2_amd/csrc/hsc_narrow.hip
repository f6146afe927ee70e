// hsc_narrow.hip -- the narrow window layout and its direct probe.
//
// The reference answers one read set at a time: for every logged write key it
// scans the read ranges of the written index with a min-length memcmp
// (db/glue.c:2937-2961).  When every (group, key) of the resident window fits
// one 64-bit code, this layout answers every range of a batch independently,
// with no bucketing of ranges at all:
//
//   key64[i] = (K_i - K_0) >> s     K = gid || word 0 || ... || word W-1 (the
//                                   composite sort key), K_0 = the first row;
//                                   s = the low bits every row agrees on
//                                   (trailing key words that never vary plus
//                                   tz low bits of the last one that does: a
//                                   9-byte int64 key, 0x08 || BE(v ^ 2^63),
//                                   has tz = 56).  Valid if the window spans
//                                   less than 2^62 << s -- any one int64 index.
//
// A probe bound X maps exactly to  rows >= X  <=>  key64 >= ceil((X - K_0) / 2^s)
// and  rows <= X  <=>  key64 <= floor((X - K_0) / 2^s), so the min-length
// memcmp range test of the reference becomes two counts over sorted u64s.
//
// Index: a 16-ary tree of key levels (level l+1 holds the last key of every
// 16-entry block of level l; one 128-byte line per block) and a parallel tree
// of commit-LSN maxima.  A group of 16 lanes answers one range: each lane
// reads one entry of the block, a ballot counts the entries below the bound,
// so every level costs one line and one ballot.  Upper levels live in LDS,
// the rest in L2 / the Infinity Cache (the window of BASELINE config 2 is
// 160 MB).  The range maximum then takes at most two partial blocks per level
// of the max tree.  Every group keeps kNP ranges (2 kNP searches) in flight.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

namespace hsc {

constexpr uint64_t kKeyPad = ~0ull;      // key padding: above every bound
constexpr uint64_t kSat = 1ull << 62;    // saturated code: above every key

// (X - B) >> shift for composite keys X = (xg, xw[j * xs]) and B = (bg,
// bw[j * bs]), limbs most significant first: limb 0 = gid, limb j + 1 = word
// j.  shift = tz bits of limb lw plus every limb after lw (the window's rows
// agree on all of those bits).  Returns false if X < B.  Otherwise v =
// min((X - B) >> shift, sat) and rem = whether the shifted-out bits of X - B
// are nonzero.
__host__ __device__ inline bool rel_diff(int W, int lw, int tz, uint64_t xg, const uint64_t *xw,
                                         size_t xs, uint64_t bg, const uint64_t *bw, size_t bs,
                                         uint64_t sat, uint64_t &v, bool &rem)
{
    uint64_t borrow = 0, d_last = 0, d_prev = 0, high = 0, below = 0;
    for (int i = W; i >= 0; --i) {
        const uint64_t x = i ? xw[(size_t)(i - 1) * xs] : xg;
        const uint64_t b = i ? bw[(size_t)(i - 1) * bs] : bg;
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
    v = (high | top) ? sat : (low < sat ? low : sat);
    return true;
}

// rel_diff for W = 1 or 2 key words held in registers: the words subtract as
// one 128-bit borrow chain, the gid limb after it; the limb roles come from
// uniform branches on lw and the shift by tz (< 64) is a funnel shift whose
// tz = 0 case needs no branch ((d << 1) << 63 = 0).
template <int W>
__device__ __forceinline__ bool rel_diff_w(int lw, int tz, uint64_t xg, const uint64_t (&xw)[W],
                                           uint64_t bg, const uint64_t *bw, uint64_t sat,
                                           uint64_t &v, bool &rem)
{
    static_assert(W == 1 || W == 2, "register form for 1 or 2 words");
    typedef unsigned __int128 u128;
    uint64_t d[W + 1];
    bool borrow;
    if constexpr (W == 2) {
        const u128 x = (u128)xw[0] << 64 | xw[1], b = (u128)bw[0] << 64 | bw[1];
        const u128 dd = x - b;
        d[1] = (uint64_t)(dd >> 64);
        d[2] = (uint64_t)dd;
        borrow = x < b;
    } else {
        d[1] = xw[0] - bw[0];
        borrow = xw[0] < bw[0];
    }
    d[0] = xg - bg - (borrow ? 1 : 0);
    if (xg < bg || (xg == bg && borrow)) return false;
    uint64_t below, d_last, d_prev, high;
    if (W == 2 && lw == 2) {
        below = 0, d_last = d[W], d_prev = d[W - 1], high = d[0];
    } else if (lw == 1) {
        below = d[W] & (W == 2 ? ~0ull : 0), d_last = d[1], d_prev = d[0], high = 0;
    } else {
        below = d[1] | d[W], d_last = d[0], d_prev = 0, high = 0;
    }
    const uint64_t top = d_prev >> tz;
    const uint64_t low = (d_last >> tz) | ((d_prev << 1) << (63 - tz));
    rem = (below | (d_last & ((1ull << tz) - 1))) != 0;
    v = (high | top) ? sat : (low < sat ? low : sat);
    return true;
}

// Compressed codes (nv.comp): code(X) = compress(X over the rows' varying
// bits) - c0.  Rows map exactly; a bound X that leaves the rows' constant
// pattern maps by its first differing constant bit b (MSB first): with the
// varying bits above b as prefix, X is above every row of that prefix when
// its bit is 1 (#rows < X = #codes < (prefix + 1) << rest) and below them
// when 0 (#codes < prefix << rest) -- the compact codes' rule
// (hsc_compact_dev.h bound_word) on one word.  upper = false: the lower code
// (ceil: #codes < it = #rows < X), else the upper (floor: #codes <= it =
// #rows <= X); false = no row <= X (upper only).
__device__ __forceinline__ bool cnarrow_bound(const NarrowView &nv, uint64_t xg, const uint64_t *xw,
                                              size_t xs, bool upper, uint64_t &code)
{
    uint64_t acc = 0;
    int pos = 0, np = -1, xb = 0;
    for (int l = 0; l <= nv.W; ++l) {
        const uint64_t *cm = nv.cmeta + 8 * l;
        const uint64_t m = cm[0], pt = cm[1];
        uint64_t x = l ? xw[(size_t)(l - 1) * xs] : xg;
        if (np < 0) {
            const uint64_t d = (x ^ pt) & ~m;
            if (d) {
                const int b = 63 - __clzll(d);
                const uint64_t above = b == 63 ? 0 : ~0ull << (b + 1);
                np = pos + __popcll(m & above);
                xb = (int)((x >> b) & 1);
                x &= above;
            }
        } else {
            x = 0;
        }
        const int c = __popcll(m);
        if (c) {
            uint64_t mv[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) mv[q] = cm[2 + q];
            acc = (c >= 64 ? 0 : acc << c) | bits_compress(x, m, mv);
            pos += c;
        }
    }
    uint64_t lo, hi;
    bool live = true;
    if (np < 0) {
        lo = hi = acc;
    } else {
        const int low = pos - np;
        const uint64_t pre = low >= 64 ? 0 : acc >> low;
        lo = (xb ? pre + 1 : pre) << low;
        live = lo != 0;
        hi = lo - 1;
    }
    if (upper) {
        if (!live || hi < nv.c0) return false;
        code = hi - nv.c0 < kSat ? hi - nv.c0 : kSat;
        return true;
    }
    code = lo <= nv.c0 ? 0 : (lo - nv.c0 < kSat ? lo - nv.c0 : kSat);
    return true;
}

// A probe bound as a code, either form: lower (ceil) / upper (floor); false
// (upper only) = no row at or below X.  Generic width (rel_diff).
__device__ __forceinline__ bool narrow_bound(const NarrowView &nv, uint64_t xg, const uint64_t *xw,
                                             size_t xs, bool upper, uint64_t &code)
{
    if (nv.comp) return cnarrow_bound(nv, xg, xw, xs, upper, code);
    uint64_t v;
    bool rem;
    if (!rel_diff(nv.W, nv.lw, nv.tz, xg, xw, xs, nv.base[0], nv.base + 1, 1, kSat, v, rem)) {
        code = 0;
        return !upper;  // below the window: lower 0, upper none
    }
    code = upper ? v : (v >= kSat ? kSat : v + (rem ? 1 : 0));
    return true;
}

bool narrow_span_fits(int W, int lw, int tz, const uint64_t *first, const uint64_t *last)
{
    uint64_t v;
    bool rem;
    if (!rel_diff(W, lw, tz, last[0], last + 1, 1, first[0], first + 1, 1, kSat, v, rem))
        return false;
    return !rem && v < kSat;
}

// ============================================================================
// window build
// ============================================================================
// rows 0 and n-1 as limbs (gid, words) -> out[0 .. W], out[W+1 .. 2W+1]
// (n_dev: the row count on the device, read there -- no host round trip)
__global__ void k_end_rows(WinView w, const uint32_t *n_dev, uint64_t *out)
{
    const int j = threadIdx.x;
    if (j > w.W) return;
    const uint32_t n = n_dev ? *n_dev : w.n;
    const size_t r[2] = {0, n ? (size_t)n - 1 : 0};
    for (int k = 0; k < 2; ++k)
        out[k * (w.W + 1) + j] =
            !n ? 0 : j ? w.words[(size_t)(j - 1) * w.stride + r[k]] : w.gid[r[k]];
}

hipError_t narrow_end_rows(const WinView &w, const uint32_t *n_dev, uint64_t *out, hipStream_t s)
{
    k_end_rows<<<1, 128, 0, s>>>(w, n_dev, out);
    return hipGetLastError();
}

namespace {
constexpr uint32_t kNoTile32 = 0xFFFFFFFFu;
constexpr int kTLog2 = 12;  // 4096-row tiles (= the code view's tiles)
}  // namespace

// Eytzinger (BFS) slot of sorted row r of a 4096-row tile: rows 0 .. 4094
// form a perfect binary tree at slots 1 .. 4095 (in-order index i = r + 1 sits
// at level 11 - ctz(i)), row 4095 at slot 0.  A root-to-leaf walk touches
// slots spread over a level instead of the power-of-two strides of a binary
// search over sorted rows, which all fall in one or two LDS banks.
static_assert(kTLog2 == 12, "eyt12 assumes 4096-row tiles");
__device__ __forceinline__ uint32_t eyt12(uint32_t r)
{
    const uint32_t i = r + 1;
    const int tz = __builtin_ctz(i);
    return i == 4096 ? 0 : (1u << (11 - tz)) + (i >> (tz + 1));
}

// level 0: key64 of every row (padding above n), lsn (padding 0)
__global__ void k_level0(WinView w, NarrowView nv, uint32_t len, uint64_t *key0, uint64_t *max0)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    uint64_t v = kKeyPad, m = 0;
    if (i < w.n) {
        bool rem;
        if (nv.comp)
            cnarrow_bound(nv, w.gid[i], w.words + i, w.stride, false, v);
        else
            rel_diff(w.W, nv.lw, nv.tz, w.gid[i], w.words + i, w.stride, nv.base[0], nv.base + 1, 1, kSat,
                     v, rem);
        m = w.lsn[i];
    }
    key0[i] = v;
    max0[i] = m;
}

// levels 0 and 1 in one pass: level 1's entry of every 16 rows from the 16
// lanes that hold them (last key, LSN maximum by shuffles) -- no second pass
// re-reading level 0's LSN column.  len0 is a multiple of the block size (whole
// tiles), level 1's entries past len0 / 16 are padding.
__device__ __forceinline__ uint64_t level0_key(const WinView &w, const NarrowView &nv, size_t i)
{
    uint64_t v = kKeyPad;
    bool rem;
    if (nv.comp)
        cnarrow_bound(nv, w.gid[i], w.words + i, w.stride, false, v);
    else
        rel_diff(w.W, nv.lw, nv.tz, w.gid[i], w.words + i, w.stride, nv.base[0], nv.base + 1, 1, kSat, v, rem);
    return v;
}

// The narrow tiles' rows from the same pass (narrow_build with key32): one
// 4096-row tile per workgroup, 4 rows per thread -- key32 = key64 - the tile's
// first key64, staged in LDS in the tile's Eytzinger order and stored
// coalesced; rank32 = LSN - base + 1 in lsn32 mode; *flag if a tile spans
// >= 2^32 (what k_key32 / k_rank_lsn32 write, without their passes over level 0)
struct Level01Tiles {
    uint32_t *key32, *rank32, *flag;
    uint64_t rank_base;
};

__global__ __launch_bounds__(256) void k_level01(WinView w, NarrowView nv, uint32_t len, uint64_t *key0,
                                                 uint64_t *max0, uint64_t *key1, uint64_t *max1, uint32_t len1)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t v = kKeyPad, m = 0;
    if (i < w.n) v = level0_key(w, nv, i), m = w.lsn[i];
    if (i < len) key0[i] = v, max0[i] = m;
    uint64_t mm = m;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        const uint64_t y = __shfl_xor(mm, o, 16);
        mm = y > mm ? y : mm;
    }
    if ((i & 15) == 15 && i < len) key1[i >> 4] = v, max1[i >> 4] = mm;
    const size_t pad = len / 16 + i;
    if (pad < len1) key1[pad] = kKeyPad, max1[pad] = 0;
}

constexpr int kL01TThreads = 1024;
__global__ __launch_bounds__(kL01TThreads) void k_level01t(WinView w, NarrowView nv, uint32_t len,
                                                           uint64_t *key0, uint64_t *max0, uint64_t *key1,
                                                           uint64_t *max1, uint32_t len1, Level01Tiles T)
{
    constexpr int R = (1 << kTLog2) / kL01TThreads;
    __shared__ uint32_t st[1 << kTLog2];
    __shared__ uint64_t tfirst;
    const size_t base = (size_t)blockIdx.x << kTLog2;
    uint64_t v[R], m[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const size_t i = base + (size_t)k * kL01TThreads + threadIdx.x;
        v[k] = kKeyPad, m[k] = 0;
        if (i < w.n) v[k] = level0_key(w, nv, i), m[k] = w.lsn[i];
    }
    if (threadIdx.x == 0) tfirst = v[0];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const size_t i = base + (size_t)k * kL01TThreads + threadIdx.x;  // (< len: whole tiles)
        key0[i] = v[k], max0[i] = m[k];
        uint64_t mm = m[k];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint64_t y = __shfl_xor(mm, o, 16);
            mm = y > mm ? y : mm;
        }
        if ((i & 15) == 15) key1[i >> 4] = v[k], max1[i >> 4] = mm;
        if (T.rank32) T.rank32[i] = i < w.n ? (uint32_t)(m[k] - T.rank_base) + 1 : 0;
    }
    if (blockIdx.x == 0 && len / 16 + threadIdx.x < len1)
        key1[len / 16 + threadIdx.x] = kKeyPad, max1[len / 16 + threadIdx.x] = 0;
    __syncthreads();
    const uint64_t f = tfirst;
    bool wide = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t r = k * kL01TThreads + threadIdx.x;
        uint32_t x = 0xFFFFFFFFu;
        if (base + r < w.n) {
            const uint64_t d = v[k] - f;
            wide |= d > 0xFFFFFFFFull;
            x = (uint32_t)d;
        }
        st[eyt12(r)] = x;
    }
    if (wide) atomicOr(T.flag, 1u);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t r = k * kL01TThreads + threadIdx.x;
        T.key32[base + r] = st[r];
    }
}

// level l + 1 from level l: last key / max lsn of every 16-entry block
__global__ void k_level_up(const uint64_t *key_src, const uint64_t *max_src, uint32_t len_src,
                           uint64_t *key_dst, uint64_t *max_dst, uint32_t len_dst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len_dst) return;
    uint64_t k = kKeyPad, m = 0;
    if (i < len_src / 16) {
        k = key_src[16 * (size_t)i + 15];
        const ulonglong2 *src = (const ulonglong2 *)(max_src + 16 * (size_t)i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const ulonglong2 v = src[j];
            m = v.x > m ? v.x : m;
            m = v.y > m ? v.y : m;
        }
    }
    key_dst[i] = k;
    max_dst[i] = m;
}

bool narrow_level01_tiles(const NarrowView &nv)
{
    static const bool sep = getenv("HSC_LEVEL_SEP") != nullptr;
    return !sep && nv.levels >= 2 && nv.len[0] % (1u << kTLog2) == 0;
}

hipError_t narrow_build(const WinView &w, const NarrowView &nv, hipStream_t s, uint32_t *key32,
                        uint32_t *rank32, uint64_t rank_base, uint32_t *flag)
{
    const uint32_t len0 = nv.len[0];
    static const bool sep = getenv("HSC_LEVEL_SEP") != nullptr;  // (A/B: level 1 by its own pass)
    int l = 1;
    if (key32 && !narrow_level01_tiles(nv)) return hipErrorInvalidValue;
    if (nv.levels >= 2 && len0 % 256 == 0 && !sep) {
        if (key32) {
            const hipError_t e = hipMemsetAsync(flag, 0, 4, s);
            if (e != hipSuccess) return e;
        }
        uint64_t *k1 = (uint64_t *)nv.keys + nv.off[1], *m1 = (uint64_t *)nv.maxs + nv.off[1];
        if (key32)
            k_level01t<<<len0 >> kTLog2, kL01TThreads, 0, s>>>(w, nv, len0, (uint64_t *)nv.keys, (uint64_t *)nv.maxs,
                                                               k1, m1, nv.len[1],
                                                               Level01Tiles{key32, rank32, flag, rank_base});
        else
            k_level01<<<len0 / 256, 256, 0, s>>>(w, nv, len0, (uint64_t *)nv.keys, (uint64_t *)nv.maxs, k1, m1,
                                                 nv.len[1]);
        l = 2;
    } else {
        k_level0<<<(len0 + 255) / 256, 256, 0, s>>>(w, nv, len0, (uint64_t *)nv.keys, (uint64_t *)nv.maxs);
    }
    for (; l < nv.levels; ++l)
        k_level_up<<<(nv.len[l] + 255) / 256, 256, 0, s>>>(
            nv.keys + nv.off[l - 1], nv.maxs + nv.off[l - 1], nv.len[l - 1],
            (uint64_t *)nv.keys + nv.off[l], (uint64_t *)nv.maxs + nv.off[l], nv.len[l]);
    return hipGetLastError();
}

// ============================================================================
// probe
// ============================================================================
constexpr int kProbeThreads = 256;
constexpr int kNP = 4;  // ranges per 16-lane group in flight

// A conflict mark.  kHost: the verdict bytes live in fine-grained host memory
// (the small-batch path) -- a system-scope store writes through to it, so the
// kernel's completion needs no L2 write-back.
template <bool kHost>
__device__ __forceinline__ void mark_verdict(uint8_t *v)
{
    if constexpr (kHost)
        __hip_atomic_store(v, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
        *v = 1;
}

// The ranges of p answered by 16-lane groups, kNP ranges each: wave w of the
// grid starts at range wave0 and strides by wstride.  Levels >= lds_from are
// read from top (LDS, lds_base = their offset), the rest from the window.
template <bool kHost = false>
__device__ __forceinline__ void narrow_probe_ranges(const NarrowView &nv, const ProbeView &p,
                                                    uint8_t *verdict, const uint64_t *top,
                                                    uint64_t lds_base, int lds_from,
                                                    uint32_t wave0, uint32_t wstride)
{
    const int lane = threadIdx.x & 63;
    const int sub = lane >> 4, l16 = lane & 15;
    const size_t ks = p.n;
    // every wave runs the same number of iterations (ballots need all lanes)
    for (uint32_t wbase = wave0; wbase < p.n; wbase += wstride) {
        const uint32_t base = wbase + sub * kNP;
        // lane k < kNP of the group maps range base + k to codes
        uint64_t mlo = kSat, mhi = 0, msnap = 0;
        uint32_t mtxn = 0;
        bool mlive = false;
        {
            const uint32_t q = base + l16;
            if (l16 < kNP && q < p.n) {
                const uint32_t g = p.gid[q];
                msnap = p.snap[q];
                mtxn = p.txn[q];
                // lower bound: ceil((lo - K0) >> s), 0 below the window;
                // upper bound: floor((hi - K0) >> s), none below the window
                narrow_bound(nv, g, p.lo + q, ks, false, mlo);
                mlive = narrow_bound(nv, g, p.hi + q, ks, true, mhi);
                if (!mlive) mhi = 0;
            }
        }
        uint64_t x[2 * kNP], snap[kNP];
        uint32_t txn[kNP];
        bool live[kNP];
#pragma unroll
        for (int k = 0; k < kNP; ++k) {
            const int src = (lane & 48) + k;
            x[2 * k] = __shfl(mlo, src, 64);
            x[2 * k + 1] = __shfl(mhi, src, 64);
            snap[k] = __shfl(msnap, src, 64);
            txn[k] = __shfl(mtxn, src, 64);
            live[k] = __shfl((int)mlive, src, 64) != 0;
        }
        // 2 kNP counts in lockstep: c[2k] = #keys < lo_k, c[2k+1] = #keys <= hi_k
        uint32_t c[2 * kNP];
#pragma unroll
        for (int j = 0; j < 2 * kNP; ++j) c[j] = 0;
        for (int l = nv.levels - 1; l >= 0; --l) {
            uint64_t e[2 * kNP];
            if (l >= lds_from) {
                const uint64_t *lv = top + (nv.off[l] - lds_base);
#pragma unroll
                for (int j = 0; j < 2 * kNP; ++j) e[j] = lv[16 * c[j] + l16];
            } else {
                const uint64_t *lv = nv.keys + nv.off[l];
#pragma unroll
                for (int j = 0; j < 2 * kNP; ++j) e[j] = lv[16 * (size_t)c[j] + l16];
            }
#pragma unroll
            for (int j = 0; j < 2 * kNP; ++j) {
                const bool below = (j & 1) ? e[j] <= x[j] : e[j] < x[j];
                const uint32_t m = (uint32_t)(__ballot(below) >> (16 * sub)) & 0xFFFFu;
                c[j] = 16 * c[j] + __popc(m);
            }
        }
        // any lsn > snapshot over rows [p, q): up the max tree, at most two
        // partial blocks per level
        uint32_t pp[kNP], qq[kNP];
        bool found[kNP];
#pragma unroll
        for (int k = 0; k < kNP; ++k) {
            pp[k] = c[2 * k];
            qq[k] = live[k] ? c[2 * k + 1] : 0;
            found[k] = false;
        }
        for (int l = 0; l < nv.levels; ++l) {
            bool more = false;
#pragma unroll
            for (int k = 0; k < kNP; ++k) more |= pp[k] < qq[k];
            if (!__any(more)) break;
            const uint64_t *lv = nv.maxs + nv.off[l];
            uint64_t vl[kNP], vr[kNP];
#pragma unroll
            for (int k = 0; k < kNP; ++k) {
                const bool act = pp[k] < qq[k];
                const uint32_t il = (pp[k] & ~15u) + l16;
                const uint32_t ir = ((qq[k] - 1) & ~15u) + l16;
                vl[k] = act && il >= pp[k] && il < qq[k] ? lv[il] : 0;
                vr[k] = act && ir >= pp[k] && ir < qq[k] ? lv[ir] : 0;
            }
#pragma unroll
            for (int k = 0; k < kNP; ++k) {
                const bool act = pp[k] < qq[k];
                const bool hit = vl[k] > snap[k] || vr[k] > snap[k];
                found[k] |= ((uint32_t)(__ballot(hit) >> (16 * sub)) & 0xFFFFu) != 0;
                const uint32_t np = (pp[k] + 15) >> 4, nq = qq[k] >> 4;
                const bool done = !act || found[k] || (pp[k] >> 4) == ((qq[k] - 1) >> 4) || np >= nq;
                pp[k] = done ? 0 : np;
                qq[k] = done ? 0 : nq;
            }
        }
        if (l16 == 0) {
#pragma unroll
            for (int k = 0; k < kNP; ++k)
                if (found[k]) mark_verdict<kHost>(verdict + txn[k]);
        }
    }
}

// table locks q = first, first + stride, ...: any write to a locked table
// after the snapshot
template <bool kHost = false>
__device__ __forceinline__ void narrow_probe_locks(const NarrowView &nv, const ProbeView &p,
                                                   uint8_t *verdict, uint32_t first, uint32_t stride)
{
    for (uint32_t q = first; q < p.n_lock; q += stride) {
        const uint32_t t = p.lock_table[q];
        if (t < nv.ntables && nv.table_max[t] > p.lock_snap[q]) mark_verdict<kHost>(verdict + p.lock_txn[q]);
    }
}

__global__ __launch_bounds__(kProbeThreads) void k_probe_narrow(NarrowView nv, ProbeView p,
                                                                uint8_t *verdict)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t top[];  // levels >= lds_from
    const uint64_t lds_base = nv.off[nv.lds_from];
    for (uint32_t i = threadIdx.x; i < nv.lds_entries; i += kProbeThreads)
        top[i] = nv.keys[lds_base + i];
    __syncthreads();
    const uint32_t groups = gridDim.x * (kProbeThreads / 16);
    const uint32_t wave0 = (blockIdx.x * (kProbeThreads / 16) + ((threadIdx.x >> 6) << 2)) * kNP;
    narrow_probe_ranges(nv, p, verdict, top, lds_base, nv.lds_from, wave0, groups * kNP);
    narrow_probe_locks(nv, p, verdict, blockIdx.x * kProbeThreads + threadIdx.x,
                       gridDim.x * kProbeThreads);
}

// Small batches of the drop-in entry (a lone bdb_osql_serial_check, a
// collector's batch of concurrent calls): one launch answers the ranges from
// the key and max trees (no LDS staging: a handful of searches would not pay
// for it), the delta run and the table locks.  The probe columns are read
// straight from the caller's pinned staging and the verdict bytes written into
// it (fine-grained host memory the GPU maps: no copies); the last block to
// finish stores `seq` into *done, which the host polls.  Completion needs no
// cache write-back: every verdict byte is a write-through system-scope store,
// each thread waits for its stores before the block counts itself done, and
// the done word is written (write-through, same path to the host) after the
// last block's count.
constexpr int kSmallThreads = 256;

// The small batches' range search, latency first: one range per 16-lane group
// (a lone call's ten ranges fill ten groups at once).  Lane 0 maps lo, lane 1
// hi.  The key tree is descended two levels per dependent step: the 256
// entries of level l - 1 under one entry of level l + 1 are contiguous (16 per
// lane, 2 KiB per group), so their count below the bound skips level l.  The
// range maximum needs no dependent chain at all: the partial blocks of every
// level follow from pa, pb by arithmetic, so kSmallRound levels' loads are
// issued together.
constexpr int kSmallRound = 4;
constexpr int kSmallLevels = kSmallMaxLevels;  // the host keeps deeper windows off this path
static_assert(kSmallLevels <= kMaxLevels, "level offsets");

__device__ __forceinline__ uint32_t group_sum16(uint32_t v)
{
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
    return v;
}

// #entries of the 16 at e (a lane's run of a level) below x (LE: <= x); none
// when the run starts at or past the level's end
template <bool LE>
__device__ __forceinline__ uint32_t run_below(const uint64_t *e, bool in, uint64_t x)
{
    if (!in) return 0;
    uint32_t n = 0;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        const ulonglong2 v = *(const ulonglong2 *)(e + i);
        n += LE ? (v.x <= x) + (v.y <= x) : (v.x < x) + (v.y < x);
    }
    return n;
}

// KW = 1, 2: the bound's words loaded together into registers (they live in
// host memory: one PCIe round trip, not one per word) and mapped by
// rel_diff_w; KW = 0: any width through rel_diff
// a small batch's conflict mark: the verdict byte (system-scope store), or
// with vmask (a packed one-block batch) the read set's bit in LDS
__device__ __forceinline__ void small_mark(uint8_t *verdict, uint32_t *vmask, uint32_t txn)
{
    if (vmask)
        atomicOr(vmask, 1u << txn);
    else
        mark_verdict<true>(verdict + txn);
}

template <int KW>
__device__ __forceinline__ void narrow_small_ranges(const NarrowView &nv, const ProbeView &p,
                                                    uint8_t *verdict, uint32_t *vmask, uint32_t wave0,
                                                    uint32_t wstride)
{
    const int lane = threadIdx.x & 63, sub = lane >> 4, l16 = lane & 15, g0 = lane & 48;
    const size_t ks = p.n;
    for (uint32_t wbase = wave0; wbase < p.n; wbase += wstride) {
        const uint32_t q = wbase + sub;
        const bool act = q < p.n;
        uint64_t xv = 0, sn = 0;
        uint32_t tx = 0;
        int ok = 0;
        if (act && l16 < 2) {
            uint64_t v = 0;
            bool rem = false;
            const uint64_t *xp = l16 ? p.hi + q : p.lo + q;
            if (nv.comp) {  // compressed codes: the bound's code either way
                ok = narrow_bound(nv, p.gid[q], xp, ks, l16 != 0, v);
                xv = ok ? v : 0;
            } else {
                if constexpr (KW > 0) {
                    const uint32_t g = p.gid[q];
                    uint64_t xw[KW];
#pragma unroll
                    for (int j = 0; j < KW; ++j) xw[j] = xp[(size_t)j * ks];
                    ok = rel_diff_w<KW>(nv.lw, nv.tz, g, xw, nv.base[0], nv.base + 1, kSat, v, rem);
                } else {
                    ok = rel_diff(nv.W, nv.lw, nv.tz, p.gid[q], xp, ks, nv.base[0], nv.base + 1, 1, kSat,
                                  v, rem);
                }
                // lower bound: ceil((lo - K0) >> s), 0 below the window; upper:
                // floor((hi - K0) >> s), none below the window
                xv = !ok ? 0 : l16 ? v : (v >= kSat ? kSat : v + (rem ? 1 : 0));
            }
        } else if (act && l16 == 2) {
            sn = p.snap[q];
            tx = p.txn[q];
        }
        const uint64_t xlo = __shfl(xv, g0, 64), xhi = __shfl(xv, g0 + 1, 64);
        const bool live = act && __shfl(ok, g0 + 1, 64) != 0;
        const uint64_t snap = __shfl(sn, g0 + 2, 64);
        const uint32_t txn = __shfl(tx, g0 + 2, 64);
        // ca / cb: the block index at level l (the count below the bound at
        // l + 1).  Levels are compile-time indices (a window of < 2^32 rows
        // has at most kSmallLevels): every level's offset is a kernel-argument
        // load the prologue issues at once, not one per step.
        uint32_t ca = 0, cb = 0;
        const int top = nv.levels - 1;
#pragma unroll
        for (int l = kSmallLevels - 1; l >= 1; --l) {
            if (l > top || ((top - l) & 1)) continue;  // uniform
            const uint64_t *lv = nv.keys + nv.off[l - 1];
            const size_t len = nv.len[l - 1];
            const size_t ia = 256 * (size_t)ca + 16 * l16, ib = 256 * (size_t)cb + 16 * l16;
            const uint32_t na = run_below<false>(lv + ia, ia < len, xlo);
            const uint32_t nb = run_below<true>(lv + ib, ib < len, xhi);
            ca = 256 * ca + group_sum16(na);
            cb = 256 * cb + group_sum16(nb);
        }
        if ((top & 1) == 0) {  // level 0 left: a 16-ary step
            const uint64_t *lv = nv.keys;
            const bool ba = lv[16 * (size_t)ca + l16] < xlo, bb = lv[16 * (size_t)cb + l16] <= xhi;
            ca = 16 * ca + __popc((uint32_t)(__ballot(ba) >> (16 * sub)) & 0xFFFFu);
            cb = 16 * cb + __popc((uint32_t)(__ballot(bb) >> (16 * sub)) & 0xFFFFu);
        }
        // any lsn > snapshot over rows [P, Q): level L's partial blocks
        uint32_t P = ca, Q = live ? cb : 0;
        bool on = act && P < Q, found = false;
#pragma unroll
        for (int lev = 0; lev < kSmallLevels; lev += kSmallRound) {
            if (!__any(on)) break;
            uint64_t vl[kSmallRound], vr[kSmallRound];
#pragma unroll
            for (int r = 0; r < kSmallRound; ++r) {
                const int L = lev + r;
                const bool a = on && L < nv.levels;
                const uint64_t *lv = nv.maxs + nv.off[L];
                const uint32_t il = (P & ~15u) + l16, ir = ((Q - 1) & ~15u) + l16;
                vl[r] = a && il >= P && il < Q ? lv[il] : 0;
                vr[r] = a && ir >= P && ir < Q ? lv[ir] : 0;
                const uint32_t np = (P + 15) >> 4, nq = Q >> 4;
                on = a && (P >> 4) != ((Q - 1) >> 4) && np < nq;
                P = np, Q = nq;
            }
            bool hit = false;
#pragma unroll
            for (int r = 0; r < kSmallRound; ++r) hit |= vl[r] > snap || vr[r] > snap;
            found |= ((uint32_t)(__ballot(hit) >> (16 * sub)) & 0xFFFFu) != 0;
            on = on && !found;
        }
        if (act && found && l16 == 0) small_mark(verdict, vmask, txn);
    }
}

// ---- the appended rows: delta runs and the pending tail --------------------
// Keys as full composites (gid, W words) held in registers, W <= kPendMaxWords.

// row i of d below the key: (gid, words) < (g, k), or <= with !strict
template <int W>
__device__ __forceinline__ bool row_below(const DeltaView &d, uint32_t i, uint32_t g,
                                          const uint64_t (&k)[W], bool strict)
{
    const uint32_t rg = d.gid[i];
    uint64_t w[W];
#pragma unroll
    for (int j = 0; j < W; ++j) w[j] = d.words[(size_t)j * d.stride + i];
    if (rg != g) return rg < g;
#pragma unroll
    for (int j = 0; j < W; ++j)
        if (w[j] != k[j]) return w[j] < k[j];
    return !strict;
}

__device__ __forceinline__ bool group_any(bool x, int sub)
{
    return ((uint32_t)(__ballot(x) >> (16 * sub)) & 0xFFFFu) != 0;
}

// A 16-lane group (sub of the wave) asks: a row of d in [lo, hi] of group g
// committed after snap?  Both bounds come from 16-ary searches run in
// lockstep -- each round every lane reads one sample row, a ballot counts the
// samples below the bound and the interval shrinks 16-fold (4 rounds for a
// full 65536-row run, against 16 dependent steps of a binary search) -- then
// the LSNs between them 16 units at a time: rows at the ends, the 64-row
// maxima between.  Every lane of the wave runs the same rounds (ballots).
template <int W>
__device__ bool delta_range16(const DeltaView &d, bool act, uint32_t g, const uint64_t (&lo)[W],
                              const uint64_t (&hi)[W], uint64_t snap, int l16, int sub)
{
    uint32_t a0 = 0, al = act ? d.n : 0, b0 = 0, bl = al;  // count in [x0, x0 + xl]
    while (__any((al | bl) != 0)) {
        const uint32_t as = (al + 15) >> 4, bs = (bl + 15) >> 4;
        const uint32_t sa = (uint32_t)(l16 + 1) * as, sb = (uint32_t)(l16 + 1) * bs;
        const bool ab = al && sa <= al && row_below<W>(d, a0 + sa - 1, g, lo, true);
        const bool bb = bl && sb <= bl && row_below<W>(d, b0 + sb - 1, g, hi, false);
        const uint32_t ma = __popc((uint32_t)(__ballot(ab) >> (16 * sub)) & 0xFFFFu);
        const uint32_t mb = __popc((uint32_t)(__ballot(bb) >> (16 * sub)) & 0xFFFFu);
        if (al) {
            const uint32_t n0 = a0 + ma * as;
            al = min(as - 1, a0 + al - n0), a0 = n0;
        }
        if (bl) {
            const uint32_t n0 = b0 + mb * bs;
            bl = min(bs - 1, b0 + bl - n0), b0 = n0;
        }
    }
    // rows [pa, pb): h head rows, nb whole 64-row blocks, t tail rows
    const uint32_t pa = a0, pb = b0;
    uint32_t h = 0, nb = 0, t = 0, hend = pa, ts = pb;
    if (pa < pb) {
        hend = min(pb, (pa + 63) & ~63u);
        const uint32_t bend = pb & ~63u;
        nb = hend < bend ? (bend - hend) >> 6 : 0;
        ts = max(hend, bend);
        h = hend - pa, t = pb - ts;
    }
    const uint32_t U = h + nb + t;
    bool found = false;
    for (uint32_t k = 0; __any(k < U && !found); k += 16) {
        const uint32_t u = k + l16;
        bool hit = false;
        if (u < U && !found) {
            const uint64_t v = u < h        ? d.lsn[pa + u]
                               : u < h + nb ? d.bmax[(hend >> 6) + (u - h)]
                                            : d.lsn[ts + (u - h - nb)];
            hit = v > snap;
        }
        found |= group_any(hit, sub);
    }
    return found;
}

// the pending tail staged in LDS by every block of the second half
struct PendLds {
    uint32_t gid[kPendRows];
    uint64_t lsn[kPendRows];
    uint64_t words[kPendMaxWords][kPendRows];
    uint32_t ttid[kPendRows];
    uint64_t tlsn[kPendRows];
};

template <int W>
__device__ __forceinline__ bool pend_range16(const PendLds &s, uint32_t n, bool act, uint32_t g,
                                             const uint64_t (&lo)[W], const uint64_t (&hi)[W],
                                             uint64_t snap, int l16, int sub)
{
    bool hit = false;
    for (uint32_t r = l16; act && r < n; r += 16) {
        if (s.gid[r] != g || s.lsn[r] <= snap) continue;
        int cl = 0, ch = 0;  // sign of row - lo, row - hi (first differing word)
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const uint64_t w = s.words[j][r];
            if (!cl && w != lo[j]) cl = w < lo[j] ? -1 : 1;
            if (!ch && w != hi[j]) ch = w < hi[j] ? -1 : 1;
        }
        hit |= cl >= 0 && ch <= 0;
    }
    return group_any(hit, sub);
}

// The second half of k_small_narrow with W <= kPendMaxWords: a 16-lane group
// per range over the live run, a frozen one and the pending tail; a thread per
// table lock over the pending table maxima.
template <int W>
__device__ void small_appended16(const DeltaView &d, const DeltaView &d2, const PendView &pd,
                                 const ProbeView &p, uint8_t *verdict, uint32_t blk, uint32_t nblk)
{
    __shared__ PendLds s;
    if (pd.n || pd.nt) {
        const uint8_t *b = pd.base;
        for (uint32_t r = threadIdx.x; r < pd.n; r += kSmallThreads) {
            s.gid[r] = ((const uint32_t *)b)[r];
            s.lsn[r] = ((const uint64_t *)(b + kPendLsn))[r];
#pragma unroll
            for (int j = 0; j < W; ++j) s.words[j][r] = ((const uint64_t *)(b + kPendWords))[j * kPendRows + r];
        }
        for (uint32_t r = threadIdx.x; r < pd.nt; r += kSmallThreads) {
            s.ttid[r] = ((const uint32_t *)(b + kPendTtid))[r];
            s.tlsn[r] = ((const uint64_t *)(b + kPendTlsn))[r];
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, sub = lane >> 4, l16 = lane & 15;
    const uint32_t wave = blk * (kSmallThreads / 64) + (threadIdx.x >> 6);
    const uint32_t nwaves = nblk * (kSmallThreads / 64);
    for (uint32_t base = 4 * wave; base < p.n; base += 4 * nwaves) {
        const uint32_t q = base + sub;
        const bool act = q < p.n;
        uint32_t g = 0;
        uint64_t lo[W], hi[W], snap = 0;
#pragma unroll
        for (int j = 0; j < W; ++j) lo[j] = hi[j] = 0;
        if (act) {
            g = p.gid[q];
            snap = p.snap[q];
#pragma unroll
            for (int j = 0; j < W; ++j) lo[j] = p.lo[(size_t)j * p.n + q], hi[j] = p.hi[(size_t)j * p.n + q];
        }
        bool hit = false;
        if (d.n) hit |= delta_range16<W>(d, act, g, lo, hi, snap, l16, sub);
        if (d2.n) hit |= delta_range16<W>(d2, act && !hit, g, lo, hi, snap, l16, sub);
        if (pd.n) hit |= pend_range16<W>(s, pd.n, act && !hit, g, lo, hi, snap, l16, sub);
        if (act && hit && l16 == 0) mark_verdict<true>(verdict + p.txn[q]);
    }
    for (uint32_t q = blk * kSmallThreads + threadIdx.x; pd.nt && q < p.n_lock; q += nblk * kSmallThreads) {
        const uint32_t t = p.lock_table[q];
        const uint64_t ls = p.lock_snap[q];
        bool hit = false;
        for (uint32_t e = 0; e < pd.nt && !hit; ++e) hit = s.ttid[e] == t && s.tlsn[e] > ls;
        if (hit) mark_verdict<true>(verdict + p.lock_txn[q]);
    }
}

// WD = 0: keys wider than kPendMaxWords (no pending tail), a thread per range
// and binary searches; WD = 1..4: small_appended16<WD>.  KW: the window's
// search form (narrow_small_ranges<KW>), one per kernel (the code a launch
// runs stays small: its first instruction fetches are on the call's path).
template <int WD, int KW>
__global__ __launch_bounds__(kSmallThreads) void k_small_narrow(NarrowView nv, DeltaView d,
                                                                DeltaView d2, PendView pd,
                                                                ProbeView p, uint8_t *verdict,
                                                                uint32_t *blocks_done,
                                                                uint64_t *done, uint32_t seq, uint32_t pack)
{
    // with appended rows not in the window, the second half of the grid
    // searches them while the first half searches the window (both dependent
    // load chains run side by side instead of one after the other)
    const bool split = d.n || d2.n || pd.n || pd.nt;
    const uint32_t half = split ? gridDim.x / 2 : gridDim.x;
    __shared__ uint32_t vbits;
    const bool packed = pack && gridDim.x == 1;  // (split grids have two blocks at least)
    if (packed) {
        if (threadIdx.x == 0) vbits = 0;
        __syncthreads();
    }
    uint32_t *vmask = packed ? &vbits : nullptr;
    if (blockIdx.x < half) {
        const uint32_t groups = half * (kSmallThreads / 16);
        const uint32_t wave0 = blockIdx.x * (kSmallThreads / 16) + ((threadIdx.x >> 6) << 2);
        if (split) {  // (measured: the appended rows' half sets the pace; kNP ranges per group)
            narrow_probe_ranges<true>(nv, p, verdict, nullptr, 0, nv.levels, wave0 * kNP, groups * kNP);
        } else {
            narrow_small_ranges<KW>(nv, p, verdict, vmask, wave0, groups);
        }
        for (uint32_t q = blockIdx.x * kSmallThreads + threadIdx.x; q < p.n_lock; q += half * kSmallThreads) {
            const uint32_t t = p.lock_table[q];
            if (t < nv.ntables && nv.table_max[t] > p.lock_snap[q]) small_mark(verdict, vmask, p.lock_txn[q]);
        }
    } else if constexpr (WD > 0) {
        small_appended16<WD>(d, d2, pd, p, verdict, blockIdx.x - half, gridDim.x - half);
    } else {  // the live run and a frozen one (background fold)
        const uint32_t tid = (blockIdx.x - half) * kSmallThreads + threadIdx.x;
        const uint32_t nth = (gridDim.x - half) * kSmallThreads;
        for (uint32_t q = tid; q < p.n; q += nth)
            if ((d.n && delta_hit(d, p, q)) || (d2.n && delta_hit(d2, p, q)))
                mark_verdict<true>(verdict + p.txn[q]);
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's verdict stores are done
    __syncthreads();
    if (threadIdx.x == 0) {
        if (gridDim.x == 1) {  // a lone call: no count to take; packed, the verdicts ride along
            const uint64_t w = (uint64_t)seq << 32 | (packed ? kSmallPacked | vbits : 0u);
            __hip_atomic_store(done, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (__hip_atomic_fetch_add(blocks_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   gridDim.x - 1) {
            // the next launch of this slot counts from zero (stream order)
            __hip_atomic_store(blocks_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, (uint64_t)seq << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

hipError_t launch_small_narrow(const NarrowView &nv, const DeltaView &d, const DeltaView &d2,
                               const PendView &pd, const ProbeView &p,
                               uint8_t *verdict, uint32_t *blocks_done, uint64_t *done,
                               uint32_t seq, bool pack, hipStream_t s)
{
    // one pass of a range per 16-lane group, at most one block per CU (two
    // with appended rows pending: one per half of the grid)
    const bool split = d.n || d2.n || pd.n || pd.nt;
    const size_t per_block = (kSmallThreads / 16) * (split ? kNP : 1);
    const size_t work = std::max<size_t>({(p.n + per_block - 1) / per_block,
                                          (p.n_lock + kSmallThreads - 1) / kSmallThreads, 1});
    const unsigned blocks = (unsigned)(std::min<size_t>(work, 256) * (split ? 2 : 1));
    const int WD = split && nv.W <= kPendMaxWords ? nv.W : 0;
    if ((pd.n || pd.nt) && (WD == 0 || !pd.base || pd.n > kPendRows || pd.nt > kPendRows))
        return hipErrorInvalidValue;  // the host mirrors a tail only for W <= kPendMaxWords
    if ((d.n && d.W != nv.W) || (d2.n && d2.W != nv.W)) return hipErrorInvalidValue;
    const int KW = nv.W == 1 || nv.W == 2 ? nv.W : 0;
#define HSC_SMALL(WD_, KW_)                                                                              \
    k_small_narrow<WD_, KW_><<<blocks, kSmallThreads, 0, s>>>(nv, d, d2, pd, p, verdict, blocks_done, done, \
                                                              seq, pack)
#define HSC_SMALL_KW(WD_)                  \
    do {                                   \
        if (KW == 2)                       \
            HSC_SMALL(WD_, 2);             \
        else if (KW == 1)                  \
            HSC_SMALL(WD_, 1);             \
        else                               \
            HSC_SMALL(WD_, 0);             \
    } while (0)
    switch (WD) {
    case 1: HSC_SMALL_KW(1); break;
    case 2: HSC_SMALL_KW(2); break;
    case 3: HSC_SMALL_KW(3); break;
    case 4: HSC_SMALL_KW(4); break;
    default: HSC_SMALL_KW(0);
    }
#undef HSC_SMALL_KW
#undef HSC_SMALL
    return hipGetLastError();
}

hipError_t launch_probe_narrow(const NarrowView &nv, const ProbeView &p, uint8_t *verdict,
                               hipStream_t s)
{
    if (p.n == 0 && p.n_lock == 0) return hipSuccess;
    const size_t groups = (p.n + kNP - 1) / kNP;
    size_t blocks = (groups + kProbeThreads / 16 - 1) / (kProbeThreads / 16);
    blocks = std::max<size_t>(blocks, (p.n_lock + kProbeThreads - 1) / kProbeThreads);
    blocks = std::min<size_t>(std::max<size_t>(blocks, 1), 256 * 8);
    k_probe_narrow<<<(unsigned)blocks, kProbeThreads, (size_t)nv.lds_entries * 8 + 16, s>>>(
        nv, p, verdict);
    return hipGetLastError();
}

// Probe bounds -> codes (a one-word probe batch for the tile pipeline):
// lo64 = ceil((lo - K0) >> s), hi64 = floor((hi - K0) >> s); a range below
// the window gets lo64 = kSat > hi64 = 0 (empty).
__global__ void k_codes(NarrowView nv, ProbeView p, uint64_t *lo64, uint64_t *hi64)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    const uint32_t g = p.gid[q];
    uint64_t lo = 0, v = 0;
    narrow_bound(nv, g, p.lo + q, p.n, false, lo);
    const bool live = narrow_bound(nv, g, p.hi + q, p.n, true, v);
    lo64[q] = live ? lo : kSat;
    hi64[q] = live ? v : 0;
}

hipError_t narrow_codes(const NarrowView &nv, const ProbeView &p, uint64_t *lo64, uint64_t *hi64,
                        hipStream_t s)
{
    if (p.n == 0) return hipSuccess;
    k_codes<<<(p.n + 255) / 256, 256, 0, s>>>(nv, p, lo64, hi64);
    return hipGetLastError();
}


// ============================================================================
// narrow tiles: 4096-row tiles of (u32 key delta, u32 commit rank)
// ============================================================================
//
// For a dense batch the window is streamed once per batch, tile by tile,
// and the ranges are bucketed by tile (hist matrix + column scan, the plan
// of hsc_kernels.hip).  A row of a tile is 8 bytes:
//
//   key32[i]  = key64[i] - key64[first row of the tile]  (every tile spans
//               < 2^32 codes: checked at build, else the narrow window keeps
//               the code-tile pipeline)
//   rank32[i] = 1 + the index of the row's commit LSN among the window's
//               distinct commit LSNs C (sorted); a snapshot S maps to
//               r(S) = #{c in C : c <= S} and  lsn > S  <=>  rank > r(S).
//
// Join records are 16 bytes: {lo delta, hi delta, r(S), read set}.

__global__ void k_check_sorted(const uint64_t *v, size_t n, uint32_t *flag)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n && v[i] < v[i - 1]) atomicOr(flag, 1u);
}

hipError_t check_sorted_u64(const uint64_t *v, size_t n, uint32_t *flag, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(flag, 0, 4, s);
    if (e != hipSuccess || n < 2) return e;
    k_check_sorted<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(v, n, flag);
    return hipGetLastError();
}

// rank32[i] = 1 + lower_bound(C, lsn[i]) (lsn[i] is in C); pads get 0.
// kRankK rows per thread searched in lockstep over the commit directory,
// whose upper levels are staged in LDS (defined with the locate kernel).
constexpr int kRankThreads = 1024, kRankK = 8;
__host__ __device__ inline uint32_t dir16_lds_entries(const Dir16 &d);
__global__ __launch_bounds__(kRankThreads) void k_rank32(const uint64_t *lsn, uint32_t n,
                                                         uint32_t len, Dir16 d, uint32_t *rank);


// key32 = key64 - first key64 of the tile, stored in the tile's Eytzinger
// order (the join copies a tile's keys into LDS as they lie); flag := 1 if a
// tile spans >= 2^32
__global__ void k_key32(const uint64_t *key64, uint32_t n, uint32_t len, uint32_t *key32,
                        uint32_t *flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const uint32_t dst = (i & ~((1u << kTLog2) - 1)) + eyt12(i & ((1u << kTLog2) - 1));
    if (i >= n) {
        key32[dst] = 0xFFFFFFFFu;
        return;
    }
    const uint64_t d = key64[i] - key64[(size_t)(i >> kTLog2) << kTLog2];
    if (d > 0xFFFFFFFFull) atomicOr(flag, 1u);
    key32[dst] = (uint32_t)d;
}

// lsn32 mode: rank32 = lsn - base + 1 (pads 0)
__global__ void k_rank_lsn32(const uint64_t *lsn, uint32_t n, uint32_t len, uint64_t base,
                             uint32_t *rank)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) rank[i] = i < n ? (uint32_t)(lsn[i] - base) + 1 : 0;
}

hipError_t narrow_tiles_build(const uint64_t *key64, const uint64_t *lsn, uint32_t n, uint32_t len,
                              const Dir16 &cdir, int rank_lsn32, uint64_t rank_base,
                              uint32_t *key32, uint32_t *rank32, uint32_t *flag, hipStream_t s)
{
    if (!flag) {  // (key32 and the flag written by the level pass: the ranks only)
        if (len == 0 || rank_lsn32) return hipSuccess;
    } else {
        hipError_t e = hipMemsetAsync(flag, 0, 4, s);
        if (e != hipSuccess || len == 0) return e;
        k_key32<<<(len + 255) / 256, 256, 0, s>>>(key64, n, len, key32, flag);
    }
    if (rank_lsn32) {
        k_rank_lsn32<<<(len + 255) / 256, 256, 0, s>>>(lsn, n, len, rank_base, rank32);
    } else {
        const uint32_t per = kRankThreads * kRankK;
        k_rank32<<<(len + per - 1) / per, kRankThreads, 8 * dir16_lds_entries(cdir), s>>>(
            lsn, n, len, cdir, rank32);
    }
    return hipGetLastError();
}

// ---- 16-ary directories over sorted u64 arrays ----
__global__ void k_dir_level0(const uint64_t *src, uint32_t n, uint32_t len, uint64_t *dst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) dst[i] = i < n ? src[i] : ~0ull;
}

__global__ void k_dir_up(const uint64_t *src, uint32_t len_src, uint64_t *dst, uint32_t len_dst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len_dst) dst[i] = i < len_src / 16 ? src[16 * (size_t)i + 15] : ~0ull;
}

hipError_t dir16_build(const uint64_t *src, uint32_t n, DBuf &buf, Dir16 &d, uint32_t max_lds,
                       hipStream_t s)
{
    d = Dir16{};
    d.n = n;
    uint32_t len = (n + 16) & ~15u;  // at least one pad: every level ends in ~0
    uint64_t off = 0;
    int L = 0;
    for (;;) {
        if (L == kDirLevels) return hipErrorInvalidValue;
        d.off[L] = (uint32_t)off;
        d.len[L] = len;
        off += len;
        ++L;
        if (len <= 16) break;
        len = ((len / 16) + 15) & ~15u;
    }
    d.levels = L;
    d.lds_from = L - 1;
    d.lds_n = d.len[L - 1];
    while (d.lds_from > 0 && d.lds_n + d.len[d.lds_from - 1] <= max_lds) d.lds_n += d.len[--d.lds_from];
    hipError_t e = buf.ensure(8 * off);
    if (e != hipSuccess) return e;
    uint64_t *v = buf.as<uint64_t>();
    d.v = v;
    k_dir_level0<<<(d.len[0] + 255) / 256, 256, 0, s>>>(src, n, d.len[0], v);
    for (int l = 1; l < L; ++l)
        k_dir_up<<<(d.len[l] + 255) / 256, 256, 0, s>>>(v + d.off[l - 1], d.len[l - 1],
                                                          v + d.off[l], d.len[l]);
    return hipGetLastError();
}

// Upper levels [lds_from, levels) of a directory into LDS, every 16-entry
// block at a 17-entry stride: entry e of block c sits at 17 c + e, so the
// same entry of different blocks falls in different banks (at a 16-entry
// stride entries 3 / 7 / 11 of every block share two of the 64 banks).
constexpr uint32_t kDirLdsStride = 17;
__host__ __device__ inline uint32_t dir16_lds_entries(const Dir16 &d)
{
    return d.lds_n / 16 * kDirLdsStride;
}
__device__ __forceinline__ void dir16_stage(const Dir16 &d, uint64_t *lds)
{
    const uint64_t *src = d.v + d.off[d.lds_from];
    for (uint32_t i = threadIdx.x; i < d.lds_n; i += blockDim.x)
        lds[(i >> 4) * kDirLdsStride + (i & 15)] = src[i];
}

// One level of a 16-ary directory for K keys in lockstep: c[k] (block index
// at this level) becomes 16 c[k] + #{entries of the block below xx[k]}.  Two
// rounds of three independent reads (entries 3, 7, 11 pick the quarter, then
// its first three entries) instead of a 4-step dependent chain.  A block's
// last entry is never below a key (levels end in ~0 padding and a block's last
// entry bounds the key one level up), so the count fits 0..15.
template <int K, uint32_t STRIDE = 16>
__device__ __forceinline__ void dir16_level(const uint64_t *lv, const uint64_t (&xx)[K],
                                            uint32_t (&c)[K])
{
    uint32_t qd[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t *b = lv + STRIDE * c[k];
        qd[k] = (uint32_t)(b[3] < xx[k]) + (uint32_t)(b[7] < xx[k]) + (uint32_t)(b[11] < xx[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t *b = lv + STRIDE * c[k] + 4 * qd[k];
        c[k] = 16 * c[k] + 4 * qd[k] + (uint32_t)(b[0] < xx[k]) + (uint32_t)(b[1] < xx[k]) +
               (uint32_t)(b[2] < xx[k]);
    }
}

// Strict bound for "entries <= x" (entries are < ~0: ~0 is padding).
__device__ __forceinline__ uint64_t dir_le(uint64_t x) { return x >= ~0ull - 1 ? ~0ull : x + 1; }

// out[k] = #{entries < xx[k]} (0 where act[k] is false).  Levels held in LDS
// and levels in global memory run as separate loops so that every read has
// a known address space (no flat loads).
template <int K>
__device__ __forceinline__ void dir16_count(const Dir16 &d, const uint64_t *lds,
                                            const uint64_t (&xx)[K], const bool (&act)[K],
                                            uint32_t (&out)[K])
{
    uint32_t c[K];
#pragma unroll
    for (int k = 0; k < K; ++k) c[k] = 0;
    const uint32_t lds_base = d.off[d.lds_from];
    for (int l = d.levels - 1; l >= d.lds_from; --l)
        dir16_level<K, kDirLdsStride>(lds + (d.off[l] - lds_base) / 16 * kDirLdsStride, xx, c);
    for (int l = d.lds_from - 1; l >= 0; --l) dir16_level<K>(d.v + d.off[l], xx, c);
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] = act[k] ? min(c[k], d.n) : 0;
}

__global__ __launch_bounds__(kRankThreads) void k_rank32(const uint64_t *lsn, uint32_t n,
                                                         uint32_t len, Dir16 d, uint32_t *rank)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t rlds[];
    const uint32_t i0 = blockIdx.x * (kRankThreads * kRankK) + threadIdx.x;
    uint64_t x[kRankK];
    bool act[kRankK];
#pragma unroll
    for (int k = 0; k < kRankK; ++k) {
        const uint32_t i = i0 + k * kRankThreads;
        act[k] = i < n;
        x[k] = act[k] ? lsn[i] : 0;
    }
    dir16_stage(d, rlds);
    __syncthreads();
    uint32_t c[kRankK];
    dir16_count<kRankK>(d, rlds, x, act, c);
#pragma unroll
    for (int k = 0; k < kRankK; ++k) {
        const uint32_t i = i0 + k * kRankThreads;
        if (i < len) rank[i] = act[k] ? c[k] + 1 : 0;
    }
}

// ---- locate: codes, snapshot ranks, end tiles, per-chunk tile histogram ----
// One workgroup per chunk of kLocTP * kLocTThreads probes; thread t owns
// probes c0 + t + kLocTThreads j, j < kLocTP (consecutive lanes =
// consecutive probes, so a read set's ranges sit in neighbouring lanes).
// Every probe load is issued up front; the tile and snapshot-rank searches
// run for all kLocTP probes in lockstep over 16-ary directories whose upper
// levels are staged in LDS (kTileLds: the whole tile directory, so the tile
// search and the tiles' first codes never leave LDS).  Output per probe: its
// first join record {tile << 12 | rank, lo, hi, r(S)} and, for a range that
// spans two tiles, its second one.
#ifndef HSC_LOC_TP
#define HSC_LOC_TP 4
#endif
#ifndef HSC_DIR_LDS
#define HSC_DIR_LDS 4400
#endif
constexpr int kLocTP = HSC_LOC_TP;
#ifndef HSC_LOC_THREADS
#define HSC_LOC_THREADS 1024
#endif
constexpr int kLocTThreads = HSC_LOC_THREADS;  // <= 4096 probes per chunk (in-chunk ranks fit 12 bits)
static_assert(kLocTP * kLocTThreads <= 4096, "in-chunk ranks are 12 bits");
constexpr int kDirLds = HSC_DIR_LDS;  // directory entries staged in LDS per directory

template <int W>
__device__ __forceinline__ void locate_codes(const NarrowView &nv, const ProbeView &p, uint32_t q,
                                             uint64_t g, const uint64_t (&xl)[2 > W ? 2 : W],
                                             const uint64_t (&xh)[2 > W ? 2 : W], uint64_t &lo,
                                             uint64_t &hi)
{
    uint64_t v = 0;
    bool rem;
    uint64_t a = 0;
    bool live;
    if (nv.comp) {  // compressed codes (the loaded words live at p.lo / p.hi + q too)
        narrow_bound(nv, g, p.lo + q, p.n, false, a);
        live = narrow_bound(nv, g, p.hi + q, p.n, true, v);
    } else if constexpr (W > 0) {
        const uint64_t(&wl)[W] = *(const uint64_t(*)[W])xl;
        const uint64_t(&wh)[W] = *(const uint64_t(*)[W])xh;
        a = rel_diff_w<W>(nv.lw, nv.tz, g, wl, nv.base[0], nv.base + 1, kSat, v, rem)
                ? (v >= kSat ? kSat : v + (rem ? 1 : 0))
                : 0;
        live = rel_diff_w<W>(nv.lw, nv.tz, g, wh, nv.base[0], nv.base + 1, kSat, v, rem);
    } else {
        a = rel_diff(nv.W, nv.lw, nv.tz, g, p.lo + q, p.n, nv.base[0], nv.base + 1, 1, kSat, v,
                     rem)
                ? (v >= kSat ? kSat : v + (rem ? 1 : 0))
                : 0;
        live = rel_diff(nv.W, nv.lw, nv.tz, g, p.hi + q, p.n, nv.base[0], nv.base + 1, 1, kSat, v,
                        rem);
    }
    lo = live ? a : kSat;  // a range below the window is empty
    hi = live ? v : 0;
}

// ---- bucket table over the tiles' first codes ----
// first[0] = 0 (codes are relative to the window's first row), so bucket k
// covers codes [k << shift, (k + 1) << shift) with shift the least that puts
// the last tile's first code below m << shift.  trad[k] = #first < k << shift
// for k <= m; trad[m + 1] = shift.
constexpr uint32_t kTradMaxTiles = 4096;   // first codes staged in LDS (32 KiB)
constexpr uint32_t kTradMax = 4096;        // buckets (u16 in LDS: 8 KiB)

uint32_t narrow_trad_buckets(uint32_t ntiles, bool force_dir)
{
    if (force_dir || ntiles == 0 || ntiles > kTradMaxTiles) return 0;  // force_dir: tests
    uint32_t m = 16;
    while (m < 2 * ntiles && m < kTradMax) m *= 2;
    return m;
}

// Log mode (trad[m + 1] = kTradLog | s, m = 64 << s): bucket of x = its
// exponent and s mantissa bits, like a float -- monotone, with the resolution
// where the codes are dense near zero (hot keys of a Zipf window crowd a few
// linear buckets); the build picks the mode whose fullest bucket holds fewer
// tiles (narrow_trad_pick).
__global__ void k_trad(const uint64_t *first, uint32_t ntiles, uint32_t m, int logmode,
                       uint32_t *trad)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m + 1) return;
    const int lg = 31 - __clz(m);
    if (logmode) {
        const int sv = lg - 6;
        if (k == m + 1) {
            trad[k] = kTradLog | (uint32_t)sv;
            return;
        }
        uint32_t lo = 0, hi = ntiles;  // #tiles whose first code's bucket < k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (trad_log_bucket(first[mid], sv) < k)
                lo = mid + 1;
            else
                hi = mid;
        }
        trad[k] = lo;
        return;
    }
    const uint64_t span = first[ntiles - 1];
    const int bits = span ? 64 - __clzll(span) : 0;
    const int shift = bits > lg ? bits - lg : 0;
    if (k == m + 1) {
        trad[k] = (uint32_t)shift;
        return;
    }
    if (k == m) {  // every first code is below m << shift (which overflows when span >= 2^63)
        trad[k] = ntiles;
        return;
    }
    const uint64_t x = (uint64_t)k << shift;
    uint32_t lo = 0, hi = ntiles;  // #first < x
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    trad[k] = lo;
}

hipError_t narrow_trad_build(const uint64_t *first, uint32_t ntiles, uint32_t m, uint32_t *trad,
                             hipStream_t s, int logmode)
{
    if (logmode && m < 64) return hipErrorInvalidValue;
    k_trad<<<(m + 2 + 255) / 256, 256, 0, s>>>(first, ntiles, m, logmode, trad);
    return hipGetLastError();
}

// LDS carve of k_locate_t (same on host and device).  Tile bucket mode:
// first codes [ntiles] + cdir levels + histogram [ntiles] + bucket table u16
// [m + 1] + per-wave snapshot lists; directory mode: tdir levels instead of
// the first codes and no bucket table.
struct LocLds {
    uint32_t first, cdir, hist, trad, sbuf, rbuf, bytes;
};
__host__ __device__ inline LocLds loc_lds(const NarrowTiles &nt, uint32_t ntiles)
{
    LocLds L{};
    uint32_t o = 0;
    L.first = o;
    o += 8 * (nt.trad ? ((ntiles + 1) & ~1u) : dir16_lds_entries(nt.tdir));
    L.cdir = o;
    o += nt.rank_lsn32 ? 0 : 8 * dir16_lds_entries(nt.cdir);
    L.hist = o;
    o += 4 * ((ntiles + 3) & ~3u);
    L.trad = o;
    o += nt.trad ? 2 * ((nt.trad_m + 1 + 7) & ~7u) : 0;
    L.sbuf = o;
    o += 8 * kLocTThreads;
    L.rbuf = o;
    o += 4 * kLocTThreads;
    L.bytes = o;
    return L;
}

// #first < x[k] over the LDS bucket table: bucket, then a binary search
// inside it (typically 0-1 steps; a crowded bucket costs log2 of its size).
template <int K>
__device__ __forceinline__ void trad_count(const uint64_t *first, const uint16_t *T, uint32_t m,
                                           int shift, uint32_t ntiles, const uint64_t (&x)[K],
                                           const bool (&act)[K], uint32_t (&out)[K])
{
    uint32_t l[K], h[K];
    const bool lg = (shift & kTradLog) != 0;
    const int sv = shift & 0xFFFF;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t b = lg ? trad_log_bucket(x[k], sv) : x[k] >> sv;
        const bool in = b < m;
        const uint32_t bi = in ? (uint32_t)b : 0;
        l[k] = in ? T[bi] : ntiles;
        h[k] = in ? T[bi + 1] : ntiles;
    }
    for (;;) {
        bool more = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (l[k] < h[k]) {
                const uint32_t mid = (l[k] + h[k]) >> 1;
                const bool below = first[mid] < x[k];
                l[k] = below ? mid + 1 : l[k];
                h[k] = below ? h[k] : mid;
                more = true;
            }
        }
        if (!more) break;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] = act[k] ? l[k] : 0;
}

// Whole-tile checks of a probe, deferred by one sub-chunk (their sparse-table
// loads then overlap the next sub-chunk's probe loads): tiles [x, y] hold a
// row committed after snap -> read set txn of probe q conflicts.
template <int K>
struct LocDefer {
    uint32_t x[K], y[K], q[K];
    uint64_t snap[K];
};

// W = key words held in registers (1 or 2), 0 = read from memory (any W).
// The chunk's kLocTP probes per thread run as kLocTP / kLocSub sub-chunks of
// kLocSub probes per thread: the loads of sub-chunk s + 1 are in flight while
// sub-chunk s is located (codes, snapshot ranks, end tiles, records), so the
// chunk's HBM reads overlap its LDS / VALU work instead of preceding it.
#ifndef HSC_LOC_SUB  // (r02, chunk-sorted records: 1 probe per sub-chunk 2.10 G vs 2 probes 2.00 G)
#define HSC_LOC_SUB 1
#endif
constexpr int kLocSub = HSC_LOC_SUB;
#ifndef HSC_LOC_WPE
#define HSC_LOC_ATTR
#else  // A/B builds: hold the locate to HSC_LOC_WPE waves per SIMD
#define HSC_LOC_ATTR __attribute__((amdgpu_waves_per_eu(HSC_LOC_WPE, HSC_LOC_WPE)))
#endif
static_assert(kLocTP % kLocSub == 0, "whole sub-chunks");
template <int W, bool kTrad>
__global__ __launch_bounds__(kLocTThreads) HSC_LOC_ATTR void k_locate_t(NarrowView nv, WinView wt,
                                                             ProbeView p, ProbeWork work,
                                                             NarrowTiles nt, uint8_t *verdict)
{
    constexpr int WR = 2 > W ? 2 : W;
    constexpr int K = kLocSub, S = kLocTP / kLocSub;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds64[];
    const uint32_t ntiles = wt.ntiles;
    const LocLds L = loc_lds(nt, ntiles);
    char *lb = (char *)lds64;
    uint64_t *tfirst = (uint64_t *)(lb + L.first);  // first codes (kTrad) / tdir levels
    uint64_t *cdir = (uint64_t *)(lb + L.cdir);
    uint32_t *hist = (uint32_t *)(lb + L.hist);
    uint16_t *T = (uint16_t *)(lb + L.trad);
    const int lane = threadIdx.x & 63;
    uint64_t *sb = (uint64_t *)(lb + L.sbuf) + (threadIdx.x & ~63u);
    uint32_t *rb = (uint32_t *)(lb + L.rbuf) + (threadIdx.x & ~63u);
    const uint32_t g = xcd_chunk(blockIdx.x, (work.G + 7) / 8);
    if (g >= work.G) return;
    HSC_STAMP(work, 0, 0);
    if (g == 0 && threadIdx.x < 3) work.item_off[threadIdx.x] = 0;  // the plan's / join's counters
    const uint32_t c0 = g * work.chunk;
    const uint32_t c1 = min(p.n, c0 + work.chunk);
    // probe registers: buffer 0 / 1 alternate between sub-chunks (the loop
    // below is unrolled, so every index is a compile-time constant)
    uint32_t qq[2][K], gg[2][K], tx[2][K];
    bool valid[2][K];
    uint64_t snap[2][K], xl[2][K][WR], xh[2][K][WR];
    // the chunk's records stay in registers until its histogram is complete,
    // then go to their tile-sorted places in the chunk's area
    uint4 R0[S][K], R1[S][K];
    uint32_t RT[S][K];
    uint64_t SS[S][K];  // ranks through the commit directory: the snapshots, ranked after the loop
    auto load = [&](int s, int buf) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = s * K + k;
            qq[buf][k] = c0 + threadIdx.x + kLocTThreads * j;
            valid[buf][k] = qq[buf][k] < c1;
            const uint32_t q = valid[buf][k] ? qq[buf][k] : 0;
            // read-once inputs: non-temporal, so they do not push the window's
            // rows out of the caches between batches
            gg[buf][k] = p.n ? __builtin_nontemporal_load(p.gid + q) : 0;
            snap[buf][k] = p.n ? __builtin_nontemporal_load(p.snap + q) : 0;
            tx[buf][k] = p.n ? __builtin_nontemporal_load(p.txn + q) : 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                xl[buf][k][w] = p.n ? __builtin_nontemporal_load(p.lo + (size_t)w * p.n + q) : 0;
                xh[buf][k][w] = p.n ? __builtin_nontemporal_load(p.hi + (size_t)w * p.n + q) : 0;
            }
        }
    };
    load(0, 0);
    int tshift = 0;
    if constexpr (kTrad) {
        const u64x2 *src = (const u64x2 *)wt.sp_w;
        for (uint32_t i = threadIdx.x; i < ntiles / 2; i += kLocTThreads)
            ((u64x2 *)tfirst)[i] = src[i];
        if ((ntiles & 1) && threadIdx.x == 0) tfirst[ntiles - 1] = wt.sp_w[ntiles - 1];
        for (uint32_t i = threadIdx.x; i <= nt.trad_m; i += kLocTThreads) T[i] = (uint16_t)nt.trad[i];
        tshift = (int)nt.trad[nt.trad_m + 1];
    } else {
        dir16_stage(nt.tdir, tfirst);
    }
    if (!nt.rank_lsn32) dir16_stage(nt.cdir, cdir);
    for (uint32_t i = threadIdx.x; i < ntiles; i += kLocTThreads) hist[i] = 0;
    __syncthreads();  // directories staged, histogram zeroed
    HSC_STAMP(work, 0, 1);
    const uint64_t *first = kTrad ? tfirst : wt.sp_w;  // first code of every tile
    LocDefer<K> dfr;
#pragma unroll
    for (int k = 0; k < K; ++k) dfr.x[k] = 1, dfr.y[k] = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int cb = s & 1;
        // 1. the previous sub-chunk's whole-tile checks: their loads are
        //    younger than this sub-chunk's probe loads, which are needed now;
        //    they are compared at the end of this sub-chunk (the loads
        //    overlap its LDS work; the read sets are in registers)
        uint64_t pm[K], psn[K];
        if (s > 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pm[k] = dfr.x[k] <= dfr.y[k] ? tiles_max(wt, dfr.x[k], dfr.y[k]) : 0;
                psn[k] = dfr.snap[k];
            }
        }
        // 2. the next sub-chunk's probe loads stay in flight through step 3
        if (s + 1 < S) load(s + 1, cb ^ 1);
        // 3. locate this sub-chunk from registers and LDS
        uint64_t lo[K], hi[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            locate_codes<W>(nv, p, valid[cb][k] ? qq[cb][k] : 0, gg[cb][k], xl[cb][k], xh[cb][k],
                            lo[k], hi[k]);
        // Snapshot ranks r(S): O(1) when the window spans < 2^32 of log, else
        // #commits <= S through the commit directory; a run of equal
        // snapshots in neighbouring lanes (a read set's ranges) has one head,
        // the wave packs its heads into a list and searches each once.
        uint32_t rs[K];
        if (nt.rank_lsn32) {
#pragma unroll
            for (int k = 0; k < K; ++k) rs[k] = lsn32_rank(snap[cb][k], nt.rank_base);
        } else {
            // the records stay in registers: every sub-chunk's heads are
            // searched together after the loop (one directory walk, not S)
#pragma unroll
            for (int k = 0; k < K; ++k) rs[k] = 0, SS[s][k] = snap[cb][k];
        }
        // end tiles: a = #first < lo - 1 (the tile holding the first row >=
        // lo), bt = #first <= hi - 1 (the tile holding the last row <= hi)
        uint32_t cnt[2 * K];
        {
            uint64_t keys[2 * K];
            bool act[2 * K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                keys[2 * k] = lo[k];
                keys[2 * k + 1] = dir_le(hi[k]);
                act[2 * k] = act[2 * k + 1] = valid[cb][k] && lo[k] <= hi[k];
            }
            if constexpr (kTrad)
                trad_count<2 * K>(tfirst, T, nt.trad_m, tshift, ntiles, keys, act, cnt);
            else
                dir16_count<2 * K>(nt.tdir, tfirst, keys, act, cnt);
        }
        // records of the partly covered end tiles; the fully covered tiles
        // between them (and fully covered end tiles) become one deferred
        // range-maximum check [x, y]
#pragma unroll
        for (int k = 0; k < K; ++k) {
            dfr.x[k] = 1, dfr.y[k] = 0;
            R0[s][k].x = R1[s][k].x = kNoTile32;
            RT[s][k] = tx[cb][k];
            if (!valid[cb][k]) continue;
            const uint32_t q = qq[cb][k];
            const uint32_t ca = cnt[2 * k], cbt = cnt[2 * k + 1];
            const uint32_t a = ca ? ca - 1 : 0;
            const uint32_t bt = cbt ? cbt - 1 : 0;
            uint4 r0 = make_uint4(kNoTile32, 0, 0, 0), r1 = r0;
            if (cbt > 0 && a <= bt && lo[k] <= hi[k]) {
                // tile-relative bounds
                const uint64_t fa = first[a], fb = first[bt];
                const uint64_t lo_a = lo[k] <= fa ? 0 : lo[k] - fa;  // > 2^32-1: none
                const uint64_t hi_a = a == bt ? (hi[k] < fa ? ~0ull : hi[k] - fa) : 0xFFFFFFFFull;
                const uint64_t hi_b = hi[k] < fb ? ~0ull : hi[k] - fb;
                const bool full_a = lo_a == 0 && (a < bt || hi_a >= 0xFFFFFFFFull);
                const bool use_a = lo_a <= 0xFFFFFFFFull && hi_a != ~0ull && lo_a <= hi_a;
                const bool use_b = a < bt && hi_b != ~0ull;
                const bool full_b = hi_b >= 0xFFFFFFFFull;
                dfr.x[k] = use_a && full_a ? a : a + 1;
                dfr.y[k] = a == bt ? (use_a && full_a ? a : 0) : (use_b && full_b ? bt : bt - 1);
                if (a == bt && !(use_a && full_a)) dfr.x[k] = 1, dfr.y[k] = 0;
                dfr.q[k] = q;
                dfr.snap[k] = snap[cb][k];
                if (use_a && !full_a)
                    r0 = make_uint4(a << 12 | atomicAdd(&hist[a], 1u), (uint32_t)lo_a,
                                    (uint32_t)min(hi_a, 0xFFFFFFFFull), rs[k]);
                if (use_b && !full_b)
                    r1 = make_uint4(bt << 12 | atomicAdd(&hist[bt], 1u), 0, (uint32_t)hi_b, rs[k]);
            }
            R0[s][k] = r0;
            R1[s][k] = r1;
        }
        if (s > 0) {  // step 1's compares (pm = 0 where there was no check)
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (pm[k] > psn[k]) verdict[RT[s - 1][k]] = 1;
        }
    }
    // the last sub-chunk's range-maximum loads are issued here and compared
    // after the tail (scan, row and record stores), which they overlap
    uint64_t dmax[K];
#pragma unroll
    for (int k = 0; k < K; ++k) dmax[k] = dfr.x[k] <= dfr.y[k] ? tiles_max(wt, dfr.x[k], dfr.y[k]) : 0;
    {
        if (!nt.rank_lsn32) {  // the chunk's snapshot ranks: heads of all sub-chunks in one list
            const uint64_t le_mask = lane == 63 ? ~0ull : ((2ull << lane) - 1);
            bool head[S][K];
            uint32_t slot[S][K];
            uint32_t H = 0;
#pragma unroll
            for (int s = 0; s < S; ++s)
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const uint64_t prev = __shfl_up(SS[s][k], 1, 64);
                    head[s][k] = lane == 0 || prev != SS[s][k];
                    const uint64_t m = __ballot(head[s][k]);
                    slot[s][k] = H + __popcll(m & le_mask) - 1;  // this lane's head
                    H += __popcll(m);
                }
            for (uint32_t b0 = 0; b0 < H; b0 += 64) {
#pragma unroll
                for (int s = 0; s < S; ++s)
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (head[s][k] && slot[s][k] - b0 < 64) sb[slot[s][k] - b0] = SS[s][k];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const bool act[1] = {lane < H - b0};
                const uint64_t xs[1] = {act[0] ? dir_le(sb[lane]) : 0};
                uint32_t r[1];
                dir16_count<1>(nt.cdir, cdir, xs, act, r);
                rb[lane] = r[0];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int s = 0; s < S; ++s)
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (slot[s][k] - b0 < 64) R0[s][k].w = R1[s][k].w = rb[slot[s][k] - b0];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
    HSC_STAMP(work, 0, 2);
    // table locks: any write to a locked table after the snapshot
    for (uint32_t q = g * kLocTThreads + threadIdx.x; q < p.n_lock; q += work.G * kLocTThreads) {
        const uint32_t t = p.lock_table[q];
        if (t < wt.ntables && wt.table_max[t] > p.lock_snap[q]) verdict[p.lock_txn[q]] = 1;
    }
    __syncthreads();
    HSC_STAMP(work, 0, 3);
    // column g of the tile-major histogram (neighbouring chunks of a line are
    // written from the same XCD)
    {
        // exclusive scan of the chunk's tile counts (thread = a run of
        // consecutive tiles): row g of the chunk-major table gets (run start
        // << 16 | count) per tile (contiguous stores; the plan transposes),
        // the runs' starts replace the counts in LDS
        const uint32_t per = (ntiles + kLocTThreads - 1) / kLocTThreads;
        const uint32_t i0 = min(ntiles, threadIdx.x * per), i1 = min(ntiles, i0 + per);
        uint32_t sum = 0;
        for (uint32_t i = i0; i < i1; ++i) sum += hist[i];
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        uint32_t *wtot = (uint32_t *)(lb + L.rbuf);
        if (lane == 63) wtot[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t run = x - sum;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) run += wtot[w];
        uint32_t *row = work.cm + (size_t)g * ((ntiles + 3) & ~3u);
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t c = hist[i];
            row[i] = run << 16 | c;
            hist[i] = run;
            run += c;
        }
        __syncthreads();
        HSC_STAMP(work, 0, 4);
        uint4 *area = nt.recs + (size_t)g * 2 * work.chunk;
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint4 a = R0[s][k], b = R1[s][k];
                if (a.x != kNoTile32)
                    area[hist[a.x >> 12] + (a.x & 0xFFFu)] = make_uint4(a.y, a.z, a.w, RT[s][k]);
                if (b.x != kNoTile32)
                    area[hist[b.x >> 12] + (b.x & 0xFFFu)] = make_uint4(b.y, b.z, b.w, RT[s][k]);
            }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (dfr.x[k] <= dfr.y[k] && dmax[k] > dfr.snap[k]) verdict[RT[S - 1][k]] = 1;
    }
    HSC_STAMP(work, 0, 5);
}

hipError_t launch_locate_t(const NarrowView &nv, const WinView &wt, const ProbeView &p,
                           const ProbeWork &work, const NarrowTiles &nt, uint8_t *verdict,
                           hipStream_t s)
{
    if (p.n == 0 && p.n_lock == 0) return hipSuccess;
    const size_t lds = loc_lds(nt, wt.ntiles).bytes;
    const bool tr = nt.trad != nullptr;
    const int w = nv.W == 1 || nv.W == 2 ? nv.W : 0;
#define HSC_LOCATE(W_, TR_) \
    k_locate_t<W_, TR_><<<8 * ((work.G + 7) / 8), kLocTThreads, lds, s>>>(nv, wt, p, work, nt, verdict)
    if (w == 1 && tr)
        HSC_LOCATE(1, true);
    else if (w == 1)
        HSC_LOCATE(1, false);
    else if (w == 2 && tr)
        HSC_LOCATE(2, true);
    else if (w == 2)
        HSC_LOCATE(2, false);
    else if (tr)
        HSC_LOCATE(0, true);
    else
        HSC_LOCATE(0, false);
#undef HSC_LOCATE
    return hipGetLastError();
}

// probes per locate workgroup, directory entries staged in LDS
uint32_t narrow_tiles_chunk() { return kLocTP * kLocTThreads; }
uint32_t narrow_tiles_dir_lds() { return kDirLds; }

// ---- plan ----
// ctl[1] (extra join items) was zeroed by this batch's locate.
// Plan of chunk-sorted records: block = 8 tiles (HSC_PLAN_S_THREADS / 64).
// The block reads the tiles' entries of every chunk row of the locate's
// chunk-major table (32 contiguous bytes per row), transposes them through LDS, and wave w scans
// tile t0 + w's column as k_plan_t does; it writes the tile-major exclusive
// offsets (hist) and run starts (cst) the join stages, the tile's count and,
// for a hot tile, join items over its own record numbers.  The verdict pack
// is folded in as in k_plan_t.
// 512 threads (8 tiles, 32-byte row pieces) vs 1024 (16 tiles, 64-byte
// pieces): one stream 62.1 vs 61.1 us, two streams 2.22 vs 2.17 G checks/s
// (r02d) -- the headline is the two-stream number
#ifndef HSC_PLAN_S_THREADS
#define HSC_PLAN_S_THREADS 512
#endif
constexpr int kPlanSThreads = HSC_PLAN_S_THREADS;  // a wave per tile
__global__ __launch_bounds__(kPlanSThreads) void k_plan_s(ProbeWork work, uint32_t ntiles,
                                                          uint32_t *ctl, uint8_t *flags,
                                                          uint32_t n_txn, uint8_t *verdict)
{
    constexpr int TB = kPlanSThreads / 64;  // tiles per block
    static_assert(TB % 4 == 0, "16-byte row pieces");
    constexpr uint32_t SR = kMaxChunks + 4;
    __shared__ __attribute__((aligned(16))) uint32_t sh[TB][SR];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t t0 = blockIdx.x * TB, t = t0 + w;
    const uint32_t G = work.G, hs = hist_stride(G), rs = (ntiles + 3) & ~3u;
    // (g, piece) pairs: TB / 4 16-byte pieces of every chunk row
    for (uint32_t i = threadIdx.x; i < G * (TB / 4); i += kPlanSThreads) {
        const uint32_t g = i / (TB / 4), pc = i % (TB / 4);
        const uint32_t c = t0 + 4 * pc;
        const u32x4 a = c < rs ? *(const u32x4 *)(work.cm + (size_t)g * rs + c) : u32x4{0, 0, 0, 0};
        sh[4 * pc][g] = a.x, sh[4 * pc + 1][g] = a.y, sh[4 * pc + 2][g] = a.z, sh[4 * pc + 3][g] = a.w;
    }
    if (verdict) {
        // (a wave covers 64 consecutive read sets, 64-aligned: one bitmap word)
        const uint32_t stride = gridDim.x * kPlanSThreads;
        for (uint32_t i = blockIdx.x * kPlanSThreads + threadIdx.x; i < n_txn; i += stride) {
            const uint8_t f = flags[i];
            verdict[i] = f != 0;
            if (f) flags[i] = 0;
            const uint64_t m = __ballot(f != 0);
            if (work.bitmap && lane == 0) work.bitmap[i >> 6] = m;
        }
    }
    __syncthreads();
    if (t >= ntiles) return;
    const uint32_t e = 8 * lane;
    uint32_t v[8], c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t x = e + k < G ? sh[w][e + k] : 0;
        v[k] = x & 0xFFFFu;
        c[k] = x >> 16;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += v[k];
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    uint32_t run = x - sum;
    if (e < hs) {
        u32x4 oa, ob;
        oa.x = run; run += v[0];
        oa.y = run; run += v[1];
        oa.z = run; run += v[2];
        oa.w = run; run += v[3];
        ob.x = run; run += v[4];
        ob.y = run; run += v[5];
        ob.z = run; run += v[6];
        ob.w = run;
        u32x4 *col = (u32x4 *)(work.hist + (size_t)t * hs);
        col[e / 4] = oa;
        col[e / 4 + 1] = ob;
        *(u32x4 *)(work.cst + (size_t)t * hs + e) =
            u32x4{c[0] | c[1] << 16, c[2] | c[3] << 16, c[4] | c[5] << 16, c[6] | c[7] << 16};
    }
    const uint32_t total = __shfl(x, 63, 64);
    if (lane == 0) work.counts[t] = total;
    if (total > kTileCap) {  // hot tile: join items over its record numbers past kTileCap
        const uint32_t over = total - kTileCap;
        const uint32_t nx = (over + kJoinChunk - 1) / kJoinChunk;
        uint32_t ib = 0;
        if (lane == 0) ib = atomicAdd(&ctl[1], nx);
        ib = __shfl(ib, 0, 64);
        for (uint32_t j = lane; j < nx; j += 64)
            work.item_desc[ib + j] = make_uint4(t, kTileCap + j * kJoinChunk,
                                                kTileCap + min((j + 1) * kJoinChunk, over), 0);
    }
}

hipError_t launch_plan_s(const ProbeWork &work, uint32_t ntiles, uint32_t *ctl, hipStream_t s,
                         uint8_t *flags, uint32_t n_txn, uint8_t *verdict)
{
    if (ntiles == 0) return hipSuccess;
    constexpr uint32_t per = kPlanSThreads / 64;
    k_plan_s<<<(ntiles + per - 1) / per, kPlanSThreads, 0, s>>>(work, ntiles, ctl, flags, n_txn,
                                                                verdict);
    return hipGetLastError();
}

// ---- join: 8-byte rows ----
// Row quad v of thread t = rows 4 (t + kJoinThreads v) .. + 3: one 16-byte
// load of keys (already in Eytzinger order, k_key32) and one of ranks per
// quad, stored to LDS as they are; 16-row maxima over 4 lanes, 128-row maxima
// over 32 lanes.

// The join is held to 8 waves per SIMD: at 85-99 SGPRs the hardware admits
// only 6-7 (measured on config 2: join 34 -> 31.7 us, one stream 71.3 -> 69 us)
#ifndef HSC_JOIN_WPE
#define HSC_JOIN_WPE 8
#endif
#define HSC_JOIN_ATTR __attribute__((amdgpu_waves_per_eu(HSC_JOIN_WPE, HSC_JOIN_WPE)))
// Chunk-sorted records: record j of tile t lives in the
// run of the chunk g whose offset inside the tile (the plan's scan of column
// t) is the last one <= j, at chunk g's area + cst[t][g] + (j - that offset).
// The tile's column is staged first (its loads ahead of the rows'), each
// thread finds its records' chunks by a 9-step search of it in LDS and issues
// the record loads while the rows are still arriving.
template <bool kTile>
__device__ __forceinline__ void join_s_item(const ProbeWork &work, const NarrowTiles &nt,
                                            uint32_t n, uint32_t xi, uint8_t *verdict,
                                            uint32_t *keys, uint32_t *rank, uint32_t *b16,
                                            uint32_t *b128, uint32_t *Es, uint32_t *Cs)
{
    constexpr uint32_t T = 1u << kTLog2;
    constexpr int RQ = T / (4 * kJoinThreads);
    constexpr int kRec = kJoinChunk / kJoinThreads;
    static_assert(kMaxChunks <= kJoinThreads, "one column entry per thread");
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
    if (threadIdx.x < G) {
        e = work.hist[col + threadIdx.x];
        cs = work.cst[col + threadIdx.x];
    }
    u32x4 rk[RQ], rr[RQ], rec[kRec];
    const size_t ts = (size_t)tile << kTLog2;
#pragma unroll
    for (int v = 0; v < RQ; ++v) {
        const size_t row = ts + 4 * (threadIdx.x + kJoinThreads * v);
        rk[v] = *(const u32x4 *)(nt.key32 + row);
        rr[v] = *(const u32x4 *)(nt.rank32 + row);
    }
    if constexpr (kTile) j1 = min(kTileCap, sload(work.counts + tile));
    if (threadIdx.x < G) Es[threadIdx.x] = e, Cs[threadIdx.x] = cs;
    __syncthreads();
    HSC_STAMP(work, 1, 1);
    const size_t area = 2 * (size_t)work.chunk;
#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t j = j0 + k * kJoinThreads + threadIdx.x;
        uint32_t g = 0;  // Es[0] = 0 <= j
#pragma unroll
        for (int b = 8; b >= 0; --b) {
            const uint32_t c = g + (1u << b);
            if (c < G && Es[c] <= j) g = c;
        }
        rec[k] = j < j1 ? *(const u32x4 *)(nt.recs + g * area + Cs[g] + (j - Es[g]))
                        : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int v = 0; v < RQ; ++v) {
        const uint32_t quad = threadIdx.x + kJoinThreads * v;
        ((u32x4 *)keys)[quad] = rk[v];
        ((u32x4 *)rank)[quad] = rr[v];
        uint32_t m = max(max(rr[v].x, rr[v].y), max(rr[v].z, rr[v].w));
        m = max(m, (uint32_t)__shfl_xor((int)m, 1, 64));
        m = max(m, (uint32_t)__shfl_xor((int)m, 2, 64));
        if ((threadIdx.x & 3) == 0) b16[quad >> 2] = m;
#pragma unroll
        for (int d = 4; d < 32; d <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
        if ((threadIdx.x & 31) == 0) b128[quad >> 5] = m;
    }
    __syncthreads();
    HSC_STAMP(work, 1, 2);
    const uint32_t tn = min(T, n - (tile << kTLog2));
#pragma unroll
    for (int k = 0; k < kRec; ++k) {
        const uint32_t j = j0 + k * kJoinThreads + threadIdx.x;
        if (j >= j1) continue;
        const uint32_t lo = rec[k].x, hi = rec[k].y, rs = rec[k].z;
        uint32_t ja = 1, jb = 1;
#pragma unroll
        for (int d = 0; d < kTLog2; ++d) {
            const uint32_t ka = keys[ja], kb = keys[jb];
            ja = 2 * ja + (ka < lo);
            jb = 2 * jb + (kb <= hi);
        }
        const uint32_t kl = keys[0];
        const uint32_t pa = min(ja - T + (kl < lo), tn);
        const uint32_t pb = min(jb - T + (kl <= hi), tn);
        if (pa < pb && any_after32(rank, b16, b128, pa, pb, rs)) {
            // (r05w, world-1 per-rank step: these atomics 50.7 / 51.9 us per
            // step, guarded by a read of the verdict byte 53.3 / 52.5, the
            // pack pass instead 52.7 / 51.9 -- the same within the spread)
            verdict[rec[k].w] = 1;
            if (work.bitmap)
                atomicOr((unsigned long long *)&work.bitmap[rec[k].w >> 6], 1ull << (rec[k].w & 63));
        }
    }
}

#ifndef HSC_JOIN_XCD  // (r02c: config 2 2.09 -> 2.16 G checks/s, join 31.7 -> 29.6 us)
#define HSC_JOIN_XCD 1
#endif
constexpr bool kJoinXcd = HSC_JOIN_XCD != 0;
__host__ __device__ inline uint32_t join_tile_blocks(uint32_t ntiles)
{
    return kJoinXcd ? 8 * ((ntiles + 7) / 8) : ntiles;
}

__global__ __launch_bounds__(kJoinThreads) HSC_JOIN_ATTR void k_join_t(ProbeWork work, NarrowTiles nt,
                                                         uint32_t n, uint32_t ntiles,
                                                         uint8_t *verdict)
{
    constexpr uint32_t T = 1u << kTLog2;
    __shared__ __attribute__((aligned(16))) uint32_t keys[T];
    __shared__ __attribute__((aligned(16))) uint32_t rank[T];
    __shared__ uint32_t b16[T / 16];
    __shared__ uint32_t b128[T / 128];
    __shared__ uint32_t Es[kMaxChunks], Cs[kMaxChunks];

    HSC_STAMP(work, 1, 0);
    // chunk-sorted records: neighbouring tiles on one XCD (their runs of a
    // chunk share lines of its record area, which that XCD's L2 then serves)
    const uint32_t tb = join_tile_blocks(ntiles);
    if (blockIdx.x < tb) {
        const uint32_t tile = kJoinXcd ? xcd_chunk(blockIdx.x, tb / 8) : blockIdx.x;
        if (tile < ntiles) join_s_item<true>(work, nt, n, tile, verdict, keys, rank, b16, b128, Es, Cs);
    } else {  // blocks past the tiles take the hot tiles' overflow items in turn
        const uint32_t nextra = work.item_off[1];
        const uint32_t stride = gridDim.x - tb;
        for (uint32_t xi = blockIdx.x - tb; xi < nextra; xi += stride) {
            __syncthreads();  // the previous item's LDS reads are done
            join_s_item<false>(work, nt, n, xi, verdict, keys, rank, b16, b128, Es, Cs);
        }
    }
    HSC_STAMP(work, 1, 3);
}

hipError_t launch_join_t(const ProbeWork &work, const NarrowTiles &nt, uint32_t n,
                         uint32_t ntiles, uint32_t max_items, uint8_t *verdict, hipStream_t s,
                         uint32_t extra_blocks)
{
    if (max_items == 0 || n == 0 || ntiles == 0) return hipSuccess;
    // one block per tile + up to extra_blocks blocks looping over the
    // overflow items (measured: one block per tile beats persistent blocks
    // that prefetch their next tile -- 27.8 vs 32 us on config 2)
    const uint32_t blocks = join_tile_blocks(ntiles) + std::min<uint32_t>(max_items - ntiles, extra_blocks);
    k_join_t<<<blocks, kJoinThreads, 0, s>>>(work, nt, n, ntiles, verdict);
    return hipGetLastError();
}

// Verdict bytes of the batch from the conflict flags the probe kernels set
// (an internal array, so nothing has to clear the caller's buffer first):
// verdict[t] = flag, bitmap bit t = flag (one ballot per 64 transactions), and
// set flags are cleared for the next batch.
__global__ void k_pack_flags(uint8_t *flags, uint32_t n, uint8_t *verdict, uint64_t *bitmap)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool v = t < n && flags[t] != 0;
    if (t < n) verdict[t] = v;
    if (v) flags[t] = 0;
    const uint64_t m = __ballot(v);
    if (bitmap && (threadIdx.x & 63) == 0 && t < n) bitmap[t >> 6] = m;
}

hipError_t launch_pack_flags(uint8_t *flags, uint32_t n_txn, uint8_t *verdict, uint64_t *bitmap,
                             hipStream_t s)
{
    if (n_txn == 0) return hipSuccess;
    k_pack_flags<<<(n_txn + 255) / 256, 256, 0, s>>>(flags, n_txn, verdict, bitmap);
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_narrow()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_end_rows);
}

}  // namespace hsc
