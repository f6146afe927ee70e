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
__global__ void k_end_rows(WinView w, uint64_t *out)
{
    const int j = threadIdx.x;
    if (j > w.W) return;
    const size_t r[2] = {0, (size_t)w.n - 1};
    for (int k = 0; k < 2; ++k)
        out[k * (w.W + 1) + j] = j ? w.words[(size_t)(j - 1) * w.stride + r[k]] : w.gid[r[k]];
}

hipError_t narrow_end_rows(const WinView &w, uint64_t *out, hipStream_t s)
{
    k_end_rows<<<1, 128, 0, s>>>(w, out);
    return hipGetLastError();
}

// level 0: key64 of every row (padding above n), lsn (padding 0)
__global__ void k_level0(WinView w, const uint64_t *base, int lw, int tz, uint32_t len,
                         uint64_t *key0, uint64_t *max0)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    uint64_t v = kKeyPad, m = 0;
    if (i < w.n) {
        bool rem;
        rel_diff(w.W, lw, tz, w.gid[i], w.words + i, w.stride, base[0], base + 1, 1, kSat, v, rem);
        m = w.lsn[i];
    }
    key0[i] = v;
    max0[i] = m;
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

hipError_t narrow_build(const WinView &w, const NarrowView &nv, hipStream_t s)
{
    const uint32_t len0 = nv.len[0];
    k_level0<<<(len0 + 255) / 256, 256, 0, s>>>(w, nv.base, nv.lw, nv.tz, len0,
                                                 (uint64_t *)nv.keys, (uint64_t *)nv.maxs);
    for (int l = 1; l < nv.levels; ++l)
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

__global__ __launch_bounds__(kProbeThreads) void k_probe_narrow(NarrowView nv, ProbeView p,
                                                                uint8_t *verdict)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t top[];  // levels >= lds_from
    const uint64_t lds_base = nv.off[nv.lds_from];
    for (uint32_t i = threadIdx.x; i < nv.lds_entries; i += kProbeThreads)
        top[i] = nv.keys[lds_base + i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int sub = lane >> 4, l16 = lane & 15;
    const uint32_t groups = gridDim.x * (kProbeThreads / 16);
    const size_t ks = p.n;
    // every wave runs the same number of iterations (ballots need all lanes)
    const uint32_t wave0 = (blockIdx.x * (kProbeThreads / 16) + ((threadIdx.x >> 6) << 2)) * kNP;
    for (uint32_t wbase = wave0; wbase < p.n; wbase += groups * kNP) {
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
                uint64_t v;
                bool rem;
                // lower bound: ceil((lo - K0) >> s), 0 below the window
                mlo = rel_diff(nv.W, nv.lw, nv.tz, g, p.lo + q, ks, nv.base[0], nv.base + 1, 1,
                               kSat, v, rem)
                          ? (v >= kSat ? kSat : v + (rem ? 1 : 0))
                          : 0;
                // upper bound: floor((hi - K0) >> s); none below the window
                mlive = rel_diff(nv.W, nv.lw, nv.tz, g, p.hi + q, ks, nv.base[0], nv.base + 1, 1,
                                 kSat, v, rem);
                mhi = mlive ? v : 0;
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
            if (l >= nv.lds_from) {
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
                if (found[k]) verdict[txn[k]] = 1;
        }
    }
    // table locks: any write to a locked table after the snapshot
    for (uint32_t q = blockIdx.x * kProbeThreads + threadIdx.x; q < p.n_lock;
         q += gridDim.x * kProbeThreads) {
        const uint32_t t = p.lock_table[q];
        if (t < nv.ntables && nv.table_max[t] > p.lock_snap[q]) verdict[p.lock_txn[q]] = 1;
    }
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
    uint64_t v;
    bool rem;
    const uint64_t lo = rel_diff(nv.W, nv.lw, nv.tz, g, p.lo + q, p.n, nv.base[0], nv.base + 1, 1,
                                 kSat, v, rem)
                            ? (v >= kSat ? kSat : v + (rem ? 1 : 0))
                            : 0;
    const bool live = rel_diff(nv.W, nv.lw, nv.tz, g, p.hi + q, p.n, nv.base[0], nv.base + 1, 1,
                               kSat, v, rem);
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

}  // namespace hsc
