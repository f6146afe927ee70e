// hsc_compact.hip -- compact codes for wide windows (composite keys, config 3).
//
// Within one (table, index, key length) group every window row agrees with
// the group's first row on most key bits (constant field bytes, the 0x08
// field headers, the unused bits of small integers, the zero padding of
// short strings).  Dropping the bit positions that never vary inside a
// group keeps the memcmp order of its rows (the order is decided by the
// first differing bit, which is always a varying one), so each row becomes a
// shorter code: bits_g varying bits, most significant first, left-aligned in
// WC = floor(max bits_g / 64) + 1 words (at least one spare bit: all-ones is
// above every code).  Config 3's 9..58-byte keys (W = 8 words) become WC = 3.
//
// A probe bound X (W words, padded per the reference's min-length memcmp:
// 0x00 for lo, 0xFF for hi) maps exactly onto the codes.  Let p be the first
// constant position where X differs from the group pattern C, and prefix =
// X's varying bits before p (np of them).  For every row r: if r's first np
// code bits differ from prefix they decide; if equal, r agrees with X up to
// p and bit p decides: r < X iff X_p = 1.  Hence
//   #rows < X  = #codes < lo'   lo' = code(X) (no p), prefix+1 then 0s
//                               (X_p = 1; overflow: X above every row),
//                               prefix then 0s (X_p = 0)
//   #rows <= X = #codes <= hi'  hi' = code(X) (no p), prefix then 1s (X_p =
//                               1), prefix-1 then 1s (X_p = 0; prefix = 0:
//                               X below every row)
// A range whose lo is above every row or whose hi is below every row (or
// whose group has no rows) matches nothing and becomes (lo' = ~0, hi' = 0).
// The window's row order, group spans, dedupe and LSNs are unchanged, so the
// wide tile pipeline (hsc_kernels.hip) runs on the codes as it does on keys.
//
// Bits are gathered with Hacker's Delight's parallel-suffix compress; its
// six move masks per (group, word) depend only on the mask and are built on
// the host (compact_tables).
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

namespace hsc {

namespace {

__device__ __forceinline__ uint64_t compress(uint64_t x, uint64_t m, const uint64_t *mv)
{
    x &= m;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const uint64_t t = x & mv[i];
        x = (x ^ t) | (t >> (1 << i));
    }
    return x;
}

// append the c low bits of v at bit position pos (MSB-first) of out[WC]
template <int WC>
__device__ __forceinline__ void put_bits(uint64_t (&out)[WC], int pos, uint64_t v, int c)
{
    if (c == 0) return;
    const int w = pos >> 6, off = pos & 63;
    if (off + c <= 64) {
        const int sh = 64 - off - c;
#pragma unroll
        for (int k = 0; k < WC; ++k)
            if (k == w) out[k] |= v << sh;
    } else {
        const int hi = off + c - 64;  // bits spilling into word w + 1
#pragma unroll
        for (int k = 0; k < WC; ++k) {
            if (k == w) out[k] |= v >> hi;
            if (k == w + 1) out[k] |= v << (64 - hi);
        }
    }
}

// add (+1) or subtract (-1) one unit at bit position pos (MSB-first) of the
// WC-word big number; returns true on carry / borrow out of the top
template <int WC>
__device__ __forceinline__ bool step_at(uint64_t (&out)[WC], int pos, int dir)
{
    const int w = pos >> 6;
    uint64_t unit = 1ull << (63 - (pos & 63));
    bool carry = false;
#pragma unroll
    for (int k = WC - 1; k >= 0; --k) {
        if (k > w) continue;
        if (k < w && !carry) break;
        const uint64_t add = k == w ? unit : 1ull;
        if (dir > 0) {
            const uint64_t r = out[k] + add;
            carry = r < out[k];
            out[k] = r;
        } else {
            carry = out[k] < add;
            out[k] -= add;
        }
        if (!carry) break;
    }
    return carry;
}

// set bits [from, to) (MSB-first) to one
template <int WC>
__device__ __forceinline__ void fill_ones(uint64_t (&out)[WC], int from, int to)
{
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        const int a = max(from, 64 * k), b = min(to, 64 * k + 64);
        if (a >= b) continue;
        const int lo = a - 64 * k, n = b - a;  // bits lo..lo+n-1 of word k from its MSB
        const uint64_t ones = n == 64 ? ~0ull : ((1ull << n) - 1) << (64 - lo - n);
        out[k] |= ones;
    }
}

struct CompactMeta {
    const uint64_t *mask, *pat, *mv;  // [ng][W], [ng][W], [ng][W][6]
    const uint32_t *bits;             // [ng]: varying bits, kNoRows = group has no rows
    const uint32_t *wlen;             // [ng]: words inside the group's key length
    int W, ng;
};
constexpr uint32_t kNoRows = 0xFFFFFFFFu;

// code of X in group g; kind 0 = exact row, 1 = lo bound, 2 = hi bound.
// Returns false if the bound puts the range outside the group's rows.
template <int WC>
__device__ bool code_of(const CompactMeta &cm, uint32_t g, const uint64_t *x, size_t xs, int kind,
                        uint64_t (&out)[WC])
{
#pragma unroll
    for (int k = 0; k < WC; ++k) out[k] = 0;
    const uint32_t bits = cm.bits[g];
    if (bits == kNoRows) return false;
    const uint64_t *mk = cm.mask + (size_t)g * cm.W, *pt = cm.pat + (size_t)g * cm.W;
    const uint64_t *mv = cm.mv + (size_t)g * cm.W * 6;
    int pos = 0, np = -1, xb = 0;
    for (int j = 0; j < cm.W; ++j) {
        const uint64_t m = mk[j];
        const int c = __popcll(m);
        if (np < 0) {
            const uint64_t xj = x[(size_t)j * xs];
            const uint64_t d = kind ? (xj ^ pt[j]) & ~m : 0;
            if (d) {
                const int b = 63 - __clzll(d);
                const uint64_t above = b == 63 ? 0 : ~0ull << (b + 1);
                put_bits(out, pos, compress(xj & above, m, mv + 6 * j), c);
                np = pos + __popcll(m & above);
                xb = (int)((xj >> b) & 1);
            } else {
                put_bits(out, pos, compress(xj, m, mv + 6 * j), c);
            }
        }
        pos += c;
    }
    if (np < 0) return true;  // X agrees with the pattern: its code is exact
    if (kind == 1) {
        if (xb && (np == 0 || step_at(out, np - 1, +1))) return false;  // above every row
        return true;
    }
    if (!xb) {
        if (np == 0) return false;
        bool zero = true;
#pragma unroll
        for (int k = 0; k < WC; ++k) zero &= out[k] == 0;
        if (zero) return false;  // below every row
        step_at(out, np - 1, -1);
    }
    fill_ones(out, np, (int)bits);
    return true;
}

// Rows are sorted by group: each thread ORs (row XOR the group's first row)
// over kVaryRows consecutive rows and flushes only when the group changes,
// and a wave whose lanes end in one group combines them first, so the
// atomics per (group, word) stay few (one per row made them contend).
constexpr int kVaryRows = 16;
__global__ __launch_bounds__(256) void k_group_vary(const uint64_t *words, size_t stride,
                                                    const uint32_t *gid, uint32_t n, int W,
                                                    const uint32_t *gstart, uint64_t *mask)
{
    const size_t base = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * kVaryRows;
    if (__shfl(base, 0) >= n) return;  // the whole wave is past the end
    const bool valid = base < n;
    const uint32_t end = valid ? (uint32_t)min((size_t)n, base + kVaryRows) : 0;
    for (int j = 0; j < W; ++j) {
        const uint64_t *wj = words + (size_t)j * stride;
        uint32_t cg = valid ? gid[base] : 0xFFFFFFFFu;
        uint64_t f = valid ? wj[gstart[cg]] : 0, acc = 0;
        for (uint32_t i = (uint32_t)base; i < end; ++i) {
            const uint32_t g = gid[i];
            if (g != cg) {
                if (acc) atomicOr((unsigned long long *)&mask[(size_t)cg * W + j], acc);
                cg = g;
                f = wj[gstart[g]];
                acc = 0;
            }
            acc |= wj[i] ^ f;
        }
        const uint32_t cg0 = __shfl(cg, 0);
        if (__all(!valid || cg == cg0)) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) acc |= __shfl_xor(acc, o);
            if (lane_id() == 0 && acc) atomicOr((unsigned long long *)&mask[(size_t)cg0 * W + j], acc);
        } else if (valid && acc) {
            atomicOr((unsigned long long *)&mask[(size_t)cg * W + j], acc);
        }
    }
}

__global__ void k_group_pattern(const uint64_t *words, size_t stride, int W, int ng,
                                const uint32_t *gstart, const uint32_t *gend, uint64_t *pat)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    const bool rows = gend[g] > gstart[g];
    for (int j = 0; j < W; ++j) pat[(size_t)g * W + j] = rows ? words[(size_t)j * stride + gstart[g]] : 0;
}

template <int WC>
__global__ __launch_bounds__(256) void k_compact_rows(const uint64_t *words, size_t stride,
                                                      const uint32_t *gid, uint32_t n,
                                                      CompactMeta cm, uint64_t *cw)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t out[WC];
    code_of<WC>(cm, gid[i], words + i, stride, 0, out);
#pragma unroll
    for (int k = 0; k < WC; ++k) cw[(size_t)k * stride + i] = out[k];
}

template <int WC>
__global__ __launch_bounds__(256) void k_compact_probes(ProbeView p, CompactMeta cm, uint64_t *clo,
                                                        uint64_t *chi)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    const uint32_t g = p.gid[q];
    uint64_t lo[WC], hi[WC];
    bool ok = code_of<WC>(cm, g, p.lo + q, p.n, 1, lo);
    ok = ok && code_of<WC>(cm, g, p.hi + q, p.n, 2, hi);
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        clo[(size_t)k * p.n + q] = ok ? lo[k] : ~0ull;
        chi[(size_t)k * p.n + q] = ok ? hi[k] : 0;
    }
}

// ---- probe bounds, keys of at most kProbeWords words ----
// The same mapping as code_of, for lo and hi of one probe in one pass over
// the group's masks, with every operand in registers: the key words are all
// loaded first, each word's compressed bits are shifted into a right-aligned
// accumulator (no indexing of the code by a run-time word number, which
// would put it in scratch), and the code is left-aligned at the end.
constexpr int kProbeWords = 8;

// a = a << c | v (0 <= c <= 64, v < 2^c) over a WC-word big number
template <int WC>
__device__ __forceinline__ void acc_push(uint64_t (&a)[WC], uint64_t v, int c)
{
#pragma unroll
    for (int k = 0; k < WC - 1; ++k) {
        const uint64_t hi = c >= 64 ? 0 : a[k] << c;
        const uint64_t lo = c == 0 ? 0 : a[k + 1] >> (64 - c);
        a[k] = hi | lo;
    }
    a[WC - 1] = (c >= 64 ? 0 : a[WC - 1] << c) | v;
}

// left-align the low `bits` bits of a (bits <= 64 WC)
template <int WC>
__device__ __forceinline__ void acc_align(uint64_t (&a)[WC], int bits)
{
    const int s = 64 * WC - bits, ws = s >> 6, bs = s & 63;
    uint64_t t[WC];
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        uint64_t v = 0;
#pragma unroll
        for (int m = k; m < WC; ++m) v = m == k + ws ? a[m] : v;
        t[k] = v;
    }
    acc_push<WC>(t, 0, bs);
#pragma unroll
    for (int k = 0; k < WC; ++k) a[k] = t[k];
}

// +- one unit at bit pos (MSB-first); true on carry / borrow out of the top
template <int WC>
__device__ __forceinline__ bool unit_step(uint64_t (&o)[WC], int pos, bool add)
{
    const int w = pos >> 6;
    const uint64_t bit = 1ull << (63 - (pos & 63));
    bool carry = false;
#pragma unroll
    for (int k = WC - 1; k >= 0; --k) {
        const uint64_t u = k == w ? bit : (k < w && carry ? 1ull : 0ull);
        if (add) {
            const uint64_t r = o[k] + u;
            carry = r < o[k];
            o[k] = r;
        } else {
            carry = o[k] < u;
            o[k] -= u;
        }
    }
    return carry;
}

// one word of a bound: compressed bits, and the first constant position
// where x leaves the pattern (np, xb) if not found yet
__device__ __forceinline__ uint64_t bound_word(uint64_t x, uint64_t m, uint64_t pt,
                                               const uint64_t (&mv)[6], int pos, int &np, int &xb)
{
    if (np >= 0) return 0;
    const uint64_t d = (x ^ pt) & ~m;
    if (d) {
        const int b = 63 - __clzll(d);
        const uint64_t above = b == 63 ? 0 : ~0ull << (b + 1);
        np = pos + __popcll(m & above);
        xb = (int)((x >> b) & 1);
        x &= above;
    }
    x &= m;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const uint64_t t = x & mv[i];
        x = (x ^ t) | (t >> (1 << i));
    }
    return x;
}

// Per-group tables staged in LDS when they fit (config 3: 32 groups x 8
// words = 16 KiB): the lanes of a wave read different groups' masks, which
// from global memory are gathers.  A thread maps P probes, the next probe's
// key words loading while the current one is mapped (the first ones load
// before the tables are staged).
constexpr int kBoundThreads = 256;
constexpr uint32_t kBoundLdsBytes = 48 * 1024;
__host__ __device__ inline uint32_t bound_lds_bytes(int ng, int W)
{
    return (uint32_t)ng * (uint32_t)W * 8 * 8 + 8 * (uint32_t)ng;
}

struct BoundIn {
    uint32_t g;
    uint64_t xl[kProbeWords], xh[kProbeWords];
};

// Words past the group's key length are zero in every bound and row (the
// marshal pads with zeros), so they are neither loaded nor mapped; the
// marshal groups a batch's probes by that length, so whole waves skip them.
__device__ __forceinline__ void bound_load(const ProbeView &p, const CompactMeta &cm, uint32_t q,
                                           BoundIn &in)
{
    const bool v = q < p.n;
    in.g = v ? p.gid[q] : 0;
    const int wl = v ? (int)cm.wlen[in.g] : 0;
#pragma unroll
    for (int j = 0; j < kProbeWords; ++j) {
        const bool u = v && j < wl;
        in.xl[j] = u ? __builtin_nontemporal_load(p.lo + (size_t)j * p.n + q) : 0;
        in.xh[j] = u ? __builtin_nontemporal_load(p.hi + (size_t)j * p.n + q) : 0;
    }
}

template <int WC>
__device__ __forceinline__ void bound_map(const ProbeView &p, const CompactMeta &cm, uint32_t q,
                                          const BoundIn &in, uint64_t *clo, uint64_t *chi)
{
    const uint32_t g = in.g;
    const uint32_t bits = cm.bits[g];
    uint64_t al[WC], ah[WC];
#pragma unroll
    for (int k = 0; k < WC; ++k) al[k] = ah[k] = 0;
    bool ok = bits != kNoRows;
    if (ok) {
        const uint64_t *mk = cm.mask + (size_t)g * cm.W, *pt = cm.pat + (size_t)g * cm.W;
        const uint64_t *mvg = cm.mv + (size_t)g * cm.W * 6;
        const int wl = (int)cm.wlen[g];
        int pos = 0, npl = -1, nph = -1, xbl = 0, xbh = 0;
#pragma unroll
        for (int j = 0; j < kProbeWords; ++j) {
            if (j >= wl) break;  // past the key length: zero bound, zero mask
            const uint64_t m = mk[j], pj = pt[j];
            uint64_t mv[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) mv[i] = mvg[6 * j + i];
            const int c = __popcll(m);
            acc_push<WC>(al, bound_word(in.xl[j], m, pj, mv, pos, npl, xbl), c);
            acc_push<WC>(ah, bound_word(in.xh[j], m, pj, mv, pos, nph, xbh), c);
            pos += c;
        }
        acc_align<WC>(al, pos);
        acc_align<WC>(ah, pos);
        // lo: #rows < X = #codes < lo'
        if (npl >= 0 && xbl && (npl == 0 || unit_step<WC>(al, npl - 1, true))) ok = false;
        // hi: #rows <= X = #codes <= hi'
        if (nph >= 0) {
            if (!xbh) {
                bool zero = true;
#pragma unroll
                for (int k = 0; k < WC; ++k) zero &= ah[k] == 0;
                if (nph == 0 || zero)
                    ok = false;
                else
                    unit_step<WC>(ah, nph - 1, false);
            }
            fill_ones<WC>(ah, nph, (int)bits);
        }
    }
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        clo[(size_t)k * p.n + q] = ok ? al[k] : ~0ull;
        chi[(size_t)k * p.n + q] = ok ? ah[k] : 0;
    }
}

template <int WC, bool kLds, int P>
__global__ __launch_bounds__(kBoundThreads) void k_compact_bounds(ProbeView p, CompactMeta cm,
                                                                  uint64_t *clo, uint64_t *chi)
{
    const uint32_t q0 = blockIdx.x * (kBoundThreads * P) + threadIdx.x;
    BoundIn cur;
    bound_load(p, cm, q0, cur);
    if constexpr (kLds) {
        extern __shared__ __attribute__((aligned(16))) uint64_t blds[];
        const uint32_t gw = (uint32_t)cm.ng * cm.W;
        uint64_t *lm = blds, *lp = blds + gw, *lv = blds + 2 * gw;
        uint32_t *lb = (uint32_t *)(blds + 8 * gw), *lw = lb + cm.ng;
        for (uint32_t i = threadIdx.x; i < gw; i += kBoundThreads) {
            lm[i] = cm.mask[i];
            lp[i] = cm.pat[i];
        }
        for (uint32_t i = threadIdx.x; i < 6 * gw; i += kBoundThreads) lv[i] = cm.mv[i];
        for (uint32_t i = threadIdx.x; i < (uint32_t)cm.ng; i += kBoundThreads) {
            lb[i] = cm.bits[i];
            lw[i] = cm.wlen[i];
        }
        __syncthreads();
        cm.mask = lm;
        cm.pat = lp;
        cm.mv = lv;
        cm.bits = lb;
        cm.wlen = lw;
    }
#pragma unroll 1
    for (int j = 0; j < P; ++j) {
        const uint32_t q = q0 + j * kBoundThreads;
        if (q >= p.n) break;
        BoundIn nxt;
        if (j + 1 < P) bound_load(p, cm, q + kBoundThreads, nxt);
        bound_map<WC>(p, cm, q, cur, clo, chi);
        if (j + 1 < P) cur = nxt;
    }
}

template <int WC>
hipError_t launch_rows_wc(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                          const CompactMeta &cm, uint64_t *cw, hipStream_t s)
{
    k_compact_rows<WC><<<(n + 255) / 256, 256, 0, s>>>(words, stride, gid, n, cm, cw);
    return hipGetLastError();
}

template <int WC>
hipError_t launch_probes_wc(const ProbeView &p, const CompactMeta &cm, uint64_t *clo,
                            uint64_t *chi, hipStream_t s)
{
    static const bool generic = getenv("HSC_COMPACT_GENERIC") != nullptr;  // tests: old kernel
    if (cm.W <= kProbeWords && !generic) {
        static const int P = getenv("HSC_BOUND_P") ? atoi(getenv("HSC_BOUND_P")) : 2;  // A/B knob
        const uint32_t per = kBoundThreads * (P == 1 ? 1 : P == 4 ? 4 : 2);
        const uint32_t blocks = (p.n + per - 1) / per;
        const bool in_lds = bound_lds_bytes(cm.ng, cm.W) <= kBoundLdsBytes;
        const uint32_t lds = in_lds ? bound_lds_bytes(cm.ng, cm.W) : 0;
#define HSC_BOUNDS(L_, P_) k_compact_bounds<WC, L_, P_><<<blocks, kBoundThreads, lds, s>>>(p, cm, clo, chi)
        if (in_lds)
            P == 1 ? HSC_BOUNDS(true, 1) : P == 4 ? HSC_BOUNDS(true, 4) : HSC_BOUNDS(true, 2);
        else
            P == 1 ? HSC_BOUNDS(false, 1) : P == 4 ? HSC_BOUNDS(false, 4) : HSC_BOUNDS(false, 2);
#undef HSC_BOUNDS
    } else
        k_compact_probes<WC><<<(p.n + 255) / 256, 256, 0, s>>>(p, cm, clo, chi);
    return hipGetLastError();
}

CompactMeta meta_of(const CompactTables &t)
{
    return CompactMeta{t.mask, t.pat, t.mv, t.bits, t.wlen, t.W, t.ng};
}

}  // namespace

// Hacker's Delight compress move masks of m (host).
void compress_moves(uint64_t m, uint64_t mv[6])
{
    uint64_t mk = ~m << 1;
    for (int i = 0; i < 6; ++i) {
        uint64_t mp = mk ^ (mk << 1);
        mp ^= mp << 2;
        mp ^= mp << 4;
        mp ^= mp << 8;
        mp ^= mp << 16;
        mp ^= mp << 32;
        const uint64_t v = mp & m;
        mv[i] = v;
        m = (m ^ v) | (v >> (1 << i));
        mk &= ~mp;
    }
}

hipError_t compact_masks(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                         int W, int ng, const uint32_t *gstart, const uint32_t *gend,
                         uint64_t *mask, uint64_t *pat, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(mask, 0, 8 * (size_t)ng * W, s);
    if (e != hipSuccess) return e;
    const uint32_t per = 256 * kVaryRows;
    if (n) k_group_vary<<<(n + per - 1) / per, 256, 0, s>>>(words, stride, gid, n, W, gstart, mask);
    if (ng) k_group_pattern<<<(ng + 63) / 64, 64, 0, s>>>(words, stride, W, ng, gstart, gend, pat);
    return hipGetLastError();
}

hipError_t compact_rows(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                        const CompactTables &t, uint64_t *cw, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    const CompactMeta cm = meta_of(t);
    switch (t.WC) {
    case 1: return launch_rows_wc<1>(words, stride, gid, n, cm, cw, s);
    case 2: return launch_rows_wc<2>(words, stride, gid, n, cm, cw, s);
    case 3: return launch_rows_wc<3>(words, stride, gid, n, cm, cw, s);
    case 4: return launch_rows_wc<4>(words, stride, gid, n, cm, cw, s);
    case 5: return launch_rows_wc<5>(words, stride, gid, n, cm, cw, s);
    case 6: return launch_rows_wc<6>(words, stride, gid, n, cm, cw, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t compact_probes(const ProbeView &p, const CompactTables &t, uint64_t *clo, uint64_t *chi,
                          hipStream_t s)
{
    if (p.n == 0) return hipSuccess;
    const CompactMeta cm = meta_of(t);
    switch (t.WC) {
    case 1: return launch_probes_wc<1>(p, cm, clo, chi, s);
    case 2: return launch_probes_wc<2>(p, cm, clo, chi, s);
    case 3: return launch_probes_wc<3>(p, cm, clo, chi, s);
    case 4: return launch_probes_wc<4>(p, cm, clo, chi, s);
    case 5: return launch_probes_wc<5>(p, cm, clo, chi, s);
    case 6: return launch_probes_wc<6>(p, cm, clo, chi, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace hsc
