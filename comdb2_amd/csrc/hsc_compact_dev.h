// hsc_compact_dev.h -- device side of the compact codes (hsc_compact.hip):
// the Hacker's Delight compress, the per-group tables, and the mapping of a
// probe's lo / hi bounds onto code bounds, shared by the bound kernel and the
// compact tiles' fused locate (hsc_ctiles.hip).  Everything here is inline.
#pragma once
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

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
    const uint64_t *mask, *pat, *mv;  // mask / pattern of word j of group g at [g * gs + j],
                                      // compress move i at mv[(g * gs + j) * vm + i * vs]
    const uint32_t *bits;             // [ng]: varying bits, kNoRows = group has no rows
    const uint32_t *wlen;             // [ng]: words inside the group's key length
    int W, ng;
    int gs, vm, vs;                   // global: W, 6, 1 ([ng][W][6]); LDS (stage_bound_tables):
                                      // odd gs, 1, ng * gs -- lanes of different groups hit
                                      // different banks
};
constexpr uint32_t kNoRows = 0xFFFFFFFFu;

// code of X in group g; kind 0 = exact row, 1 = lo bound, 2 = hi bound.
// Returns false if the bound puts the range outside the group's rows.
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
    return (uint32_t)ng * (uint32_t)(W | 1) * 8 * 8 + 8 * (uint32_t)ng;
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

// lo and hi of one probe as code bounds al / ah (false: the range misses its
// group's rows)
template <int WC>
__device__ __forceinline__ bool bound_codes(const CompactMeta &cm, const BoundIn &in,
                                            uint64_t (&al)[WC], uint64_t (&ah)[WC])
{
    const uint32_t g = in.g;
    const uint32_t bits = cm.bits[g];
#pragma unroll
    for (int k = 0; k < WC; ++k) al[k] = ah[k] = 0;
    // a wave of points (lo == hi in every lane: the marshal lays a length's
    // points out together) maps one bound for both; lo and hi differ only in
    // the adjustments after the loop
    bool pt = true;
#pragma unroll
    for (int j = 0; j < kProbeWords; ++j) pt &= in.xl[j] == in.xh[j];
    const bool wpt = __all(pt);
    bool ok = bits != kNoRows;
    if (ok) {
        const uint64_t *mk = cm.mask + (size_t)g * cm.gs, *pt = cm.pat + (size_t)g * cm.gs;
        const uint64_t *mvg = cm.mv + (size_t)g * cm.gs * cm.vm;
        const int wl = (int)cm.wlen[g];
        int pos = 0, npl = -1, nph = -1, xbl = 0, xbh = 0;
#pragma unroll
        for (int j = 0; j < kProbeWords; ++j) {
            if (j >= wl) break;  // past the key length: zero bound, zero mask
            const uint64_t m = mk[j], pj = pt[j];
            uint64_t mv[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) mv[i] = mvg[j * cm.vm + i * cm.vs];
            const int c = __popcll(m);
            const uint64_t vl = bound_word(in.xl[j], m, pj, mv, pos, npl, xbl);
            acc_push<WC>(al, vl, c);
            uint64_t vh = vl;
            if (!wpt) vh = bound_word(in.xh[j], m, pj, mv, pos, nph, xbh);
            acc_push<WC>(ah, vh, c);
            pos += c;
        }
        if (wpt) nph = npl, xbh = xbl;
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
    return ok;
}

template <int WC>
__device__ __forceinline__ void bound_map(const ProbeView &p, const CompactMeta &cm, uint32_t q,
                                          const BoundIn &in, uint64_t *clo, uint64_t *chi)
{
    uint64_t al[WC], ah[WC];
    const bool ok = bound_codes<WC>(cm, in, al, ah);
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        clo[(size_t)k * p.n + q] = ok ? al[k] : ~0ull;
        chi[(size_t)k * p.n + q] = ok ? ah[k] : 0;
    }
}

// The bound tables of cm into LDS at blds (bound_lds_bytes(ng, W)); cm then
// points at them.  Callers synchronize before use.
template <int NT>
__device__ __forceinline__ void stage_bound_tables(CompactMeta &cm, uint64_t *blds)
{
    const uint32_t W = (uint32_t)cm.W, gs = W | 1, gw = (uint32_t)cm.ng * gs;
    uint64_t *lm = blds, *lp = blds + gw, *lv = blds + 2 * gw;
    uint32_t *lb = (uint32_t *)(blds + 8 * gw), *lw = lb + cm.ng;
    for (uint32_t i = threadIdx.x; i < (uint32_t)cm.ng * W; i += NT) {
        const uint32_t g = i / W, j = i - g * W;
        lm[g * gs + j] = cm.mask[i];
        lp[g * gs + j] = cm.pat[i];
    }
    for (uint32_t i = threadIdx.x; i < 6 * (uint32_t)cm.ng * W; i += NT) {
        const uint32_t gj = i / 6, k = i - 6 * gj, g = gj / W, j = gj - g * W;
        lv[k * gw + g * gs + j] = cm.mv[i];
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)cm.ng; i += NT) {
        lb[i] = cm.bits[i];
        lw[i] = cm.wlen[i];
    }
    cm.mask = lm;
    cm.pat = lp;
    cm.mv = lv;
    cm.bits = lb;
    cm.wlen = lw;
    cm.gs = (int)gs;
    cm.vm = 1;
    cm.vs = (int)gw;
}

}  // namespace
}  // namespace hsc
