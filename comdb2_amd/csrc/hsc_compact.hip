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
#include "hsc_compact_dev.h"
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

namespace hsc {

namespace {

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

// ---- exact-key index for point probes (PointHash, hsc_internal.h) ----
__device__ __forceinline__ uint64_t ph_mix(uint64_t k0, uint64_t k1, uint64_t k2)
{
    uint64_t h = k0 * 0x9E3779B97F4A7C15ull;
    h ^= (k1 + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= (k2 + 0x165667B19E3779F9ull) * 0xD6E8FEB86659FD93ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 29);
}

// the tiles' key of code c in group g (hsc_ctiles.hip compose), 3 words with
// the words past WG zero
template <int WC>
__device__ __forceinline__ void ph_key(uint32_t g, int gb, int WG, const uint64_t (&c)[WC], uint64_t (&k)[3])
{
    uint64_t x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = j < WC ? c[j < WC ? j : 0] : 0;
    if (gb == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) k[j] = x[j];
    } else {
        k[0] = ((uint64_t)g << (64 - gb)) | (x[0] >> gb);
        k[1] = (x[0] << (64 - gb)) | (x[1] >> gb);
        k[2] = (x[1] << (64 - gb)) | (x[2] >> gb);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) k[j] = j < WG ? k[j] : 0;
}

// rank of key k in the index (false: not a window key).  A bucket is one
// 128-byte line of four entries; a lookup reads its home line and goes on
// only past a full one
__device__ __forceinline__ bool ph_find(const PointHash &ph, const uint64_t (&k)[3], uint32_t &rank)
{
    uint64_t b = __umul64hi(ph_mix(k[0], k[1], k[2]), ph.nb);
    for (uint64_t it = 0; it < ph.nb; ++it) {
        const u64x2 *e = (const u64x2 *)(ph.e + 16 * b);
        u64x2 x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = e[q];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const u64x2 a0 = x[2 * s], a1 = x[2 * s + 1];
            if ((a1.y >> 40) != ph.ep) return false;  // empty: a slot of an older build
            if (a0.x == k[0] && a0.y == k[1] && a1.x == k[2]) {
                rank = (uint32_t)a1.y;
                return true;
            }
        }
        b = b + 1 == ph.nb ? 0 : b + 1;
    }
    return false;
}

// one thread per window key: claim a slot by its rank word (ep << 40 | 1 <<
// 32 | rank; a slot whose epoch is not this build's is empty, so a rebuild
// needs no clearing pass), then write the key words
__global__ __launch_bounds__(256) void k_ph_insert(CTiles ct, uint64_t *e, uint64_t nb, uint32_t ep)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ct.n) return;
    uint64_t k[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) k[j] = j < ct.WG ? ct.key[(size_t)j * ct.len + i] : 0;
    const unsigned long long r = (unsigned long long)ct.rank[i] | (1ull << 32) | ((unsigned long long)ep << 40);
    uint64_t b = __umul64hi(ph_mix(k[0], k[1], k[2]), nb);
    for (uint64_t it = 0; it < nb; ++it) {
        for (int s = 0; s < 4; ++s) {
            unsigned long long *w = (unsigned long long *)(e + 16 * b + 4 * s + 3);
            unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while ((cur >> 40) != ep) {  // empty this build: claim it
                const unsigned long long was = atomicCAS(w, cur, r);
                if (was == cur) {
                    uint64_t *x = e + 16 * b + 4 * s;
                    x[0] = k[0], x[1] = k[1], x[2] = k[2];
                    return;
                }
                cur = was;  // another key took it (or its epoch moved): look again
            }
        }
        b = b + 1 == nb ? 0 : b + 1;
    }
}

template <int WC, bool kLds>
__global__ __launch_bounds__(kBoundThreads) void k_compact_bounds(ProbeView p, CompactMeta cm,
                                                                  uint64_t *clo, uint64_t *chi,
                                                                  PointHash ph)
{
    const uint32_t q = blockIdx.x * kBoundThreads + threadIdx.x;
    BoundIn cur;
    bound_load(p, cm, q, cur);
    uint64_t snap = 0;
    uint32_t txn = 0;
    if (ph.nb && q < p.n) snap = p.snap[q], txn = p.txn[q];  // (used by points only)
    if constexpr (kLds) {
        extern __shared__ __attribute__((aligned(16))) uint64_t blds[];
        stage_bound_tables<kBoundThreads>(cm, blds);
        __syncthreads();
    }
    if (q >= p.n) return;
    if constexpr (WC <= 3) {
        if (ph.nb) {
            uint64_t al[WC], ah[WC];
            const bool ok = bound_codes<WC>(cm, cur, al, ah);
            bool point = ok;
#pragma unroll
            for (int k = 0; k < WC; ++k) point &= al[k] == ah[k];
            if (point) {  // answered here: an empty code range for the locate
                uint64_t key[3];
                ph_key<WC>(cur.g, ph.gb, ph.WG, al, key);
                uint32_t rk = 0;
                if (ph_find(ph, key, rk) && rk > lsn32_rank(snap, ph.rank_base)) ph.flags[txn] = 1;
                clo[q] = ~0ull;  // word 0 decides: lo above hi whatever the others hold
                chi[q] = 0;
                return;
            }
#pragma unroll
            for (int k = 0; k < WC; ++k) {
                clo[(size_t)k * p.n + q] = ok ? al[k] : ~0ull;
                chi[(size_t)k * p.n + q] = ok ? ah[k] : 0;
            }
            return;
        }
    }
    bound_map<WC>(p, cm, q, cur, clo, chi);
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
                            uint64_t *chi, hipStream_t s, const PointHash &ph)
{
    // (r02: one probe per thread beat 2 and 4 in flight on config 3)
    if (cm.W <= kProbeWords) {
        // (measured on config 3, r05: 1024-thread blocks staging the tables
        // once per 1024 probes 60.7 vs 59.0 us with the locate; the tables read
        // in place, no LDS, 79.7 us)
        const uint32_t blocks = (p.n + kBoundThreads - 1) / kBoundThreads;
        const bool in_lds = bound_lds_bytes(cm.ng, cm.W) <= kBoundLdsBytes;
        const uint32_t lds = in_lds ? bound_lds_bytes(cm.ng, cm.W) : 0;
        if (in_lds)
            k_compact_bounds<WC, true><<<blocks, kBoundThreads, lds, s>>>(p, cm, clo, chi, ph);
        else
            k_compact_bounds<WC, false><<<blocks, kBoundThreads, lds, s>>>(p, cm, clo, chi, ph);
    } else
        k_compact_probes<WC><<<(p.n + 255) / 256, 256, 0, s>>>(p, cm, clo, chi);
    return hipGetLastError();
}

CompactMeta meta_of(const CompactTables &t)
{
    return CompactMeta{t.mask, t.pat, t.mv, t.bits, t.wlen, t.W, t.ng, t.W, 6, 1};
}

// ---- compact tables of unsorted rows, sort keys, unpack (hsc_csort.hip) ----
// rep[g] = the smallest row index of group g (rep preset to ~0): a workgroup
// takes the minimum of its kCsRepRows rows per group in LDS, then one global
// atomic per group it saw (one atomic per row on a few dozen group words
// serialised the whole pass)
constexpr int kCsRepRows = 8192;
__global__ __launch_bounds__(256) void k_cs_rep(const uint32_t *gid, uint32_t n, int ng, uint32_t *rep)
{
    extern __shared__ uint32_t rl[];
    for (int g = threadIdx.x; g < ng; g += blockDim.x) rl[g] = 0xFFFFFFFFu;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kCsRepRows;
    for (uint32_t r = threadIdx.x; r < (uint32_t)kCsRepRows; r += blockDim.x) {
        const size_t i = base + r;
        if (i >= n) break;
        const uint32_t g = gid[i];
        if ((uint32_t)i < rl[g]) atomicMin(&rl[g], (uint32_t)i);
    }
    __syncthreads();
    for (int g = threadIdx.x; g < ng; g += blockDim.x)
        if (rl[g] != 0xFFFFFFFFu) atomicMin(&rep[g], rl[g]);
}

// pat[g][j] = word j of group g's representative row (0 for a group without rows)
__global__ void k_cs_pat(const uint64_t *words, size_t stride, int W, int ng, const uint32_t *rep,
                         uint64_t *pat)
{
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (uint32_t)(ng * W)) return;
    const uint32_t g = e / W, j = e - g * W, r = rep[g];
    pat[e] = r != 0xFFFFFFFFu ? words[(size_t)j * stride + r] : 0;
}

// mask[g][j] |= row XOR pattern over unsorted rows: a workgroup ORs its rows
// into LDS accumulators (one 64-bit LDS atomic per nonzero word), then one
// global atomic per nonzero accumulator
constexpr int kCsVaryRows = 4096;
__global__ __launch_bounds__(256) void k_cs_vary(const uint64_t *words, size_t stride, const uint32_t *gid,
                                                 uint32_t n, int W, int ng, const uint64_t *pat,
                                                 uint64_t *mask)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t cl[];  // [ng W] pattern, [ng W] acc
    const uint32_t gw = (uint32_t)(ng * W);
    uint64_t *pl = cl, *acc = cl + gw;
    for (uint32_t e = threadIdx.x; e < gw; e += blockDim.x) pl[e] = pat[e], acc[e] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kCsVaryRows;
    for (uint32_t r = threadIdx.x; r < (uint32_t)kCsVaryRows; r += blockDim.x) {
        const size_t i = base + r;
        if (i >= n) break;
        const uint32_t g = gid[i];
        for (int j = 0; j < W; ++j) {
            const uint64_t m = words[(size_t)j * stride + i] ^ pl[g * W + j];
            if (m) atomicOr((unsigned long long *)&acc[g * W + j], (unsigned long long)m);
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < gw; e += blockDim.x)
        if (acc[e]) atomicOr((unsigned long long *)&mask[e], (unsigned long long)acc[e]);
}

// The tables of cm copied into LDS in their global layout ([ng][W] masks and
// patterns, [ng][W][6] moves, [ng] bits) when they fit kCsTabLds; cm then
// points at the copies (the lanes of a wave read different groups' entries,
// gathers that L1 serves poorly).  Callers synchronize before use.
constexpr uint32_t kCsTabLds = 48 * 1024;
__host__ __device__ inline uint32_t cs_tab_bytes(int ng, int W) { return (uint32_t)(64 * ng * W + 4 * ng); }

__device__ __forceinline__ void cs_stage_tables(CompactMeta &cm, uint64_t *lds)
{
    const uint32_t gw = (uint32_t)(cm.ng * cm.W);
    uint64_t *m = lds, *p = lds + gw, *v = lds + 2 * gw;
    uint32_t *b = (uint32_t *)(lds + 8 * gw);
    for (uint32_t e = threadIdx.x; e < gw; e += blockDim.x) m[e] = cm.mask[e], p[e] = cm.pat[e];
    for (uint32_t e = threadIdx.x; e < 6 * gw; e += blockDim.x) v[e] = cm.mv[e];
    for (uint32_t e = threadIdx.x; e < (uint32_t)cm.ng; e += blockDim.x) b[e] = cm.bits[e];
    cm.mask = m, cm.pat = p, cm.mv = v, cm.bits = b;
}

// sort key of every row: gid (32) || code (64 WC) || row index (32), WC + 1 words
template <int WC>
__global__ __launch_bounds__(256) void k_cs_keys(const uint64_t *words, size_t stride, const uint32_t *gid,
                                                 uint32_t n, CompactMeta cm, uint64_t *keys, bool lds)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t tl[];
    if (lds) {
        cs_stage_tables(cm, tl);
        __syncthreads();
    }
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = gid[i];
    uint64_t c[WC];
    code_of<WC>(cm, g, words + i, stride, 0, c);
    uint64_t *k = keys + (size_t)i * (WC + 1);
    k[0] = (uint64_t)g << 32 | c[0] >> 32;
#pragma unroll
    for (int m = 1; m < WC; ++m) k[m] = c[m - 1] << 32 | c[m] >> 32;
    k[WC] = c[WC - 1] << 32 | i;
}

// k_cs_keys for keys of at most kProbeWords words with the tables in LDS: a
// row's words up to its group's last varying one are loaded together (one
// round of loads instead of one per word of a run-time loop), mapped in
// registers (shift-in accumulator, as bound_codes), and words past the last
// varying one -- config 3's zero padding -- are neither loaded nor mapped.
template <int WC>
__global__ __launch_bounds__(256) void k_cs_keys_r(const uint64_t *words, size_t stride, const uint32_t *gid,
                                                   uint32_t n, CompactMeta cm, uint64_t *keys)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t tl[];
    cs_stage_tables(cm, tl);
    uint32_t *lnw = (uint32_t *)(tl + 8 * (size_t)cm.ng * cm.W) + cm.ng;  // after the bits
    __syncthreads();
    for (int g = threadIdx.x; g < cm.ng; g += blockDim.x) {
        int nw = 0;
        for (int j = 0; j < cm.W; ++j)
            if (cm.mask[(size_t)g * cm.W + j]) nw = j + 1;
        lnw[g] = (uint32_t)nw;
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = gid[i];
    const int nw = (int)lnw[g];
    uint64_t x[kProbeWords];
#pragma unroll
    for (int j = 0; j < kProbeWords; ++j) x[j] = j < nw ? words[(size_t)j * stride + i] : 0;
    uint64_t c[WC];
#pragma unroll
    for (int k = 0; k < WC; ++k) c[k] = 0;
    int pos = 0;
    const uint64_t *mk = cm.mask + (size_t)g * cm.W, *mvg = cm.mv + (size_t)g * cm.W * 6;
#pragma unroll
    for (int j = 0; j < kProbeWords; ++j) {
        if (j >= nw) break;
        const uint64_t m = mk[j];
        uint64_t v = x[j] & m;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const uint64_t t = v & mvg[j * 6 + q];
            v = (v ^ t) | (t >> (1 << q));
        }
        const int cnt = __popcll(m);
        acc_push<WC>(c, v, cnt);
        pos += cnt;
    }
    acc_align<WC>(c, pos);
    uint64_t *k = keys + (size_t)i * (WC + 1);
    k[0] = (uint64_t)g << 32 | c[0] >> 32;
#pragma unroll
    for (int m = 1; m < WC; ++m) k[m] = c[m - 1] << 32 | c[m] >> 32;
    k[WC] = c[WC - 1] << 32 | i;
}

// inverse of compress (Hacker's Delight expand: the same moves, reversed)
__device__ __forceinline__ uint64_t expand(uint64_t x, uint64_t m, const uint64_t *mv)
{
#pragma unroll
    for (int i = 5; i >= 0; --i) x = (x & ~mv[i]) | ((x << (1 << i)) & mv[i]);
    return x & m;
}

// bits [pos, pos + cnt) (MSB-first, cnt <= 64) of the WC-word number c, right-aligned
template <int WC>
__device__ __forceinline__ uint64_t code_bits(const uint64_t (&c)[WC], int pos, int cnt)
{
    if (cnt == 0) return 0;
    const int w = pos >> 6, off = pos & 63;
    uint64_t x = 0, nx = 0;
#pragma unroll
    for (int k = 0; k < WC; ++k) {
        x = k == w ? c[k] : x;
        nx = k == w + 1 ? c[k] : nx;
    }
    const uint64_t v = off ? (x << off) | (nx >> (64 - off)) : x;
    return cnt == 64 ? v : v >> (64 - cnt);
}

// ---- the unpack fused with the dedupe (as the packed sort's, hsc_ingest.hip) ----
// The last version of a key is the last of its run of equal (gid, code):
// the keys minus their row-index bits.  Blocks of kCsUdTile sorted rows: one
// pass counts the blocks' distinct rows (their exclusive scan gives each
// block's place), the next writes every version to the *_o rows and the last
// of each key to its place among the *_d rows.
constexpr int kCsUdThreads = 1024;
constexpr int kCsUdRows = 2;
constexpr int kCsUdTile = kCsUdThreads * kCsUdRows;

template <int KW>
__device__ __forceinline__ bool cs_last(const uint64_t *keys, size_t n, size_t i)
{
    if (i + 1 >= n) return true;
    const uint64_t *a = keys + i * KW, *b = a + KW;
#pragma unroll
    for (int k = 0; k < KW - 1; ++k)
        if (a[k] != b[k]) return true;
    return (a[KW - 1] >> 32) != (b[KW - 1] >> 32);
}

template <int KW>
__global__ __launch_bounds__(kCsUdThreads) void k_cs_bcount(const uint64_t *keys, size_t n, uint32_t *bc)
{
    __shared__ uint32_t wsum[kCsUdThreads / 64];
    const size_t base = (size_t)blockIdx.x * kCsUdTile;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) {
        const size_t i = base + (size_t)r * kCsUdThreads + threadIdx.x;
        if (i < n) c += cs_last<KW>(keys, n, i);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kCsUdThreads / 64; ++w) t += wsum[w];
        bc[blockIdx.x] = t;
    }
}

template <int WC>
__global__ __launch_bounds__(kCsUdThreads) void k_cs_unpack_dd(
    const uint64_t *keys, size_t n, CompactMeta cm, const uint64_t *lsn_in, uint32_t *gid_o,
    uint64_t *words_o, uint64_t *lsn_o, size_t stride_o, const uint32_t *boff, uint32_t *gid_d,
    uint64_t *words_d, uint64_t *lsn_d, size_t stride_d, uint32_t *d_count, uint64_t *codes_d, bool lds)
{
    constexpr int KW = WC + 1;
    extern __shared__ __attribute__((aligned(16))) uint64_t tl[];
    if (lds) cs_stage_tables(cm, tl);  // synchronized by the scan's barrier below
    __shared__ uint32_t pos[kCsUdTile];
    __shared__ uint32_t wsum[kCsUdThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * kCsUdTile;
    const uint32_t nrows = (uint32_t)min((size_t)kCsUdTile, n - base);
    // thread t ranks rows 8t .. 8t + 7 of the block: flags, wave scan, block scan
    uint32_t fl = 0, cnt = 0;
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) {
        const uint32_t j = threadIdx.x * kCsUdRows + r;
        const bool last = j < nrows && cs_last<KW>(keys, n, base + j);
        fl |= (uint32_t)last << r;
        cnt += last;
    }
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t run = inc - cnt, total = 0;
#pragma unroll
    for (int w = 0; w < kCsUdThreads / 64; ++w) {
        run += w < wv ? wsum[w] : 0;
        total += wsum[w];
    }
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) {
        const uint32_t j = threadIdx.x * kCsUdRows + r;
        if (j < nrows) pos[j] = (fl >> r & 1u) ? run : 0xFFFFFFFFu;
        run += fl >> r & 1u;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *d_count = boff[blockIdx.x] + total;
    __syncthreads();
    const uint32_t b0 = boff[blockIdx.x];
    // every key of the thread's rows first, then their LSN gathers, then the
    // stores (a loop that loads after the previous row's stores waits on two
    // dependent loads per row: the compiler cannot move loads above stores
    // that may alias them)
    uint64_t kr[kCsUdRows][KW], lr[kCsUdRows];
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) {
        const uint32_t j = threadIdx.x + r * kCsUdThreads;  // consecutive rows per wave
        const uint64_t *k = keys + (base + (j < nrows ? j : 0)) * KW;
#pragma unroll
        for (int m = 0; m < KW; ++m) kr[r][m] = k[m];
    }
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) lr[r] = lsn_in[(uint32_t)kr[r][WC]];
#pragma unroll
    for (int r = 0; r < kCsUdRows; ++r) {
        const uint32_t j = threadIdx.x + r * kCsUdThreads;
        if (j >= nrows) break;
        const size_t i = base + j;
        const uint64_t(&kk)[KW] = kr[r];
        const uint32_t g = (uint32_t)(kk[0] >> 32);
        uint64_t c[WC];
#pragma unroll
        for (int m = 0; m < WC; ++m) c[m] = kk[m] << 32 | kk[m + 1] >> 32;
        const uint64_t lv = lr[r];
        const uint32_t d = pos[j];
        const bool last = d != 0xFFFFFFFFu;
        lsn_o[i] = lv;
        gid_o[i] = g;
        if (last) {
            lsn_d[b0 + d] = lv, gid_d[b0 + d] = g;
            if (codes_d)  // the compact tiles' row codes (k_compact_rows of these rows)
#pragma unroll
                for (int m = 0; m < WC; ++m) codes_d[(size_t)m * stride_d + b0 + d] = c[m];
        }
        const uint64_t *mk = cm.mask + (size_t)g * cm.W, *pt = cm.pat + (size_t)g * cm.W;
        const uint64_t *mv = cm.mv + (size_t)g * cm.W * 6;
        int p = 0;
        for (int w = 0; w < cm.W; ++w) {
            const uint64_t m = mk[w];
            const int cn = __popcll(m);
            const uint64_t part = code_bits<WC>(c, p, cn);
            p += cn;
            const uint64_t v = (pt[w] & ~m) | (m ? expand(part, m, mv + 6 * w) : 0);
            words_o[(size_t)w * stride_o + i] = v;
            if (last) words_d[(size_t)w * stride_d + b0 + d] = v;
        }
    }
}

}  // namespace

hipError_t compact_unpack_dedupe(const uint64_t *keys, size_t n, const CompactTables &t,
                                 const uint64_t *lsn_in, uint32_t *gid_o, uint64_t *words_o,
                                 uint64_t *lsn_o, size_t stride_o, uint32_t *gid_d, uint64_t *words_d,
                                 uint64_t *lsn_d, size_t stride_d, uint32_t *d_count, uint32_t *scratch,
                                 uint64_t *codes_d, hipStream_t s)
{
    if (n == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
    const CompactMeta cm = meta_of(t);
    const uint32_t ud = (uint32_t)((n + kCsUdTile - 1) / kCsUdTile);
    uint32_t *bc = scratch, *btmp = scratch + ud + 16;
    switch (t.WC) {
    case 1: k_cs_bcount<2><<<ud, kCsUdThreads, 0, s>>>(keys, n, bc); break;
    case 2: k_cs_bcount<3><<<ud, kCsUdThreads, 0, s>>>(keys, n, bc); break;
    case 3: k_cs_bcount<4><<<ud, kCsUdThreads, 0, s>>>(keys, n, bc); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = scan_exclusive_u32(bc, ud, btmp, s);
    if (e != hipSuccess) return e;
    const uint32_t tb = cs_tab_bytes(t.ng, t.W);
    const bool lds = tb <= kCsTabLds;
#define HSC_CS_UD(WC_)                                                            \
    k_cs_unpack_dd<WC_><<<ud, kCsUdThreads, lds ? tb : 0, s>>>(keys, n, cm, lsn_in, gid_o, words_o, \
                                                               lsn_o, stride_o, bc, gid_d, words_d, \
                                                               lsn_d, stride_d, d_count, codes_d, lds)
    if (t.WC == 1)
        HSC_CS_UD(1);
    else if (t.WC == 2)
        HSC_CS_UD(2);
    else
        HSC_CS_UD(3);
#undef HSC_CS_UD
    return hipGetLastError();
}

hipError_t compact_masks_unsorted(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                                  int W, int ng, uint32_t *rep, uint64_t *mask, uint64_t *pat,
                                  hipStream_t s)
{
    const size_t gw = (size_t)ng * W;
    if (2 * 8 * gw > kCsVaryLds) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(rep, 0xFF, 4 * (size_t)ng, s);
    if (e == hipSuccess) e = hipMemsetAsync(mask, 0, 8 * gw, s);
    if (e != hipSuccess) return e;
    if (n) k_cs_rep<<<(n + kCsRepRows - 1) / kCsRepRows, 256, 4 * (size_t)ng, s>>>(gid, n, ng, rep);
    if (gw) k_cs_pat<<<(uint32_t)((gw + 255) / 256), 256, 0, s>>>(words, stride, W, ng, rep, pat);
    if (n)
        k_cs_vary<<<(n + kCsVaryRows - 1) / kCsVaryRows, 256, 2 * 8 * gw, s>>>(words, stride, gid, n, W,
                                                                             ng, pat, mask);
    return hipGetLastError();
}

hipError_t compact_sort_keys(const uint64_t *words, size_t stride, const uint32_t *gid, uint32_t n,
                             const CompactTables &t, uint64_t *keys, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    const CompactMeta cm = meta_of(t);
    const uint32_t b = (n + 255) / 256;
    const uint32_t tb = cs_tab_bytes(t.ng, t.W);
    const bool lds = tb <= kCsTabLds;
    const uint32_t ldsb = lds ? tb : 0;
    if (lds && t.W <= kProbeWords) {
        const uint32_t lb = tb + 4 * (uint32_t)t.ng;  // + each group's words to its last varying one
        switch (t.WC) {
        case 1: k_cs_keys_r<1><<<b, 256, lb, s>>>(words, stride, gid, n, cm, keys); break;
        case 2: k_cs_keys_r<2><<<b, 256, lb, s>>>(words, stride, gid, n, cm, keys); break;
        case 3: k_cs_keys_r<3><<<b, 256, lb, s>>>(words, stride, gid, n, cm, keys); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (t.WC) {
    case 1: k_cs_keys<1><<<b, 256, ldsb, s>>>(words, stride, gid, n, cm, keys, lds); break;
    case 2: k_cs_keys<2><<<b, 256, ldsb, s>>>(words, stride, gid, n, cm, keys, lds); break;
    case 3: k_cs_keys<3><<<b, 256, ldsb, s>>>(words, stride, gid, n, cm, keys, lds); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

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
                          hipStream_t s, const PointHash *php)
{
    if (p.n == 0) return hipSuccess;
    const CompactMeta cm = meta_of(t);
    PointHash ph{};
    if (php && php->nb && php->e && php->flags && t.WC <= 3 && t.W <= kProbeWords) ph = *php;
    switch (t.WC) {
    case 1: return launch_probes_wc<1>(p, cm, clo, chi, s, ph);
    case 2: return launch_probes_wc<2>(p, cm, clo, chi, s, ph);
    case 3: return launch_probes_wc<3>(p, cm, clo, chi, s, ph);
    case 4: return launch_probes_wc<4>(p, cm, clo, chi, s, ph);
    case 5: return launch_probes_wc<5>(p, cm, clo, chi, s, ph);
    case 6: return launch_probes_wc<6>(p, cm, clo, chi, s, ph);
    default: return hipErrorInvalidValue;
    }
}

// one four-slot bucket per key: a quarter full, so a lookup of a key the
// window does not hold -- half of config 3's points -- stops at its home
// line nearly always (two-slot buckets three quarters full walked ~4 of
// them: the bound kernel 30 -> 59 us, r06d)
uint64_t point_hash_buckets(uint32_t n) { return (uint64_t)n + 64; }

hipError_t point_hash_build(const CTiles &ct, uint64_t *e, uint64_t nb, uint32_t ep, bool clear, hipStream_t s)
{
    hipError_t r = clear ? hipMemsetAsync(e, 0, 128 * nb, s) : hipSuccess;
    if (r != hipSuccess || ct.n == 0) return r;
    k_ph_insert<<<(ct.n + 255) / 256, 256, 0, s>>>(ct, e, nb, ep);
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_compact()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_group_pattern);
}

}  // namespace hsc
