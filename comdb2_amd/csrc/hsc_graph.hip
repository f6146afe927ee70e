// hsc_graph.hip -- WR/WW/RW dependency graph + strongly connected components
// on gfx950 (the Jepsen-style extension of the check).
//
// History: micro-ops (txn, key, read|write, observed writer) of committed
// transactions, txn ids in commit order (a key's version order is the commit
// order of its writers).  Edges (Adya):
//   ww  w_i -> w_{i+1}                 consecutive writers of a key
//   wr  writer(observed) -> reader
//   rw  reader -> next writer after the observed version
// Build: sort the writers by (key, txn) with the window's LSD radix sort,
// emit edges with one thread per op (binary search of the next writer),
// radix-sort (src, dst), merge duplicates (type bits OR-ed), and build CSR
// (out-edges) and CSC (in-edges).
// SCC: Orzan's colouring.  Per round every live node starts with colour =
// its id; colours propagate forward along live edges (max) from a frontier
// until stable; a node whose colour is still its own id is the largest
// member of its SCC (every member reaches it), and a backward sweep over
// in-edges restricted to that colour marks the SCC.  Marked nodes retire
// with scc = colour.  In a dependency graph almost every edge goes forward in
// commit order, so colours only move across stale-read (rw) windows and the
// rounds are few.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

namespace hsc {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Writers of the history -> rows (gid 0, words (key, txn), lsn 0), gathered
// without a flag array or a scan over the ops: a block of
// kGwThreads x kGwItems ops counts its writers (k_gw_count: no atomics, one
// word per block), the block counts are scanned (24k words for 100M ops), and
// k_gw_place writes each block's writers in op order at its offset (wave
// ballots + one LDS scan).  (r06: one atomic per block on a single cursor
// instead of the count pass serialised 24k blocks: 1.48 ms per 100M ops.)
constexpr int kGwThreads = 256, kGwItems = 16;
// thread t of a block takes ops base + 16 t .. base + 16 t + 15 (one 16-byte
// load of is_write): the block's writers come out in op order, so writers of
// txn-ordered ops stay txn-ordered (the writer sort then skips the txn bits)
__device__ __forceinline__ uint32_t gw_bits(size_t nops, const uint8_t *is_write, size_t base, uint32_t &cnt)
{
    const size_t i0 = base + (size_t)threadIdx.x * kGwItems;
    uint32_t w = 0;  // bit k: op i0 + k writes
    if (i0 + kGwItems <= nops && ((uintptr_t)(is_write + i0) & 15) == 0) {
        const uint4 v = *(const uint4 *)(is_write + i0);
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < kGwItems; ++k) w |= (uint32_t)(((x[k >> 2] >> (8 * (k & 3))) & 0xFFu) != 0) << k;
    } else {
#pragma unroll
        for (int k = 0; k < kGwItems; ++k) {
            const size_t i = i0 + k;
            w |= (uint32_t)(i < nops && is_write[i]) << k;
        }
    }
    cnt = (uint32_t)__popc(w);
    return w;
}

// (bad != null: the observed ids' range check here too -- bit 0 -- for the
// builds whose edge pass does not check them itself; the txns' range and order
// are k_gw_place's)
// out[0] / out[1] = the varying bits of the writers' key / txn, out[2] = 0
// (their gid): OR & ~AND over k_gw_place's block partials; out[3] / out[4]
// the ANDs
__global__ __launch_bounds__(1024) void k_vary_reduce(uint32_t nb, const uint64_t *vp, uint64_t *out,
                                                       const uint32_t *nwb)
{
    __shared__ uint64_t red[16][4];
    uint64_t ko = 0, ka = ~0ull, to = 0, ta = ~0ull;
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        ko |= vp[4 * (size_t)b], ka &= vp[4 * (size_t)b + 1];
        to |= vp[4 * (size_t)b + 2], ta &= vp[4 * (size_t)b + 3];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ko |= __shfl_xor(ko, o, 64), ka &= __shfl_xor(ka, o, 64);
        to |= __shfl_xor(to, o, 64), ta &= __shfl_xor(ta, o, 64);
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red[wv][0] = ko, red[wv][1] = ka, red[wv][2] = to, red[wv][3] = ta;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) ko |= red[w][0], ka &= red[w][1], to |= red[w][2], ta &= red[w][3];
        out[0] = ko & ~ka;
        out[1] = to & ~ta;
        out[2] = 0;
        out[3] = ka;  // (their constant bits: AND & ~varying)
        out[4] = ta;
        out[5] = nwb[0];  // (the writer count and the place pass's check bits: one read)
        out[6] = nwb[1];
    }
}

__global__ __launch_bounds__(kGwThreads) void k_gw_count(size_t nops, const uint8_t *is_write, uint32_t *bc,
                                                         const uint32_t *observed, uint32_t ntxn, uint32_t *bad)
{
    __shared__ uint32_t wsum[kGwThreads / 64];
    uint32_t cnt;
    const size_t base = (size_t)blockIdx.x * (kGwThreads * kGwItems);
    (void)gw_bits(nops, is_write, base, cnt);
    if (bad) {  // (coalesced: op base + 256 k + t)
        uint32_t b = 0;
#pragma unroll
        for (int k = 0; k < kGwItems; ++k) {
            const size_t i = base + (size_t)k * kGwThreads + threadIdx.x;
            if (i >= nops) break;
            const uint32_t o = observed[i];
            b |= (o != kNone && o >= ntxn) ? 1u : 0u;
        }
        const uint64_t any = __ballot(b != 0);
        if (any && b) atomicOr(bad, b);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int q = 0; q < kGwThreads / 64; ++q) t += wsum[q];
        bc[blockIdx.x] = t;
    }
}

// Coalesced: round k of wave v takes the 64 ops base + 256 k + 64 v + lane
// -- 64 segments in op order, each one ballot -- so a writer's place in the
// block is its segment's exclusive count (one wave scans the 64) plus the
// writers before it in the ballot; a segment's writers store as one
// contiguous run straight from the lanes (no LDS staging: the 64 KB of it held
// the kernel to 2 workgroups per CU).  (A thread taking 16 consecutive ops,
// the count pass's shape, issued every key / txn load over 64 lines: 0.57 ms
// per 100M ops.)  bad != null: the txns' check -- bit 0 a txn >= ntxn, bit 1 a
// txn below its predecessor's -- on the txn words it loads anyway.
// vp: the block's writers' OR and AND of key and txn (vp[4 b + 0..3]), which
// k_vary_reduce turns into the writer rows' varying bits (no pass over the
// gathered rows for them)
__global__ __launch_bounds__(kGwThreads) void k_gw_place(size_t nops, const uint32_t *txn, const uint64_t *key,
                                                         const uint8_t *is_write, const uint32_t *boff,
                                                         uint32_t *gid, uint64_t *words, size_t stride,
                                                         uint32_t ntxn, uint32_t *bad, uint64_t *vp)
{
    __shared__ uint64_t vred[kGwThreads / 64][4];
    constexpr int kSeg = kGwItems * (kGwThreads / 64);
    static_assert(kSeg == 64, "one wave scans the segments");
    __shared__ uint32_t segc[kSeg];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * (kGwThreads * kGwItems);
    // every load issued before the first use (2 blocks per CU by the LDS:
    // the latency is hidden by the loads in flight, not by waves)
    uint64_t m[kGwItems], kv[kGwItems];
    uint32_t tv[kGwItems];
    uint8_t wv8[kGwItems];
#pragma unroll
    for (int k = 0; k < kGwItems; ++k) {
        const size_t i = base + (size_t)k * kGwThreads + threadIdx.x;
        const bool in = i < nops;
        wv8[k] = in ? is_write[i] : 0;
        tv[k] = in ? txn[i] : 0;
        kv[k] = in ? key[i] : 0;
    }
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < kGwItems; ++k) {
        const size_t i = base + (size_t)k * kGwThreads + threadIdx.x;
        m[k] = __ballot(wv8[k] != 0);
        if (lane == 0) segc[k * 4 + wv] = (uint32_t)__popcll(m[k]);
        if (bad) {  // (the predecessor: the lane before's, lane 0 loads it)
            uint32_t prev = __shfl_up(tv[k], 1, 64);
            if (lane == 0) prev = i > 0 && i < nops ? txn[i - 1] : 0;
            if (i < nops) {
                b |= tv[k] >= ntxn ? 1u : 0u;
                b |= tv[k] < prev ? 2u : 0u;
            }
        }
    }
    if (bad) {
        const uint64_t any = __ballot(b != 0);
        if (any && b) atomicOr(bad, b);
    }
    uint64_t ko = 0, ka = ~0ull, to = 0, ta = ~0ull;
#pragma unroll
    for (int k = 0; k < kGwItems; ++k) {
        if (!wv8[k]) continue;
        ko |= kv[k], ka &= kv[k], to |= tv[k], ta &= tv[k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ko |= __shfl_xor(ko, o, 64), ka &= __shfl_xor(ka, o, 64);
        to |= __shfl_xor(to, o, 64), ta &= __shfl_xor(ta, o, 64);
    }
    if (lane == 0) vred[wv][0] = ko, vred[wv][1] = ka, vred[wv][2] = to, vred[wv][3] = ta;
    __syncthreads();
    if (vp && threadIdx.x < 4) {
        const int q = threadIdx.x;
        uint64_t v = vred[0][q];
#pragma unroll
        for (int w = 1; w < kGwThreads / 64; ++w) v = (q & 1) ? (v & vred[w][q]) : (v | vred[w][q]);
        vp[4 * (size_t)blockIdx.x + q] = v;
    }
    if (wv == 0) {
        const uint32_t v = segc[lane];
        uint32_t inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        segc[lane] = inc - v;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
    const size_t b0 = boff[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kGwItems; ++k) {
        if (!((m[k] >> lane) & 1ull)) continue;
        const size_t p = b0 + segc[k * 4 + wv] + (uint32_t)__popcll(m[k] & lt);
        words[p] = kv[k];
        words[stride + p] = tv[k];
        gid[p] = 0;
    }
}

// a backward edge a -> b (a > b) covers [b, a] (graph_cover's k_back_diff,
// done while a raw build emits the row: one pass over the raw rows less)
__device__ __forceinline__ void back_row(uint32_t *diff, uint64_t row)
{
    if (!diff || row == ~0ull) return;
    const uint32_t a = (uint32_t)(row >> 32), b = (uint32_t)row;
    if (a > b) {
        atomicAdd(&diff[b], 1u);
        atomicAdd(&diff[a + 1], 0xFFFFFFFFu);
    }
}

// Where a raw build's backward edges go: the interval diffs (diff), or a
// list of the rows themselves (list: config 4 has a few thousand among 95M
// edges -- the cover is then their intervals marked in place of a scan of
// ntxn diffs; past cap only counted, and graph_cover takes the diffs)
struct BackSink {
    uint32_t *diff;
    uint64_t *list;
    uint32_t *cnt;
    uint32_t cap;
};

// (every active lane calls it: one wave-aggregated atomic for the list)
__device__ __forceinline__ void back_push(const BackSink &bs, uint64_t row)
{
    if (!bs.list) {
        back_row(bs.diff, row);
        return;
    }
    const bool is = row != ~0ull && (uint32_t)(row >> 32) > (uint32_t)row;
    const uint64_t m = __ballot(is);
    if (!m) return;
    const int lane = threadIdx.x & 63, first = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(bs.cnt, (uint32_t)__popcll(m));
    base = __shfl(base, first, 64);
    const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (is && slot < bs.cap) bs.list[slot] = row;
}

// Edge rows: word = src << 32 | dst, payload = type; invalid = ~0.
// Slots [0, nu): ww of unique writer i -> i+1; slots nu + 2i, nu + 2i + 1:
// wr / rw of op i.
// (et / eg null: a raw build -- the rows alone; the type is the slot's)
__global__ void k_edges_ww(uint32_t nu, const uint64_t *wkey, const uint64_t *wtxn,
                           uint64_t *ew, uint64_t *et, uint32_t *eg)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu) return;
    uint64_t e = ~0ull;
    if (i + 1 < nu && wkey[i] == wkey[i + 1]) e = (wtxn[i] << 32) | wtxn[i + 1];
    ew[i] = e;
    if (et) {
        et[i] = kDepWW;
        eg[i] = 0;
    }
}

// chk_n != 0: an observed id >= chk_n sets bit 0 of *bad and the op gives no
// rows (the build's check: the txns are k_gw_place's)
__device__ __forceinline__ bool obs_bad(uint32_t ob, uint32_t chk_n, uint32_t *bad)
{
    if (chk_n == 0 || ob == kNone || ob < chk_n) return false;
    atomicOr(bad, 1u);
    return true;
}

__global__ void k_edges_reads(size_t nops, const uint32_t *txn, const uint64_t *key,
                              const uint8_t *is_write, const uint32_t *observed, uint32_t nu,
                              const uint64_t *wkey, const uint64_t *wtxn, uint64_t *ew,
                              uint64_t *et, uint32_t *eg, int skip_rw, uint32_t chk_n, uint32_t *bad)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nops) return;
    uint64_t wr = ~0ull, rw = ~0ull;
    // (every op's observed id checked, a write's too: the build's contract)
    if (!obs_bad(observed[i], chk_n, bad) && !is_write[i]) {
        const uint32_t r = txn[i], ob = observed[i];
        const uint64_t k = key[i];
        if (ob != kNone && ob != r) wr = ((uint64_t)ob << 32) | r;
        // first writer (key, txn) > (k, ob), or >= (k, 0) for the initial version
        uint32_t lo = 0, hi = nu;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t mk = wkey[mid], mt = wtxn[mid];
            const bool before = mk < k || (mk == k && (ob == kNone ? false : mt <= ob));
            if (before)
                lo = mid + 1;
            else
                hi = mid;
        }
        if (!skip_rw && lo < nu && wkey[lo] == k && wtxn[lo] != r)
            rw = ((uint64_t)r << 32) | wtxn[lo];
    }
    const size_t s = (size_t)nu + 2 * i;
    ew[s] = wr;
    ew[s + 1] = rw;
    if (et) {
        et[s] = kDepWR;
        eg[s] = 0;
        et[s + 1] = kDepRW;
        eg[s + 1] = 0;
    }
}

// ---- packed writer search ----
// When the writers sorted as packed (key, txn) words (graph_build), every
// distinct writer is one u64 pk[i] = compress(key) << tb | compress(txn),
// ascending, and a directory of 2^D buckets over [pk[0], pk[nu - 1]] gives
// each bucket's first writer: a read's "first writer after (k, ob)" is one
// directory line plus a binary search inside its bucket (~30 writers on
// uniform keys) instead of ~26 dependent steps over the 16-byte rows.
// (struct PairPack: hsc_internal.h -- GraphBufs keeps the last build's)

// bucket of x: 0 below the range, 2^D past it
__device__ __forceinline__ uint64_t pair_bucket(const PairPack &pp, uint64_t x)
{
    if (x <= pp.base) return 0;
    const uint64_t b = pp.shift >= 64 ? 0 : (x - pp.base) >> pp.shift;
    return b < (1ull << pp.D) ? b : (1ull << pp.D);
}

__device__ __forceinline__ uint64_t pair_key(const PairPack &pp, uint64_t kp) { return pp.tb >= 64 ? 0 : kp << pp.tb; }

// the first writer of key kp (compressed) with txn > ob, ob having bits
// outside the writers' txn bits (so not compressible): a search of pk on the
// expanded txns (compress / expand keep the order of values sharing the
// constant bits); the rw row r -> it, or ~0
__device__ __forceinline__ uint64_t pk_rw_slow(uint32_t nu, const uint64_t *pk, const PairPack &pp,
                                               const uint64_t (&tmv)[6], uint64_t kp, uint32_t ob, uint32_t r)
{
    const uint64_t tmask = pp.tb >= 64 ? ~0ull : (1ull << pp.tb) - 1;
    uint32_t lo = 0, hi = nu;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t v = pk[mid], kv = pp.tb >= 64 ? 0 : v >> pp.tb;
        if (kv < kp || (kv == kp && (bits_expand(v & tmask, pp.tm, tmv) | pp.tc) <= ob))
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo >= nu) return ~0ull;
    const uint64_t v = pk[lo];
    if ((pp.tb >= 64 ? 0 : v >> pp.tb) != kp) return ~0ull;
    const uint32_t wt = (uint32_t)(bits_expand(v & tmask, pp.tm, tmv) | pp.tc);
    return wt != r ? ((uint64_t)r << 32) | wt : ~0ull;
}

// k_edges_ww over the packed distinct writers
__global__ void k_edges_ww_pk(uint32_t nu, const uint64_t *pk, PairPack pp, uint64_t *ew, uint64_t *et,
                              uint32_t *eg)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu) return;
    uint64_t e = ~0ull;
    if (i + 1 < nu) {
        const uint64_t a = pk[i], b = pk[i + 1];
        if (pp.tb >= 64 || (a >> pp.tb) == (b >> pp.tb)) {
            uint64_t tm[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) tm[q] = pp.tmv[q];
            const uint64_t tmask = pp.tb >= 64 ? ~0ull : (1ull << pp.tb) - 1;
            e = ((bits_expand(a & tmask, pp.tm, tm) | pp.tc) << 32) | (bits_expand(b & tmask, pp.tm, tm) | pp.tc);
        }
    }
    ew[i] = e;
    if (et) {
        et[i] = kDepWW;
        eg[i] = 0;
    }
}

__global__ void k_pair_keys(uint32_t nu, const uint64_t *wkey, const uint64_t *wtxn, PairPack pp, uint64_t *pk)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu) return;
    uint64_t km[6], tm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) km[q] = pp.kmv[q], tm[q] = pp.tmv[q];
    pk[i] = pair_key(pp, bits_compress(wkey[i], pp.km, km)) | bits_compress(wtxn[i], pp.tm, tm);
}

// dir[b] = first writer >= base + (b << shift), b in [0, 2^D + 1] (one
// binary search per bucket: the same cost for any key distribution -- a
// thread per writer filling the buckets up to the next one serialises on
// empty stretches)
__global__ void k_pair_dir(uint32_t nu, const uint64_t *pk, PairPack pp, uint32_t *dir)
{
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > (1ull << pp.D) + 1) return;
    uint32_t lo = nu;
    if (b == 0) {
        lo = 0;
    } else if (pp.shift < 64 && b <= ((pp.last - pp.base) >> pp.shift)) {
        const uint64_t x = pp.base + (b << pp.shift);
        uint32_t hi = nu;
        lo = 0;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pk[mid] < x)
                lo = mid + 1;
            else
                hi = mid;
        }
    }
    dir[b] = lo;
}

__global__ void k_edges_reads_pk(size_t nops, const uint32_t *txn, const uint64_t *key,
                                 const uint8_t *is_write, const uint32_t *observed, uint32_t nu,
                                 const uint64_t *wkey, const uint64_t *wtxn, const uint64_t *pk,
                                 const uint32_t *dir, PairPack pp, uint64_t *ew, uint64_t *et,
                                 uint32_t *eg, int skip_rw, BackSink diff, uint32_t chk_n,
                                 uint32_t *bad)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nops) return;
    uint64_t wr = ~0ull, rw = ~0ull;
    // (every op's observed id checked, a write's too: the build's contract)
    if (!obs_bad(observed[i], chk_n, bad) && !is_write[i]) {
        const uint32_t r = txn[i], ob = observed[i];
        const uint64_t k = key[i];
        if (ob != kNone && ob != r) wr = ((uint64_t)ob << 32) | r;
        // a key outside the writers' constant bits has no writer at all
        if (!skip_rw && (k & ~pp.km) == pp.kc) {
            uint32_t lo = 0, hi = nu;
            bool found = false;
            if (ob == kNone || (ob & ~pp.tm) == pp.tc) {
                uint64_t km[6], tm[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) km[q] = pp.kmv[q], tm[q] = pp.tmv[q];
                const uint64_t kp = bits_compress(k, pp.km, km);
                // initial version: first writer >= (k, any); else first > (k, ob)
                const uint64_t x = pair_key(pp, kp) | (ob == kNone ? 0 : bits_compress(ob, pp.tm, tm));
                const bool strict = ob != kNone;
                const uint64_t b = pair_bucket(pp, x);
                lo = dir[b];
                hi = dir[b + 1];
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    const uint64_t v = pk[mid];
                    if (strict ? v <= x : v < x)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                if (lo < nu) {
                    const uint64_t v = pk[lo];
                    const uint64_t tmask = pp.tb >= 64 ? ~0ull : (1ull << pp.tb) - 1;
                    if ((pp.tb >= 64 ? 0 : v >> pp.tb) == kp) {
                        const uint32_t wt = (uint32_t)(bits_expand(v & tmask, pp.tm, tm) | pp.tc);
                        if (wt != r) rw = ((uint64_t)r << 32) | wt;
                    }
                }
                found = true;
            }
            if (!found) {  // an observed txn outside the writers' bits
                uint64_t km[6], tm[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) km[q] = pp.kmv[q], tm[q] = pp.tmv[q];
                rw = pk_rw_slow(nu, pk, pp, tm, bits_compress(k, pp.km, km), ob, r);
            }
        }
    }
    const size_t s = (size_t)nu + 2 * i;
    ew[s] = wr;
    ew[s + 1] = rw;
    back_push(diff, wr);
    back_push(diff, rw);
    if (et) {
        et[s] = kDepWR;
        eg[s] = 0;
        et[s + 1] = kDepRW;
        eg[s + 1] = 0;
    }
}

// ---- bucket lines: the directory's buckets inline ----
// k_edges_reads_pk reads a directory line, then one or two lines of pk: ~2.5
// random lines and ~4 dependent loads per read (config 4: 3.5 ms, 22 GB).
// Here bucket b is one 64-byte line: a header lo << 32 | has_next << 31 | n
// (lo = the bucket's first writer in pk, n its writers), the first writer
// after the bucket (the answer when every writer of the bucket is <= the
// read's x), then its first kPtE writers as 32-bit offsets from the bucket's
// start base + (b << shift) -- writers of one bucket differ only in their low
// shift bits.  Config 4's 4M buckets are 256 MB: the Infinity Cache's size.
// A read is one line; a bucket of more than kPtE writers (~5 % at 8 per
// bucket) searches pk as before.  (A first form with 14 full 8-byte entries
// per 128-byte line, 512 MB: the search 3.5 -> 2.85 ms, but stored a u64 per
// thread 128 bytes apart -- 5 GB of partial-line writes, 1.05 ms.)
// LW = 8: 64-byte lines, 12 offsets, about 8 writers per bucket (default);
// LW = 16: 128-byte lines, 28 offsets, about 16 writers per bucket -- the same
// table bytes, ~0.3 % of the buckets overflow instead of ~5 %, but measured
// slower (r06x).
__device__ __forceinline__ uint64_t bucket_start(const PairPack &pp, uint64_t b)
{
    return pp.base + (pp.shift >= 64 ? 0 : b << pp.shift);
}

// LW threads per bucket, one 8-byte word each: coalesced lines.  (The bucket
// bounds searched here instead of by k_pair_dir -- lane 0 of each bucket,
// shuffled to the rest -- measured 1.07 ms against 0.28 ms for the two
// passes, r06aa: 8 searches per wave instead of 64.)
template <int LW>
__global__ void k_pair_table(uint32_t nu, const uint64_t *pk, const uint32_t *dir, uint64_t nb, PairPack pp,
                             uint64_t *tab)
{
    const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t b = id / LW;
    const int w = (int)(id % LW);
    if (b >= nb) return;
    const uint32_t lo = dir[b], hi = dir[b + 1];
    const uint32_t n = hi - lo;
    uint64_t v;
    if (w == 0) {
        v = ((uint64_t)lo << 32) | ((uint64_t)(hi < nu) << 31) | (uint64_t)min(n, 0x7FFFFFFFu);
    } else if (w == 1) {
        v = hi < nu ? pk[hi] : ~0ull;
    } else {
        const uint64_t s0 = bucket_start(pp, b);
        const uint32_t j0 = 2 * (uint32_t)(w - 2), j1 = j0 + 1;
        const uint32_t e0 = j0 < n ? (uint32_t)(pk[lo + j0] - s0) : 0xFFFFFFFFu;
        const uint32_t e1 = j1 < n ? (uint32_t)(pk[lo + j1] - s0) : 0xFFFFFFFFu;
        v = (uint64_t)e0 | ((uint64_t)e1 << 32);
    }
    tab[(uint64_t)LW * b + w] = v;
}

// NT: the op columns (read once) and the rows (not read back by this step's
// cover or cut on the usual path) move with non-temporal loads / stores, so
// they do not push the bucket lines -- the only re-read data -- out of the
// caches
template <int LW, bool NT>
__global__ void k_edges_reads_pt(size_t nops, const uint32_t *txn, const uint64_t *key,
                                 const uint8_t *is_write, const uint32_t *observed, uint32_t nu,
                                 const uint64_t *wkey, const uint64_t *wtxn, const uint64_t *pk,
                                 const uint64_t *tab, PairPack pp, uint64_t *ew, uint64_t *et,
                                 uint32_t *eg, int skip_rw, BackSink diff, uint32_t chk_n,
                                 uint32_t *bad)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nops) return;
    uint64_t wr = ~0ull, rw = ~0ull;
    const uint32_t ob0 = NT ? __builtin_nontemporal_load(observed + i) : observed[i];
    const bool isw = (NT ? __builtin_nontemporal_load(is_write + i) : is_write[i]) != 0;
    // (every op's observed id checked, a write's too: the build's contract)
    if (!obs_bad(ob0, chk_n, bad) && !isw) {
        const uint32_t r = NT ? __builtin_nontemporal_load(txn + i) : txn[i], ob = ob0;
        const uint64_t k = NT ? __builtin_nontemporal_load(key + i) : key[i];
        if (ob != kNone && ob != r) wr = ((uint64_t)ob << 32) | r;
        if (!skip_rw && (k & ~pp.km) == pp.kc) {
            uint64_t km[6], tm[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) km[q] = pp.kmv[q], tm[q] = pp.tmv[q];
            if (ob == kNone || (ob & ~pp.tm) == pp.tc) {
                const uint64_t kp = bits_compress(k, pp.km, km);
                const uint64_t x = pair_key(pp, kp) | (ob == kNone ? 0 : bits_compress(ob, pp.tm, tm));
                const bool strict = ob != kNone;
                const uint64_t b = pair_bucket(pp, x);
                constexpr int kPtE = 2 * (LW - 2);
                const u64x2 *line = (const u64x2 *)(tab + (uint64_t)LW * b);
                u64x2 e[LW / 2];
#pragma unroll
                for (int q = 0; q < LW / 2; ++q) e[q] = line[q];
                const uint64_t hd = e[0].x;
                const uint32_t n = (uint32_t)(hd & 0x7FFFFFFFu), lo = (uint32_t)(hd >> 32);
                bool have = false;
                uint64_t v = 0;
                if (n <= (uint32_t)kPtE) {
                    // the first entry > x (>= x for the initial version), in
                    // offsets from the bucket's start (x below it: every entry)
                    const uint64_t s0 = bucket_start(pp, b);
                    const int64_t xr = x < s0 ? -1 : (int64_t)(x - s0);
                    uint32_t ent[kPtE];
#pragma unroll
                    for (int q = 0; q < kPtE / 2; ++q) {
                        const uint64_t pw = (q & 1) ? e[1 + q / 2].y : e[1 + q / 2].x;  // word 2 + q
                        ent[2 * q] = (uint32_t)pw, ent[2 * q + 1] = (uint32_t)(pw >> 32);
                    }
#pragma unroll
                    for (int j = kPtE - 1; j >= 0; --j) {
                        const int64_t ej = ent[j];
                        if ((uint32_t)j < n && (strict ? ej > xr : ej >= xr)) v = s0 + (uint64_t)ent[j], have = true;
                    }
                    if (!have && ((hd >> 31) & 1)) v = e[0].y, have = true;  // the next bucket's first
                } else {  // an overflowing bucket: its writers in pk
                    uint32_t a = lo, h = lo + n;
                    while (a < h) {
                        const uint32_t mid = (a + h) >> 1;
                        const uint64_t pv = pk[mid];
                        if (strict ? pv <= x : pv < x)
                            a = mid + 1;
                        else
                            h = mid;
                    }
                    if (a < nu) v = pk[a], have = true;
                }
                if (have) {
                    const uint64_t tmask = pp.tb >= 64 ? ~0ull : (1ull << pp.tb) - 1;
                    if ((pp.tb >= 64 ? 0 : v >> pp.tb) == kp) {
                        const uint32_t wt = (uint32_t)(bits_expand(v & tmask, pp.tm, tm) | pp.tc);
                        if (wt != r) rw = ((uint64_t)r << 32) | wt;
                    }
                }
            } else {  // an observed txn outside the writers' bits
                rw = pk_rw_slow(nu, pk, pp, tm, bits_compress(k, pp.km, km), ob, r);
            }
        }
    }
    const size_t s = (size_t)nu + 2 * i;
    if (NT) {
        __builtin_nontemporal_store(wr, ew + s);
        __builtin_nontemporal_store(rw, ew + s + 1);
    } else {
        ew[s] = wr;
        ew[s + 1] = rw;
    }
    back_push(diff, wr);
    back_push(diff, rw);
    if (et) {
        et[s] = kDepWR;
        eg[s] = 0;
        et[s + 1] = kDepRW;
        eg[s + 1] = 0;
    }
}

// ---- partitioned read search (the packed writers) ----
// k_edges_reads_pk answers each read with a directory line and a search of
// pk: two dependent random lines per read over a 33M-writer array (config 4:
// 3.4 ms of a 10.5 ms step).  Instead the reads are partitioned by directory
// range (2^14 partitions of ~2k writers): one pass counts, one scatters the
// search items (x, reader) into their partitions, and a workgroup per
// partition stages its writers in LDS once and answers every item there --
// the reads' random accesses become streams plus LDS searches.  Edge rows:
// [nu, nu + nops) the wr edge of op i, [nu + nops, + items + fallbacks) the
// rw edges in partition order (raw rows carry no slot meaning; a full build
// sorts them).
constexpr int kRpBitsMax = 14;        // at most 2^14 partitions
constexpr uint32_t kRpLds = 6144;     // writers a partition stages (48 KiB of LDS)
constexpr int kRpThreads = 256;

struct RpArgs {
    size_t nops;
    const uint32_t *txn;
    const uint64_t *key;
    const uint8_t *is_write;
    const uint32_t *observed;
    uint32_t nu;
    const uint64_t *wkey, *wtxn, *pk;
    const uint32_t *dir;
    uint32_t ps;         // partition = bucket >> ps
    uint32_t np;         // partitions (incl. the one past the range)
    uint32_t *cnt;       // [np + 1] counts, then offsets (exclusive scan; [np] = items)
    uint32_t *cur;       // [np + 1] cursors; cur[np] = fallback rows
    ulonglong2 *items;   // (x, reader | strict << 32)
    uint64_t *ew;        // edge rows
    uint64_t *et;        // types (full builds) or null
    uint32_t *eg;
    uint32_t *diff;      // raw builds: the cover's interval diffs of backward edges (else null)
    int skip_rw;
};

// x of a read's "first writer after (k, ob)" search, or false when it needs
// none (key without writers) / the row search (an observed txn outside the
// writers' bits).  *fb: the row search is needed.
__device__ __forceinline__ bool rp_x(const PairPack &pp, uint64_t k, uint32_t ob, uint64_t *x, bool *fb)
{
    *fb = false;
    if ((k & ~pp.km) != pp.kc) return false;
    if (ob != kNone && (ob & ~pp.tm) != pp.tc) {
        *fb = true;
        return false;
    }
    uint64_t km[6], tm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) km[q] = pp.kmv[q], tm[q] = pp.tmv[q];
    *x = pair_key(pp, bits_compress(k, pp.km, km)) | (ob == kNone ? 0 : bits_compress(ob, pp.tm, tm));
    return true;
}

__global__ __launch_bounds__(kRpThreads) void k_rp_count(RpArgs a, PairPack pp)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.nops || a.skip_rw || a.is_write[i]) return;
    uint64_t x;
    bool fb;
    if (rp_x(pp, a.key[i], a.observed[i], &x, &fb))
        atomicAdd(&a.cnt[(uint32_t)(pair_bucket(pp, x) >> a.ps)], 1u);
}

// exclusive scan of cnt[0, np) in place, cnt[np] = total; cur zeroed
__global__ __launch_bounds__(1024) void k_rp_scan(RpArgs a)
{
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, per = (a.np + 1023) / 1024;
    const uint32_t b = t * per, e = min(a.np, b + per);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += a.cnt[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan of the parts
        const uint32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t c = a.cnt[i];
        a.cnt[i] = run;
        run += c;
    }
    if (t == 1023) a.cnt[a.np] = part[1023];
    for (uint32_t i = t; i <= a.np; i += 1024) a.cur[i] = 0;
}

__global__ __launch_bounds__(kRpThreads) void k_rp_scatter(RpArgs a, PairPack pp)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.nops) return;
    uint64_t wr = ~0ull;
    if (!a.is_write[i]) {
        const uint32_t r = a.txn[i], ob = a.observed[i];
        const uint64_t k = a.key[i];
        if (ob != kNone && ob != r) wr = ((uint64_t)ob << 32) | r;
        uint64_t x;
        bool fb;
        if (!a.skip_rw && rp_x(pp, k, ob, &x, &fb)) {
            const uint32_t p = (uint32_t)(pair_bucket(pp, x) >> a.ps);
            const uint32_t slot = a.cnt[p] + atomicAdd(&a.cur[p], 1u);
            a.items[slot] = make_ulonglong2(x, (uint64_t)r | (ob != kNone ? 1ull << 32 : 0));
        } else if (!a.skip_rw && fb) {  // the row search (rare): its rw row after the items
            uint32_t lo = 0, hi = a.nu;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                const uint64_t mk = a.wkey[mid], mt = a.wtxn[mid];
                if (mk < k || (mk == k && mt <= ob))
                    lo = mid + 1;
                else
                    hi = mid;
            }
            if (lo < a.nu && a.wkey[lo] == k && a.wtxn[lo] != r) {
                const size_t o = (size_t)a.nu + a.nops + a.cnt[a.np] + atomicAdd(&a.cur[a.np], 1u);
                const uint64_t row = ((uint64_t)r << 32) | a.wtxn[lo];
                a.ew[o] = row;
                if (a.et) a.et[o] = kDepRW, a.eg[o] = 0;
                back_row(a.diff, row);
            }
        }
    }
    const size_t s = (size_t)a.nu + i;
    a.ew[s] = wr;
    if (a.et) a.et[s] = kDepWR, a.eg[s] = 0;
    back_row(a.diff, wr);
}

__global__ __launch_bounds__(kRpThreads) void k_rp_join(RpArgs a, PairPack pp)
{
    __shared__ uint64_t sw[kRpLds];
    const uint32_t p = blockIdx.x;
    const uint32_t i0 = a.cnt[p], i1 = p + 1 < a.np ? a.cnt[p + 1] : a.cnt[a.np];
    if (i0 == i1) return;
    const uint64_t nb = (1ull << pp.D) + 1;  // dir entries [0, 2^D + 1]
    const uint32_t w0 = a.dir[min((uint64_t)p << a.ps, nb)];
    const uint32_t w1 = a.dir[min(((uint64_t)p + 1) << a.ps, nb)];
    const uint32_t n = w1 - w0;
    const bool lds = n <= kRpLds;
    if (lds)
        for (uint32_t j = threadIdx.x; j < n; j += kRpThreads) sw[j] = a.pk[w0 + j];
    __syncthreads();
    uint64_t tm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) tm[q] = pp.tmv[q];
    const uint64_t tmask = pp.tb >= 64 ? ~0ull : (1ull << pp.tb) - 1;
    for (uint32_t it = i0 + threadIdx.x; it < i1; it += kRpThreads) {
        const ulonglong2 q = a.items[it];
        const uint64_t x = q.x;
        const uint32_t r = (uint32_t)q.y;
        const bool strict = (q.y >> 32) & 1;
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t v = lds ? sw[mid] : a.pk[w0 + mid];
            if (strict ? v <= x : v < x)
                lo = mid + 1;
            else
                hi = mid;
        }
        uint64_t rw = ~0ull;
        const uint32_t g = w0 + lo;
        if (g < a.nu) {
            const uint64_t v = lo < n && lds ? sw[lo] : a.pk[g];
            const uint64_t kp = pp.tb >= 64 ? 0 : x >> pp.tb;
            if ((pp.tb >= 64 ? 0 : v >> pp.tb) == kp) {
                const uint32_t wt = (uint32_t)(bits_expand(v & tmask, pp.tm, tm) | pp.tc);
                if (wt != r) rw = ((uint64_t)r << 32) | wt;
            }
        }
        const size_t o = (size_t)a.nu + a.nops + it;
        a.ew[o] = rw;
        if (a.et) a.et[o] = kDepRW, a.eg[o] = 0;
        back_row(a.diff, rw);
    }
}

// Merge runs of equal edges (rows sorted, invalid ~0 rows at the end):
// head flag for the scan, types OR-ed into the head.
__global__ void k_edge_heads(size_t n, const uint64_t *ew, uint64_t *et, uint32_t *flags)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = ew[i];
    const bool head = e != ~0ull && (i == 0 || ew[i - 1] != e);
    flags[i] = head ? 1u : 0u;
    if (head) {
        uint64_t t = et[i];
        for (size_t j = i + 1; j < n && ew[j] == e; ++j) t |= et[j];
        et[i] = t;
    }
}

__global__ void k_edge_compact(size_t n, const uint64_t *ew, const uint64_t *et,
                               const uint32_t *pos, const uint32_t *flags_copy, uint32_t *src,
                               uint32_t *dst, uint32_t *type, int swap)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flags_copy[i]) return;
    const uint32_t p = pos[i];
    const uint64_t e = ew[i];
    const uint32_t a = (uint32_t)(e >> 32), b = (uint32_t)e;
    src[p] = swap ? b : a;
    dst[p] = swap ? a : b;
    if (type) type[p] = (uint32_t)et[i];
}

// off[v] = first edge whose key (sorted) is >= v, for v in [0, n]
__global__ void k_csr_offsets(size_t ne, const uint32_t *key, uint32_t nnodes, uint32_t *off)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > ne) return;
    const uint32_t cur = i < ne ? key[i] : nnodes;
    const uint32_t prev = i == 0 ? 0 : key[i - 1] + 1;
    if (i == 0)
        for (uint32_t v = 0; v <= cur && v <= nnodes; ++v) off[v] = 0;
    else
        for (uint32_t v = prev; v <= cur && v <= nnodes; ++v) off[v] = (uint32_t)i;
    if (i == ne)
        for (uint32_t v = cur; v <= nnodes; ++v) off[v] = (uint32_t)ne;
}

// ---- colouring SCC ----------------------------------------------------------
__global__ void k_scc_init(uint32_t n, uint32_t *scc, uint32_t *active)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    scc[v] = kNone;
    active[v] = 1;
}

// colour = id; frontier = live nodes with a live out-edge to a smaller id
__global__ void k_color_init(uint32_t n, const uint32_t *out_off, const uint32_t *out_dst,
                             const uint32_t *active, uint32_t *color, uint32_t *front,
                             uint32_t *nfront)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    if (!active[v]) return;
    color[v] = v;
    bool back = false;
    for (uint32_t e = out_off[v]; e < out_off[v + 1] && !back; ++e) {
        const uint32_t u = out_dst[e];
        back = u < v && active[u];
    }
    if (back) front[atomicAdd(nfront, 1u)] = v;
}

__global__ void k_color_step(const uint32_t *front, uint32_t nf, const uint32_t *out_off,
                             const uint32_t *out_dst, const uint32_t *active, uint32_t *color,
                             uint32_t *next, uint32_t *nnext)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nf) return;
    const uint32_t v = front[k];
    const uint32_t cv = __hip_atomic_load(&color[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t e = out_off[v]; e < out_off[v + 1]; ++e) {
        const uint32_t u = out_dst[e];
        if (!active[u]) continue;
        if (__hip_atomic_load(&color[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= cv) continue;
        const uint32_t old = atomicMax(&color[u], cv);
        if (old < cv) next[atomicAdd(nnext, 1u)] = u;
    }
}

// roots (colour == id) start the backward sweep
__global__ void k_bw_init(uint32_t n, const uint32_t *active, const uint32_t *color,
                          uint32_t *mark, uint32_t *front, uint32_t *nfront)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n || !active[v]) return;
    if (color[v] == v) {
        mark[v] = 1;
        front[atomicAdd(nfront, 1u)] = v;
    }
}

__global__ void k_bw_step(const uint32_t *front, uint32_t nf, const uint32_t *in_off,
                          const uint32_t *in_src, const uint32_t *active, const uint32_t *color,
                          uint32_t *mark, uint32_t *next, uint32_t *nnext)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nf) return;
    const uint32_t x = front[k];
    const uint32_t c = color[x];
    for (uint32_t e = in_off[x]; e < in_off[x + 1]; ++e) {
        const uint32_t w = in_src[e];
        if (!active[w] || color[w] != c) continue;
        if (__hip_atomic_load(&mark[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) continue;
        if (atomicExch(&mark[w], 1u) == 0) next[atomicAdd(nnext, 1u)] = w;
    }
}

__global__ void k_finalize(uint32_t n, uint32_t *active, const uint32_t *color, uint32_t *mark,
                           uint32_t *scc, uint32_t *remaining)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n || !active[v]) return;
    if (mark[v]) {
        scc[v] = color[v];
        active[v] = 0;
        mark[v] = 0;
    } else {
        atomicAdd(remaining, 1u);
    }
}

static inline unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }

// Edge rows g.ew/g.et/g.eg [0, ne_raw) (capacity ecap; invalid rows ~0) ->
// sorted unique out-edges (src, out_dst, type), in-edges (in_src, in_dst) and
// CSR / CSC offsets over nn nodes.
static hipError_t graph_rows_csr(size_t ne_raw, size_t ecap, uint32_t nn, GraphBufs &g,
                                 hipStream_t s)
{
    hipError_t e = hipSuccess;
#define CK(x)                                 \
    do {                                      \
        e = (x);                              \
        if (e != hipSuccess) return e;        \
    } while (0)
    // 3. sort by (src, dst), merge, compact: out-edges; then (dst, src): in-edges
    for (int pass = 0; pass < 2; ++pass) {
        DBuf *ew = &g.ew, *et = &g.et, *eg = &g.eg;
        if (pass == 1) {  // rebuild rows keyed (dst, src) from the compacted out-edges
            CK(hipMemcpyAsync(g.ew.p, g.swap_rows.p, 8 * g.ne, hipMemcpyDeviceToDevice, s));
            CK(hipMemsetAsync(g.et.p, 0, 8 * g.ne, s));
            CK(hipMemsetAsync(g.eg.p, 0, 4 * g.ne, s));
        }
        const size_t n = pass == 0 ? ne_raw : g.ne;
        CK(g.scratch.ensure(std::max(radix_scratch_bytes(n, 1), scan_scratch_bytes(n + 1) + 64)));
        bool a2 = false;
        CK(radix_sort_rows(1, n, eg->as<uint32_t>(), ew->as<uint64_t>(), et->as<uint64_t>(), ecap,
                           g.eg2.as<uint32_t>(), g.ew2.as<uint64_t>(), g.et2.as<uint64_t>(),
                           g.scratch.p, g.scratch.bytes, &a2, nullptr, s));
        const uint64_t *rw = a2 ? g.ew2.as<uint64_t>() : g.ew.as<uint64_t>();
        uint64_t *rt = a2 ? g.et2.as<uint64_t>() : g.et.as<uint64_t>();
        CK(g.flags.ensure(4 * (n + 64)));
        CK(g.flags2.ensure(4 * (n + 64)));
        if (n) k_edge_heads<<<blocks(n), 256, 0, s>>>(n, rw, rt, g.flags.as<uint32_t>());
        CK(hipMemsetAsync(g.flags.as<uint32_t>() + n, 0, 4, s));
        CK(hipMemcpyAsync(g.flags2.p, g.flags.p, 4 * (n + 1), hipMemcpyDeviceToDevice, s));
        CK(scan_exclusive_u32(g.flags.as<uint32_t>(), n + 1, g.scratch.as<uint32_t>(), s));
        uint32_t m = 0;
        CK(hipMemcpyAsync(&m, g.flags.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (pass == 0) {
            g.ne = m;
            CK(g.out_dst.ensure(4 * ((size_t)m + 1)));
            CK(g.src.ensure(4 * ((size_t)m + 1)));
            CK(g.type.ensure(4 * ((size_t)m + 1)));
            if (n)
                k_edge_compact<<<blocks(n), 256, 0, s>>>(n, rw, rt, g.flags.as<uint32_t>(),
                                                         g.flags2.as<uint32_t>(), g.src.as<uint32_t>(),
                                                         g.out_dst.as<uint32_t>(), g.type.as<uint32_t>(), 0);
            // rows for the in-edge pass: dst << 32 | src
            CK(g.swap_rows.ensure(8 * ((size_t)m + 1)));
            CK(swap_edge_words(m, g.src.as<uint32_t>(), g.out_dst.as<uint32_t>(),
                               g.swap_rows.as<uint64_t>(), s));
        } else {
            CK(g.in_src.ensure(4 * ((size_t)m + 1)));
            CK(g.in_dst.ensure(4 * ((size_t)m + 1)));
            if (n)
                k_edge_compact<<<blocks(n), 256, 0, s>>>(n, rw, rt, g.flags.as<uint32_t>(),
                                                         g.flags2.as<uint32_t>(), g.in_src.as<uint32_t>(),
                                                         g.in_dst.as<uint32_t>(), nullptr, 1);
        }
        CK(hipGetLastError());
    }
    // 4. CSR / CSC offsets
    CK(g.out_off.ensure(4 * ((size_t)nn + 1)));
    CK(g.in_off.ensure(4 * ((size_t)nn + 1)));
    k_csr_offsets<<<blocks(g.ne + 1), 256, 0, s>>>(g.ne, g.src.as<uint32_t>(), nn, g.out_off.as<uint32_t>());
    k_csr_offsets<<<blocks(g.ne + 1), 256, 0, s>>>(g.ne, g.in_dst.as<uint32_t>(), nn, g.in_off.as<uint32_t>());
    CK(hipGetLastError());
#undef CK
    return hipSuccess;
}

// out = {distinct writers, wkey[0], wtxn[0], pk[0], pk[nu - 1]} (pk null: 0s)
__global__ void k_graph_meta(const uint32_t *count, const uint64_t *wkey, const uint64_t *wtxn, const uint64_t *pk,
                             uint64_t *out, uint32_t *ebad)
{
    if (threadIdx.x != 0) return;
    ebad[0] = 0;
    ebad[-1] = 0;  // (the backward-row list's count)
    const uint32_t nu = count[0];
    out[0] = nu;
    out[1] = nu ? wkey[0] : 0;
    out[2] = nu ? wtxn[0] : 0;
    out[3] = nu && pk ? pk[0] : 0;
    out[4] = nu && pk ? pk[nu - 1] : 0;
}

hipError_t graph_build(const GraphInput &in, GraphBufs &g, bool full, hipStream_t s)
{
    hipError_t e = hipSuccess;
#define CK(x)                                 \
    do {                                      \
        e = (x);                              \
        if (e != hipSuccess) return e;        \
    } while (0)
    const size_t nops = in.nops;
    // 1. writers -> unique sorted (key, txn); room for every op (the count
    // comes back with the gather)
    const size_t wcap = std::max<size_t>(64, (nops + 63) & ~(size_t)63);
    CK(g.wg.ensure(4 * wcap));
    CK(g.ww.ensure(16 * wcap));
    CK(g.wl.ensure(8 * wcap));
    CK(g.wg2.ensure(4 * wcap));
    CK(g.ww2.ensure(16 * wcap));
    CK(g.wl2.ensure(8 * wcap));
    const size_t gwb = (nops + kGwThreads * kGwItems - 1) / (kGwThreads * kGwItems);
    // the partitioned read search (A/B, HSC_GRAPH_RP=1) does not check the
    // observed ids: the count pass does then (else the edge pass, guarded)
    static const bool rp_env = getenv("HSC_GRAPH_RP") != nullptr && atoi(getenv("HSC_GRAPH_RP")) != 0;
    const bool obs_in_count = rp_env;
    CK(g.flags.ensure(4 * (gwb + 2)));
    CK(g.gvary.ensure(32 * (gwb + 3)));
    CK(g.scratch.ensure(std::max(scan_scratch_bytes(gwb + 1), (size_t)1024)));
    uint32_t *bc = g.flags.as<uint32_t>();
    CK(hipMemsetAsync(bc + gwb, 0, 8, s));  // the total slot and the check's bits
    if (gwb)
        k_gw_count<<<(unsigned)gwb, kGwThreads, 0, s>>>(nops, in.is_write, bc, in.observed, in.ntxn,
                                                         in.check && obs_in_count ? bc + gwb + 1 : nullptr);
    CK(scan_exclusive_u32(bc, gwb + 1, g.scratch.as<uint32_t>(), s));
    if (gwb)
        k_gw_place<<<(unsigned)gwb, kGwThreads, 0, s>>>(nops, in.txn, in.key, in.is_write, bc, g.wg.as<uint32_t>(),
                                                         g.ww.as<uint64_t>(), wcap, in.ntxn,
                                                         in.check ? bc + gwb + 1 : nullptr, g.gvary.as<uint64_t>());
    uint64_t *dvary = g.gvary.as<uint64_t>() + 4 * gwb;
    k_vary_reduce<<<1, 1024, 0, s>>>((uint32_t)gwb, g.gvary.as<uint64_t>(), dvary, bc + gwb);
    CK(hipGetLastError());
    // the writers' varying bits (key, txn, gid), the key / txn ANDs, the
    // writer count and the check's bits
    uint64_t hvary[7] = {0, 0, 0, 0, 0, 0, 0};
    CK(hipMemcpyAsync(hvary, dvary, sizeof hvary, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    const uint32_t nwb[2] = {(uint32_t)hvary[5], (uint32_t)hvary[6]};
    const uint32_t nw = nwb[0];
    g.bad = in.check ? nwb[1] : 0;
    if (g.bad & 1) return hipErrorInvalidValue;  // an op out of range: the caller reports it
    const bool txn_sorted = in.check ? !(g.bad & 2) : in.txn_sorted;
    size_t rsb = std::max(radix_scratch_bytes(nw, 2), scan_scratch_bytes(nw) + 64);
    rsb = std::max(rsb, packed_scratch_bytes(nw));
    CK(g.scratch.ensure(rsb));
    CK(g.count.ensure(128));  // (+ the meta words below)
    // (key, txn) pairs whose varying bits fit 64 sort as single words, the
    // pair itself being the key (no row index, nothing to gather): one 8-byte
    // read + write per pass and varying byte, the dedupe fused into the
    // unpack (hsc_ingest.hip).  Else the whole-row sort + dedupe.
    uint64_t vary[3] = {~0ull, ~0ull, ~0ull};
    PackPlan P{};
    bool packed = false;
    if (nw) {
        for (int j = 0; j < 3; ++j) vary[j] = hvary[j];
        packed = packed_plan(2, nw, vary, &P, false);
        // writers gathered in op order from txn-ordered ops are ordered by
        // txn already: the stable passes need only the key bits (config 4:
        // 3 passes instead of 6)
        static const bool no_skip = getenv("HSC_GRAPH_NO_TXN_SKIP") != nullptr;  // (A/B)
        if (packed && txn_sorted && !no_skip && P.nl > 0 && P.limb[P.nl - 1] == 1) P.skip = P.bits[P.nl - 1];
    }
    // the packed writers' layout (PairPack's key / txn bits) is known from the
    // place pass's masks: a raw build's ww rows come out of the sort's unpack
    // (edge slots [0, nu); capacity for every writer)
    PairPack pp{};
    if (packed) {
        pp.km = vary[0], pp.tm = vary[1];
        pp.kc = hvary[3] & ~pp.km, pp.tc = hvary[4] & ~pp.tm;  // (constant bits: the place pass's ANDs)
        compress_moves(pp.km, pp.kmv);
        compress_moves(pp.tm, pp.tmv);
        pp.tb = __builtin_popcountll(pp.tm);
    }
    static const bool no_ww_fuse = getenv("HSC_GRAPH_NO_WW_FUSE") != nullptr;  // (A/B)
    const bool ww_fused = packed && nops && !full && !in.n_extra && !rp_env && !no_ww_fuse;
    if (ww_fused) {
        const size_t ecap0 = std::max<size_t>(64, ((size_t)nw + 2 * nops + 63) & ~(size_t)63);
        CK(g.ew.ensure(8 * ecap0));
    }
    DBuf *dw = &g.ww2;
    uint64_t *lsn_d = nullptr;  // packed: the distinct packed keys themselves (no LSN input, I = 0)
    // the packed build reads its writers as the packed keys alone (the ww
    // rows, the searches and their fallbacks): the distinct rows are written
    // for the partitioned search's A/B only
    const bool writer_rows = !packed || rp_env;
    if (packed) {
        CK(packed_sort_dedupe(P, nw, g.wg.as<uint32_t>(), g.ww.as<uint64_t>(), nullptr, wcap,
                              g.wl.as<uint64_t>(), g.wl2.as<uint64_t>(), nullptr, nullptr, nullptr, 0,
                              writer_rows ? g.wg2.as<uint32_t>() : nullptr, g.ww2.as<uint64_t>(), wcap, &lsn_d,
                              g.count.as<uint32_t>(), g.scratch.p, g.scratch.bytes, s,
                              g.count.as<uint32_t>() + 28,  // (its stall flag: read after the build)
                              ww_fused ? g.ew.as<uint64_t>() : nullptr, ww_fused ? &pp : nullptr));
    } else {
        bool alt = false;
        if (nw) CK(hipMemsetAsync(g.wl.p, 0, 8 * (size_t)nw, s));  // (k_gw_place writes no LSNs)
        CK(radix_sort_rows(2, nw, g.wg.as<uint32_t>(), g.ww.as<uint64_t>(), g.wl.as<uint64_t>(), wcap,
                           g.wg2.as<uint32_t>(), g.ww2.as<uint64_t>(), g.wl2.as<uint64_t>(),
                           g.scratch.p, g.scratch.bytes, &alt, nullptr, s));
        DBuf *sg = alt ? &g.wg2 : &g.wg, *sw = alt ? &g.ww2 : &g.ww, *sl = alt ? &g.wl2 : &g.wl;
        DBuf *dg = alt ? &g.wg : &g.wg2, *dl = alt ? &g.wl : &g.wl2;
        dw = alt ? &g.ww : &g.ww2;
        CK(g.flags.ensure(4 * (wcap + 64)));
        CK(dedupe_rows(2, nw, sg->as<uint32_t>(), sw->as<uint64_t>(), sl->as<uint64_t>(), wcap,
                       dg->as<uint32_t>(), dw->as<uint64_t>(), dl->as<uint64_t>(), wcap,
                       g.flags.as<uint32_t>(), g.scratch.p, g.scratch.bytes, g.count.as<uint32_t>(), s));
    }
    g.writer_packed = packed;
    g.ww_pk = false;
    const uint64_t *wkey = dw->as<uint64_t>(), *wtxn = dw->as<uint64_t>() + wcap;
    // the distinct count with what the packed search's parameters need -- the
    // first writer row, the first and last packed writer -- in one read
    uint64_t meta[5] = {0, 0, 0, 0, 0};
    // (the edge pass's check word, g.count's u32 30, cleared by the same kernel)
    uint32_t *ebad = g.count.as<uint32_t>() + 30;
    const uint32_t chk_n = in.check && !obs_in_count ? std::max<uint32_t>(in.ntxn, 1) : 0;
    g.edge_bad = chk_n ? ebad : nullptr;
    g.post = g.count.as<uint32_t>() + 29;  // [-1] the writer sort's stall flag, [0] backward rows
                                           // listed, [1] the edge check's bits
    k_graph_meta<<<1, 64, 0, s>>>(g.count.as<uint32_t>(), wkey, wtxn, packed ? lsn_d : nullptr,
                                  g.count.as<uint64_t>() + 8, ebad);
    CK(hipMemcpyAsync(meta, g.count.as<uint64_t>() + 8, sizeof meta, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    uint32_t nu = nw ? (uint32_t)meta[0] : 0;
    // 2. edges (capacity for the widest layout: nu + 2 nops + extras)
    const size_t ne_cap = (size_t)nu + 2 * nops + in.n_extra;
    const size_t ecap = std::max<size_t>(64, (ne_cap + 63) & ~(size_t)63);
    size_t rw_rows = 0;
    bool slot_layout = false, diff_done = false, back_listed = false;
    CK(g.ew.ensure(8 * ecap));
    CK(g.et.ensure(8 * ecap));
    CK(g.eg.ensure(4 * ecap));
    CK(g.ew2.ensure(8 * ecap));
    CK(g.et2.ensure(8 * ecap));
    CK(g.eg2.ensure(4 * ecap));
    uint64_t *et = full || in.n_extra ? g.et.as<uint64_t>() : nullptr;  // raw: rows only
    uint32_t *eg = full || in.n_extra ? g.eg.as<uint32_t>() : nullptr;
    if (nu && !(packed && nops)) k_edges_ww<<<blocks(nu), 256, 0, s>>>(nu, wkey, wtxn, g.ew.as<uint64_t>(), et, eg);
    if (nops && packed && nu) {
        // about kPer writers per bucket, at most 2^kDMax buckets (diagnostics:
        // HSC_GRAPH_DIR = "per,dmax").  Config 4 (33M writers, r05o): 32 / 2^20
        // 11.2 ms per step, 8 / 2^23 10.4 ms (a read's search touches the
        // directory line and one line of pk instead of ~3), 4 / 2^24 10.4,
        // 2 / 2^25 10.6 (the directory's own build grows)
        // bucket lines of kLine words (HSC_GRAPH_PT_LINE = 8 | 16, an A/B):
        // twice the writers per bucket with the 128-byte lines -- slower
        // (r06x, config 4: the search 2.28 -> 2.62 ms; a random 64-byte line
        // costs less than a 128-byte one, the overflow searches saved less)
        static int kPer = 8, kDMax = 23, kLine = 8;
        static const bool env_read = [] {
            if (const char *v = getenv("HSC_GRAPH_PT_LINE")) kLine = atoi(v) == 16 ? 16 : 8;
            if (kLine == 16) kPer = 16, kDMax = 22;
            if (const char *v = getenv("HSC_GRAPH_DIR")) sscanf(v, "%d,%d", &kPer, &kDMax);
            return true;
        }();
        (void)env_read;
        pp.D = 1;
        while (pp.D < kDMax && ((size_t)kPer << pp.D) < nu) ++pp.D;
        CK(g.pdir.ensure(4 * (((size_t)1 << pp.D) + 2)));
        // the sort's unpack left the distinct packed keys -- compress(key) <<
        // tb | compress(txn), the same words (no gid limb: gid is 0) -- in lsn_d
        const uint64_t *pkv = lsn_d;
        if (!pkv) return hipErrorInvalidValue;  // (a packed sort leaves them)
        pp.base = meta[3], pp.last = meta[4];
        if (!ww_fused) k_edges_ww_pk<<<blocks(nu), 256, 0, s>>>(nu, pkv, pp, g.ew.as<uint64_t>(), et, eg);
        g.ww_pk = true, g.pp = pp, g.ppk = pkv, g.pnu = nu;  // (graph_cut: ww rows by their source)
        pp.shift = 0;  // (last - base) >> shift < 2^D
        while (pp.shift < 64 && ((pp.last - pp.base) >> pp.shift) >= ((uint64_t)1 << pp.D)) ++pp.shift;
        k_pair_dir<<<blocks(((size_t)1 << pp.D) + 2), 256, 0, s>>>(nu, pkv, pp, g.pdir.as<uint32_t>());
        // the partitioned read search: measured slower on config 4 (r06c trace:
        // count 3.0 + scatter 3.2 + join 1.0 ms against 3.5 ms for the
        // directory search -- the count's per-read global atomics on 16k
        // partition counters), so off unless HSC_GRAPH_RP=1 (A/B)
        const bool rp = rp_env;
        // bucket lines (HSC_GRAPH_PT=0: the directory + pk search, an A/B)
        static const bool pt = getenv("HSC_GRAPH_PT") == nullptr || atoi(getenv("HSC_GRAPH_PT")) != 0;
        // raw builds (the sharded SCC's): the cover's backward-edge diffs as
        // the rows are emitted (ww rows are forward: txns ascend inside a key)
        uint32_t *diff = nullptr;
        BackSink sink{nullptr, nullptr, nullptr, 0};
        if (!full && !in.n_extra && in.ntxn) {
            if (rp) {  // (the partitioned search's kernels: the diffs)
                CK(g.diff.ensure(4 * ((size_t)in.ntxn + 2)));
                CK(hipMemsetAsync(g.diff.p, 0, 4 * ((size_t)in.ntxn + 2), s));
                diff = g.diff.as<uint32_t>();
                diff_done = true;
            } else {  // the rows themselves (the counter: g.count's u32 29, cleared by k_graph_meta)
                // (HSC_GRAPH_BACK_CAP: a smaller list, read per build -- the
                // tests' way to the diff fallback)
                uint32_t cap = kBackCap;
                if (const char *v = getenv("HSC_GRAPH_BACK_CAP")) cap = std::min<uint32_t>(kBackCap, (uint32_t)atoi(v));
                CK(g.back.ensure(8 * (size_t)std::max<uint32_t>(cap, 1)));
                sink = BackSink{nullptr, g.back.as<uint64_t>(), g.count.as<uint32_t>() + 29, cap};
                g.back_cap = cap;
                back_listed = true;
            }
        }
        if (rp) {
            RpArgs a{};
            a.nops = nops, a.txn = in.txn, a.key = in.key, a.is_write = in.is_write, a.observed = in.observed;
            a.nu = nu, a.wkey = wkey, a.wtxn = wtxn, a.pk = pkv, a.dir = g.pdir.as<uint32_t>();
            a.ps = pp.D > kRpBitsMax ? (uint32_t)(pp.D - kRpBitsMax) : 0;
            a.np = (uint32_t)((((uint64_t)1 << pp.D) >> a.ps) + 1);
            CK(g.rp_cnt.ensure(8 * ((size_t)a.np + 2)));
            a.cnt = g.rp_cnt.as<uint32_t>();
            a.cur = a.cnt + a.np + 1;
            CK(g.rp_items.ensure(16 * std::max<size_t>(nops, 1)));
            a.items = g.rp_items.as<ulonglong2>();
            a.ew = g.ew.as<uint64_t>(), a.et = et, a.eg = eg, a.skip_rw = in.skip_rw ? 1 : 0;
            a.diff = diff;
            CK(hipMemsetAsync(a.cnt, 0, 4 * ((size_t)a.np + 1), s));
            k_rp_count<<<blocks(nops), kRpThreads, 0, s>>>(a, pp);
            k_rp_scan<<<1, 1024, 0, s>>>(a);
            k_rp_scatter<<<blocks(nops), kRpThreads, 0, s>>>(a, pp);
            k_rp_join<<<a.np, kRpThreads, 0, s>>>(a, pp);
            CK(hipGetLastError());
            uint32_t tot[2];
            CK(hipMemcpyAsync(&tot[0], a.cnt + a.np, 4, hipMemcpyDeviceToHost, s));
            CK(hipMemcpyAsync(&tot[1], a.cur + a.np, 4, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            rw_rows = (size_t)tot[0] + tot[1];
            slot_layout = true;
        } else if (pt && pp.shift <= 31) {  // (a bucket's offsets fit 32 bits)
            const uint64_t nb = ((uint64_t)1 << pp.D) + 1;
            CK(g.ptab.ensure(8 * (size_t)kLine * nb));
            // (HSC_GRAPH_NT=0: cached op loads and row stores, an A/B)
            static const bool nt = getenv("HSC_GRAPH_NT") == nullptr || atoi(getenv("HSC_GRAPH_NT")) != 0;
#define HSC_PT(LW_, NT_)                                                                                  \
    k_pair_table<LW_><<<blocks(LW_ * nb), 256, 0, s>>>(nu, pkv, g.pdir.as<uint32_t>(), nb, pp,              \
                                                       g.ptab.as<uint64_t>());                             \
    k_edges_reads_pt<LW_, NT_><<<blocks(nops), 256, 0, s>>>(nops, in.txn, in.key, in.is_write, in.observed, \
                                                            nu, wkey, wtxn, pkv, g.ptab.as<uint64_t>(), pp, \
                                                            g.ew.as<uint64_t>(), et, eg, in.skip_rw ? 1 : 0, \
                                                            sink, chk_n, ebad)
            if (kLine == 16) {
                HSC_PT(16, false);
            } else if (nt) {
                HSC_PT(8, true);
            } else {
                HSC_PT(8, false);
            }
#undef HSC_PT
        } else {
            k_edges_reads_pk<<<blocks(nops), 256, 0, s>>>(nops, in.txn, in.key, in.is_write, in.observed, nu,
                                                          wkey, wtxn, pkv, g.pdir.as<uint32_t>(),
                                                          pp, g.ew.as<uint64_t>(), et, eg, in.skip_rw ? 1 : 0,
                                                          sink, chk_n, ebad);
        }
    } else if (nops) {
        k_edges_reads<<<blocks(nops), 256, 0, s>>>(nops, in.txn, in.key, in.is_write, in.observed,
                                                   nu, wkey, wtxn, g.ew.as<uint64_t>(), et, eg,
                                                   in.skip_rw ? 1 : 0, chk_n, ebad);
    }
    CK(hipGetLastError());
    // the partitioned search filled [nu, nu + nops + rw_rows) (else [nu, nu + 2 nops))
    const size_t ne_hist = slot_layout ? (size_t)nu + nops + rw_rows : (size_t)nu + 2 * nops;
    const size_t ne_raw = ne_hist + in.n_extra;
    if (in.n_extra) {  // staged edges (rw pairs of the validator's join) after the history's
        const size_t o = ne_hist;
        CK(hipMemcpyAsync(g.ew.as<uint64_t>() + o, in.x_rows, 8 * in.n_extra,
                          hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(g.et.as<uint64_t>() + o, in.x_type, 8 * in.n_extra,
                          hipMemcpyDeviceToDevice, s));
        CK(hipMemsetAsync(g.eg.as<uint32_t>() + o, 0, 4 * in.n_extra, s));
    }
    g.raw = !full;
    g.ne_raw = ne_raw;
    g.op_cut = !full && !slot_layout && txn_sorted;
    g.op_at = nu, g.op_n = nops, g.x_at = ne_hist, g.x_n = in.n_extra;
    g.diff_nn = diff_done ? in.ntxn : 0;  // graph_cover: the diffs are there already
    g.back_listed = back_listed;          // graph_cover: the backward rows (count: graph_build_timed)
    g.back_n = 0;
    g.cover_nn = in.ntxn;
    if (!full) {  // raw edge rows only (duplicates, ~0 holes): enough for cover / cut
        g.ne = 0;
        return hipSuccess;
    }
    CK(graph_rows_csr(ne_raw, ecap, in.ntxn, g, s));
#undef CK
    return hipSuccess;
}

__global__ void k_pairs_rows(size_t n, const uint32_t *txn, const uint64_t *lsn, uint32_t nrs,
                             const uint32_t *rs_txn, size_t ncommit, const uint64_t *commit_lsn,
                             const uint32_t *commit_txn, uint64_t *rows, uint64_t *type,
                             uint32_t *bad)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t c = lsn[i];
    size_t lo = 0, hi = ncommit;
    while (lo < hi) {
        const size_t mid = (lo + hi) >> 1;
        if (commit_lsn[mid] < c)
            lo = mid + 1;
        else
            hi = mid;
    }
    const uint32_t t = txn[i];
    uint64_t row = ~0ull;
    if (lo == ncommit || commit_lsn[lo] != c || t >= nrs) {
        atomicOr(bad, 1u);
    } else {
        const uint32_t a = rs_txn[t], b = commit_txn[lo];
        if (a != b) row = ((uint64_t)a << 32) | b;
    }
    rows[i] = row;
    type[i] = kDepRW;
}

hipError_t graph_pairs_rows(size_t n, const uint32_t *txn, const uint64_t *lsn, uint32_t nrs,
                            const uint32_t *rs_txn, size_t ncommit, const uint64_t *commit_lsn,
                            const uint32_t *commit_txn, uint64_t *rows, uint64_t *type,
                            uint32_t *bad, hipStream_t s)
{
    if (n)
        k_pairs_rows<<<blocks(n), 256, 0, s>>>(n, txn, lsn, nrs, rs_txn, ncommit, commit_lsn,
                                               commit_txn, rows, type, bad);
    return hipGetLastError();
}

__global__ void k_swap_words(uint32_t m, const uint32_t *src, const uint32_t *dst, uint64_t *rows)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) rows[i] = ((uint64_t)dst[i] << 32) | src[i];
}

hipError_t swap_edge_words(uint32_t m, const uint32_t *src, const uint32_t *dst, uint64_t *rows,
                           hipStream_t s)
{
    if (m) k_swap_words<<<blocks(m), 256, 0, s>>>(m, src, dst, rows);
    return hipGetLastError();
}

hipError_t graph_scc(uint32_t nn, GraphBufs &g, uint32_t *rounds, uint32_t *iterations,
                     hipStream_t s)
{
    hipError_t e = hipSuccess;
#define CK(x)                                 \
    do {                                      \
        e = (x);                              \
        if (e != hipSuccess) return e;        \
    } while (0)
    *rounds = *iterations = 0;
    if (nn == 0) return hipSuccess;
    CK(g.scc.ensure(4 * (size_t)nn));
    CK(g.active.ensure(4 * (size_t)nn));
    CK(g.color.ensure(4 * (size_t)nn));
    CK(g.mark.ensure(4 * (size_t)nn));
    CK(g.front.ensure(4 * (size_t)nn + 64));
    CK(g.front2.ensure(4 * (size_t)nn + 64));
    CK(g.count.ensure(64));
    CK(hipMemsetAsync(g.mark.p, 0, 4 * (size_t)nn, s));
    k_scc_init<<<blocks(nn), 256, 0, s>>>(nn, g.scc.as<uint32_t>(), g.active.as<uint32_t>());
    uint32_t *cnt = g.count.as<uint32_t>();
    uint32_t h[4];
    for (;;) {
        ++*rounds;
        // forward colouring
        CK(hipMemsetAsync(cnt, 0, 16, s));
        k_color_init<<<blocks(nn), 256, 0, s>>>(nn, g.out_off.as<uint32_t>(), g.out_dst.as<uint32_t>(),
                                                g.active.as<uint32_t>(), g.color.as<uint32_t>(),
                                                g.front.as<uint32_t>(), cnt);
        CK(hipMemcpyAsync(h, cnt, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        uint32_t nf = h[0];
        uint32_t *f = g.front.as<uint32_t>(), *f2 = g.front2.as<uint32_t>();
        while (nf) {
            ++*iterations;
            CK(hipMemsetAsync(cnt + 1, 0, 4, s));
            k_color_step<<<blocks(nf), 256, 0, s>>>(f, nf, g.out_off.as<uint32_t>(), g.out_dst.as<uint32_t>(),
                                                    g.active.as<uint32_t>(), g.color.as<uint32_t>(), f2,
                                                    cnt + 1);
            CK(hipMemcpyAsync(h, cnt + 1, 4, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            nf = h[0];
            std::swap(f, f2);
        }
        // backward sweep from the roots
        CK(hipMemsetAsync(cnt, 0, 16, s));
        k_bw_init<<<blocks(nn), 256, 0, s>>>(nn, g.active.as<uint32_t>(), g.color.as<uint32_t>(),
                                             g.mark.as<uint32_t>(), g.front.as<uint32_t>(), cnt);
        CK(hipMemcpyAsync(h, cnt, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        nf = h[0];
        f = g.front.as<uint32_t>();
        f2 = g.front2.as<uint32_t>();
        while (nf) {
            ++*iterations;
            CK(hipMemsetAsync(cnt + 1, 0, 4, s));
            k_bw_step<<<blocks(nf), 256, 0, s>>>(f, nf, g.in_off.as<uint32_t>(), g.in_src.as<uint32_t>(),
                                                 g.active.as<uint32_t>(), g.color.as<uint32_t>(),
                                                 g.mark.as<uint32_t>(), f2, cnt + 1);
            CK(hipMemcpyAsync(h, cnt + 1, 4, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            nf = h[0];
            std::swap(f, f2);
        }
        CK(hipMemsetAsync(cnt + 2, 0, 4, s));
        k_finalize<<<blocks(nn), 256, 0, s>>>(nn, g.active.as<uint32_t>(), g.color.as<uint32_t>(),
                                              g.mark.as<uint32_t>(), g.scc.as<uint32_t>(), cnt + 2);
        CK(hipMemcpyAsync(h, cnt + 2, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (h[0] == 0) break;
        if (*rounds > nn) return hipErrorUnknown;  // cannot happen: every round retires >= 1 node
    }
#undef CK
    return hipSuccess;
}


// ---- sharded SCC: cover, cut, SCC of the cut --------------------------------
// Txn ids are commit order.  Every node of a cycle lies inside [dst, src] of
// one of the cycle's backward (src > dst) edges, so only nodes
// covered by a backward edge's interval can share a component: the SCCs of
// the graph induced on covered nodes are the nontrivial SCCs of the whole
// graph, and every other node is its own component.  Shards (histories split
// by key: all WW/WR/RW edges are per key) OR their covers, exchange only the
// edges between covered nodes, and run the colouring on that small graph.

// Edge i of a graph: raw rows (src << 32 | dst, ~0 = none) or sorted arrays.
struct EdgeSet {
    const uint64_t *rows;  // raw build, else nullptr
    const uint32_t *src, *dst;
    size_t n;
    __device__ __forceinline__ bool get(size_t i, uint32_t &a, uint32_t &b) const
    {
        if (rows) {
            const uint64_t r = rows[i];
            a = (uint32_t)(r >> 32);
            b = (uint32_t)r;
            return r != ~0ull;
        }
        a = src[i];
        b = dst[i];
        return true;
    }
};

static EdgeSet edge_set(const GraphBufs &g)
{
    if (g.raw) return EdgeSet{g.ew.as<uint64_t>(), nullptr, nullptr, g.ne_raw};
    return EdgeSet{nullptr, g.src.as<uint32_t>(), g.out_dst.as<uint32_t>(), g.ne};
}

__global__ void k_back_diff(EdgeSet es, uint32_t *diff)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= es.n) return;
    uint32_t a, b;
    if (es.get(i, a, b) && a > b) {
        atomicAdd(&diff[b], 1u);
        atomicAdd(&diff[a + 1], 0xFFFFFFFFu);  // -1 mod 2^32: prefix sums stay >= 0
    }
}

// ex = exclusive scan of the interval diffs: node v is covered iff ex[v + 1] != 0
__global__ void k_cover_flags(uint32_t nn, const uint32_t *ex, uint8_t *cover)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < nn) cover[v] = ex[v + 1] != 0;
}

__global__ void k_cut_flags(EdgeSet es, const uint8_t *cover, uint32_t *flags)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= es.n) return;
    uint32_t a, b;
    flags[i] = es.get(i, a, b) && cover[a] && cover[b];
}

__global__ void k_cut_rows(EdgeSet es, const uint8_t *cover, const uint32_t *pos, uint64_t *rows)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= es.n) return;
    uint32_t a, b;
    if (es.get(i, a, b) && cover[a] && cover[b]) rows[pos[i]] = ((uint64_t)a << 32) | b;
}

// counts[0..2] += edges carrying the ww / wr / rw bit
__global__ void k_type_counts(size_t ne, const uint32_t *type, unsigned long long *counts)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t t = i < ne ? type[i] : 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t m = __ballot((t >> k) & 1u);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&counts[k], (unsigned long long)__popcll(m));
    }
}

hipError_t graph_type_counts(GraphBufs &g, uint64_t out[3], hipStream_t s)
{
    hipError_t e = g.count.ensure(64);
    if (e != hipSuccess) return e;
    unsigned long long *c = (unsigned long long *)(g.count.as<uint32_t>() + 16);
    if ((e = hipMemsetAsync(c, 0, 24, s)) != hipSuccess) return e;
    if (g.ne) k_type_counts<<<blocks(g.ne), 256, 0, s>>>(g.ne, g.type.as<uint32_t>(), c);
    if ((e = hipMemcpyAsync(out, c, 24, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

// The cut's node ids from the cover as a bitmap: word w's bits and their
// exclusive count wc[w] (a scan of nn / 64 words, not of nn) -- covered v is
// cut node wc[v / 64] + (its bit's rank in its word)
__global__ void k_cover_words(uint32_t nn, const uint8_t *cover, uint64_t *bits, uint32_t *wc)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = __ballot(v < nn && cover[v] != 0);
    if ((threadIdx.x & 63) == 0 && v < nn) bits[v >> 6] = m, wc[v >> 6] = (uint32_t)__popcll(m);
}

__device__ __forceinline__ bool cover_has(const uint64_t *bits, uint32_t v) { return (bits[v >> 6] >> (v & 63)) & 1; }

__device__ __forceinline__ uint32_t cover_id(const uint64_t *bits, const uint32_t *wc, uint32_t v)
{
    return wc[v >> 6] + (uint32_t)__popcll(bits[v >> 6] & ((1ull << (v & 63)) - 1));
}

// txn_of[cut id] = txn, a thread per bitmap word
__global__ void k_txn_of_w(uint32_t nw, const uint64_t *bits, const uint32_t *wc, uint32_t *txn_of)
{
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    uint64_t m = bits[w];
    uint32_t id = wc[w];
    while (m) {
        txn_of[id++] = w * 64 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
        m &= m - 1;
    }
}

// cut rows (txn ids; ~0 = padding) -> edge rows over cut node ids
__global__ void k_relabel(size_t m, uint32_t nn, const uint64_t *rows, const uint64_t *bits,
                          const uint32_t *wc, uint64_t *ew, uint64_t *et, uint32_t *eg,
                          uint32_t *bad)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t r = rows[i];
    uint64_t e = ~0ull;
    if (r != ~0ull) {
        const uint32_t a = (uint32_t)(r >> 32), b = (uint32_t)r;
        if (a < nn && b < nn && cover_has(bits, a) && cover_has(bits, b) && a != b)
            e = ((uint64_t)cover_id(bits, wc, a) << 32) | cover_id(bits, wc, b);
        else
            atomicOr(bad, 1u);
    }
    ew[i] = e;
    et[i] = 0;
    eg[i] = 0;
}

__global__ void k_scc_out(uint32_t nn, const uint64_t *bits, const uint32_t *wc, const uint32_t *sub_scc,
                          const uint32_t *txn_of, uint32_t *scc)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < nn) scc[v] = cover_has(bits, v) ? txn_of[sub_scc[cover_id(bits, wc, v)]] : v;
}

// one workgroup per listed backward row: its interval [b, a] marked covered
__global__ void k_mark_intervals(const uint64_t *list, uint32_t n, uint8_t *cover)
{
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        const uint64_t r = list[j];
        const uint32_t a = (uint32_t)(r >> 32), b = (uint32_t)r;
        for (uint32_t v = b + threadIdx.x; v <= a; v += blockDim.x) cover[v] = 1;
    }
}

hipError_t graph_cover(GraphBufs &g, uint32_t nn, uint8_t *cover, hipStream_t s)
{
    hipError_t e = hipSuccess;
    if (nn == 0) return hipSuccess;
    if (g.raw && g.back_listed && g.cover_nn == nn && g.back_n <= g.back_cap) {
        // the listed backward rows' intervals (no diffs, no scan of nn)
        if ((e = hipMemsetAsync(cover, 0, nn, s)) != hipSuccess) return e;
        if (g.back_n)
            k_mark_intervals<<<std::min<uint32_t>(g.back_n, 65535), 256, 0, s>>>(g.back.as<uint64_t>(), g.back_n,
                                                                               cover);
        return hipGetLastError();
    }
    DBuf &diff = g.diff, &scratch = g.scratch;
    if ((e = diff.ensure(4 * ((size_t)nn + 2))) != hipSuccess) return e;
    if ((e = scratch.ensure(std::max(scan_scratch_bytes((size_t)nn + 1), (size_t)1024))) != hipSuccess)
        return e;
    if (!(g.raw && g.diff_nn == nn)) {  // (a raw build accumulated them while emitting its rows)
        if ((e = hipMemsetAsync(diff.p, 0, 4 * ((size_t)nn + 2), s)) != hipSuccess) return e;
        const EdgeSet es = edge_set(g);
        if (es.n) k_back_diff<<<blocks(es.n), 256, 0, s>>>(es, diff.as<uint32_t>());
    }
    g.diff_nn = 0;  // (the scan below consumes them)
    if ((e = scan_exclusive_u32(diff.as<uint32_t>(), (size_t)nn + 1, scratch.as<uint32_t>(), s)) !=
        hipSuccess)
        return e;
    k_cover_flags<<<blocks(nn), 256, 0, s>>>(nn, diff.as<uint32_t>(), cover);
    return hipGetLastError();
}

// One pass for the usual tiny cut: edges with both ends covered appended
// at a wave-aggregated atomic cursor (rows beyond cap are counted, not
// stored: the caller then takes the flag + scan path).
// The cover as a bitmap (bit v of word v / 64): 2 MB for 16.7M txns stays in
// L2, where the byte array's 16.7 MB did not (the cut tests both ends of
// every edge row).
__global__ void k_cover_bits(uint32_t nn, const uint8_t *cover, uint64_t *bits)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = __ballot(v < nn && cover[v] != 0);
    if ((threadIdx.x & 63) == 0 && v < nn) bits[v >> 6] = m;
}

__device__ __forceinline__ bool cover_bit(const uint64_t *bits, uint32_t v) { return (bits[v >> 6] >> (v & 63)) & 1; }

// (Measured on config 4's 233M raw rows, r06o: four rows per thread with
// both cover words of every row loaded together 1.02 ms against 0.67 ms for
// this form, which reads the second cover word only when the first bit is
// set -- 1179 of 16.7M txns are covered.)
__global__ void k_cut_append(EdgeSet es, const uint64_t *cover, uint64_t *rows, uint32_t *cnt, uint32_t cap)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = 0, b = 0;
    const bool hit = i < es.n && es.get(i, a, b) && cover_bit(cover, a) && cover_bit(cover, b);
    const uint64_t m = __ballot(hit);
    if (!m) return;
    const int lane = threadIdx.x & 63, first = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, first, 64);
    const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (hit && slot < cap) rows[slot] = ((uint64_t)a << 32) | b;
}

constexpr uint32_t kCutFastCap = 1u << 16;

constexpr uint32_t kCoverListCap = 1u << 16;
constexpr uint32_t kCutLanes = 8;  // k_cut_txn_ops lanes per covered txn

// the cover as a bitmap and as a list of its txns (wave-aggregated appends;
// past cap counted only)
__global__ void k_cover_list(uint32_t nn, const uint8_t *cover, uint64_t *bits, uint32_t *list,
                             uint32_t *cnt, uint32_t cap)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = v < nn && cover[v] != 0;
    const uint64_t m = __ballot(on);
    const int lane = threadIdx.x & 63;
    if (lane == 0 && v < nn) bits[v >> 6] = m;
    if (!m) return;
    const int first = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, first, 64);
    const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (on && slot < cap) list[slot] = v;
}

// one thread per covered txn t: its ops (txn-sorted: one run, found by a
// binary search) and their two rows each -- a cut row at op i has its reader
// t as one end, so a row whose txn is not covered is never in the cut
// pk != null: the ww rows too, from their source side -- a ww row j (writer
// j -> j + 1 of one key) is emitted by the covered txn of writer j, found
// by an exact search of pk for (key, txn) of each of its write ops (a txn's
// repeated write of a key: once) -- so no pass over the nu ww rows
__global__ void k_cut_txn_ops(const uint32_t *list, const uint32_t *lcnt, const uint32_t *op_txn, size_t nops,
                              const uint64_t *op_rows, const uint64_t *cover, uint64_t *rows, uint32_t *cnt,
                              uint32_t cap, const uint64_t *op_key, const uint8_t *op_isw, const uint64_t *pk,
                              uint32_t nu, const uint64_t *ww, PairPack pp)
{
    // kCutLanes lanes per covered txn: the first finds its ops' run, the
    // lanes take its ops in turn (a txn's ~6 ops' searches side by side
    // instead of one after another: 81 -> ~25 us for config 4's 1179 txns)
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t j = id / kCutLanes, sub = id % kCutLanes;
    if (j >= min(*lcnt, kCoverListCap)) return;  // (a whole group: its lanes share j)
    const uint32_t t = list[j];
    uint32_t lo = 0;
    if (sub == 0) {
        uint32_t hi = (uint32_t)nops;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (op_txn[mid] < t)
                lo = mid + 1;
            else
                hi = mid;
        }
    }
    lo = __shfl(lo, (int)(threadIdx.x & 63) & ~(kCutLanes - 1), 64);
    const size_t first = lo;
    for (size_t i = (size_t)lo + sub; i < nops && op_txn[i] == t; i += kCutLanes) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            uint64_t r = ~0ull;
            if (q < 2) {
                r = op_rows[2 * i + q];
            } else if (pk && op_isw[i]) {
                const uint64_t k = op_key[i];
                bool dup = false;
                for (size_t i2 = first; i2 < i && !dup; ++i2) dup = op_isw[i2] && op_key[i2] == k;
                if (!dup && (k & ~pp.km) == pp.kc && (t & ~pp.tm) == pp.tc) {
                    uint64_t km[6], tm[6];
#pragma unroll
                    for (int z = 0; z < 6; ++z) km[z] = pp.kmv[z], tm[z] = pp.tmv[z];
                    const uint64_t x =
                        (pp.tb >= 64 ? 0 : bits_compress(k, pp.km, km) << pp.tb) | bits_compress(t, pp.tm, tm);
                    uint32_t a = 0, h = nu;
                    while (a < h) {
                        const uint32_t mid = (a + h) >> 1;
                        if (pk[mid] < x)
                            a = mid + 1;
                        else
                            h = mid;
                    }
                    if (a < nu && pk[a] == x) r = ww[a];
                }
            }
            if (r == ~0ull) continue;
            const uint32_t a = (uint32_t)(r >> 32), b = (uint32_t)r;
            if (cover_bit(cover, a) && cover_bit(cover, b)) {
                const uint32_t slot = atomicAdd(cnt, 1u);
                if (slot < cap) rows[slot] = r;
            }
        }
    }
}

hipError_t graph_cut(GraphBufs &g, const uint8_t *cover, size_t *m, hipStream_t s, const uint32_t *op_txn,
                     const uint64_t *op_key, const uint8_t *op_isw, bool host_sort)
{
    hipError_t e = hipSuccess;
    const EdgeSet es = edge_set(g);
    const size_t ne = es.n;
    *m = 0;
    {
        // the usual tiny cut: one pass, then sorted on the host
        if ((e = g.cut.ensure(8 * (size_t)kCutFastCap)) != hipSuccess) return e;
        if ((e = g.count.ensure(64)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(g.count.p, 0, 8, s)) != hipSuccess) return e;
        const uint32_t nn = g.cover_nn;
        if ((e = g.cover_bits.ensure(8 * ((size_t)nn / 64 + 2))) != hipSuccess) return e;
        uint32_t k = 0;
        // by the covered txns' ops (config 4: 1179 covered of 16.7M txns --
        // the ww rows and ~7k op rows tested instead of all 233M rows), unless
        // the cover has more than kCoverListCap txns (then every row, below)
        static const bool no_op_cut = getenv("HSC_GRAPH_NO_OP_CUT") != nullptr;  // (A/B)
        bool done = false;
        if (op_txn && g.raw && g.op_cut && !no_op_cut && nn) {
            if ((e = g.cover_list.ensure(4 * (size_t)kCoverListCap)) != hipSuccess) return e;
            uint32_t *cnt = g.count.as<uint32_t>();  // [0] cut rows, [1] covered txns
            k_cover_list<<<blocks(nn), 256, 0, s>>>(nn, cover, g.cover_bits.as<uint64_t>(),
                                                    g.cover_list.as<uint32_t>(), cnt + 1, kCoverListCap);
            const uint64_t *ew = g.ew.as<uint64_t>();
            // the ww rows from the covered txns' write ops when the build's
            // writers are packed keys (else a pass over them)
            const bool ww_src = g.ww_pk && op_key && op_isw && g.op_at == g.pnu;
            if (g.op_at && !ww_src)
                k_cut_append<<<blocks(g.op_at), 256, 0, s>>>(EdgeSet{ew, nullptr, nullptr, g.op_at},
                                                             g.cover_bits.as<uint64_t>(), g.cut.as<uint64_t>(), cnt,
                                                             kCutFastCap);
            if (g.x_n)
                k_cut_append<<<blocks(g.x_n), 256, 0, s>>>(EdgeSet{ew + g.x_at, nullptr, nullptr, g.x_n},
                                                           g.cover_bits.as<uint64_t>(), g.cut.as<uint64_t>(), cnt,
                                                           kCutFastCap);
            if (g.op_n)
                k_cut_txn_ops<<<blocks((size_t)kCoverListCap * kCutLanes), 256, 0, s>>>(g.cover_list.as<uint32_t>(), cnt + 1, op_txn,
                                                                    g.op_n, ew + g.op_at, g.cover_bits.as<uint64_t>(),
                                                                    g.cut.as<uint64_t>(), cnt, kCutFastCap, op_key,
                                                                    op_isw, ww_src ? g.ppk : nullptr, g.pnu, ew,
                                                                    g.pp);
            uint32_t kc[2] = {0, 0};
            if ((e = hipMemcpyAsync(kc, g.count.p, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
            done = kc[1] <= kCoverListCap;
            if (done)
                k = kc[0];
            else if ((e = hipMemsetAsync(g.count.p, 0, 8, s)) != hipSuccess)
                return e;
        }
        if (!done) {
            if (nn) k_cover_bits<<<blocks(nn), 256, 0, s>>>(nn, cover, g.cover_bits.as<uint64_t>());
            if (ne)
                k_cut_append<<<blocks(ne), 256, 0, s>>>(es, g.cover_bits.as<uint64_t>(), g.cut.as<uint64_t>(),
                                                        g.count.as<uint32_t>(), kCutFastCap);
            if ((e = hipMemcpyAsync(&k, g.count.p, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        }
        if (k <= kCutFastCap) {
            std::vector<uint64_t> h(k);
            if (k && host_sort) {
                // both copies on the caller's stream, then a sync: a NULL-stream
                // hipMemcpy from pageable memory may return before its DMA
                // lands, and the next reader of the rows (k_relabel, the
                // multi step's copies) runs on a non-blocking stream
                if ((e = hipMemcpyAsync(h.data(), g.cut.p, 8 * (size_t)k, hipMemcpyDeviceToHost, s)) != hipSuccess)
                    return e;
                if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
                std::sort(h.begin(), h.end());
                if ((e = hipMemcpyAsync(g.cut.p, h.data(), 8 * (size_t)k, hipMemcpyHostToDevice, s)) != hipSuccess)
                    return e;
                if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
            }
            *m = k;
            return hipGetLastError();
        }
    }
    if ((e = g.flags.ensure(4 * (ne + 64))) != hipSuccess) return e;
    if ((e = g.scratch.ensure(std::max(scan_scratch_bytes(ne + 1), (size_t)1024))) != hipSuccess)
        return e;
    if (ne) k_cut_flags<<<blocks(ne), 256, 0, s>>>(es, cover, g.flags.as<uint32_t>());
    if ((e = hipMemsetAsync(g.flags.as<uint32_t>() + ne, 0, 4, s)) != hipSuccess) return e;
    if ((e = scan_exclusive_u32(g.flags.as<uint32_t>(), ne + 1, g.scratch.as<uint32_t>(), s)) !=
        hipSuccess)
        return e;
    uint32_t k = 0;
    if ((e = hipMemcpyAsync(&k, g.flags.as<uint32_t>() + ne, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    DBuf &rows = g.cut;
    if ((e = rows.ensure(8 * ((size_t)k + 1))) != hipSuccess) return e;
    if (ne) k_cut_rows<<<blocks(ne), 256, 0, s>>>(es, cover, g.flags.as<uint32_t>(), rows.as<uint64_t>());
    *m = k;
    return hipGetLastError();
}

// The SCC of a small cut in ONE workgroup, every array in LDS: the same
// colouring as graph_scc (colour = the largest id reaching a node, roots =
// nodes of their own colour, a backward sweep inside each colour; repeat on
// what is left), with edge sweeps instead of frontiers and barriers instead
// of host round trips (graph_scc: a launch, a copy and a stream sync per
// frontier step -- 1.4 ms for config 4's ~1k-node cut).  Rows: cut-id edges
// (a << 32 | b, ~0 = none).  Labels = the largest node id of each SCC, as
// graph_scc's.  out[0] rounds, out[1] sweeps.
constexpr uint32_t kSccSmallNodes = 4096, kSccSmallEdges = 24576;
constexpr int kSccSmallThreads = 1024;
__global__ __launch_bounds__(kSccSmallThreads) void k_scc_small(uint32_t nn, size_t m, const uint64_t *rows,
                                                               uint32_t *scc, uint32_t *out)
{
    __shared__ uint32_t E[kSccSmallEdges];  // a << 16 | b
    __shared__ uint32_t col[kSccSmallNodes];
    __shared__ uint8_t act[kSccSmallNodes], mk[kSccSmallNodes];
    __shared__ uint32_t ne, changed, left, rounds, sweeps;
    const uint32_t t = threadIdx.x;
    if (t == 0) ne = 0, rounds = 0, sweeps = 0;
    for (uint32_t v = t; v < nn; v += kSccSmallThreads) act[v] = 1, mk[v] = 0;
    __syncthreads();
    for (size_t i = t; i < m; i += kSccSmallThreads) {
        const uint64_t r = rows[i];
        if (r == ~0ull) continue;
        const uint32_t a = (uint32_t)(r >> 32), b = (uint32_t)r;
        if (a >= nn || b >= nn || a == b) continue;
        E[atomicAdd(&ne, 1u)] = a << 16 | b;
    }
    __syncthreads();
    const uint32_t n_e = ne;
    for (;;) {
        if (t == 0) rounds++, left = 0;
        for (uint32_t v = t; v < nn; v += kSccSmallThreads)
            if (act[v]) col[v] = v;
        __syncthreads();
        do {  // forward: colour = the largest active id reaching the node
            __syncthreads();
            if (t == 0) changed = 0, sweeps++;
            __syncthreads();
            for (uint32_t i = t; i < n_e; i += kSccSmallThreads) {
                const uint32_t a = E[i] >> 16, b = E[i] & 0xFFFFu;
                if (!act[a] || !act[b]) continue;
                const uint32_t ca = col[a];
                if (ca > col[b] && atomicMax(&col[b], ca) < ca) changed = 1;
            }
            __syncthreads();
        } while (changed);
        for (uint32_t v = t; v < nn; v += kSccSmallThreads)
            if (act[v] && col[v] == v) mk[v] = 1;
        __syncthreads();
        do {  // backward from the roots, inside a colour
            __syncthreads();
            if (t == 0) changed = 0, sweeps++;
            __syncthreads();
            for (uint32_t i = t; i < n_e; i += kSccSmallThreads) {
                const uint32_t a = E[i] >> 16, b = E[i] & 0xFFFFu;
                if (!act[a] || !act[b] || mk[a] || !mk[b] || col[a] != col[b]) continue;
                mk[a] = 1;
                changed = 1;
            }
            __syncthreads();
        } while (changed);
        for (uint32_t v = t; v < nn; v += kSccSmallThreads) {
            if (!act[v]) continue;
            if (mk[v]) {
                scc[v] = col[v];
                act[v] = 0;
                mk[v] = 0;
            } else {
                left = 1;
            }
        }
        __syncthreads();
        if (!left) break;
        __syncthreads();
    }
    if (t == 0) out[0] = rounds, out[1] = sweeps;
}

hipError_t graph_scc_rows(uint32_t nn, const uint8_t *cover, const uint64_t *rows, size_t m,
                          GraphBufs &g, uint32_t *scc_out, uint32_t *n_cut, uint32_t *rounds,
                          uint32_t *iterations, hipStream_t s)
{
    hipError_t e = hipSuccess;
#define CK(x)                                 \
    do {                                      \
        e = (x);                              \
        if (e != hipSuccess) return e;        \
    } while (0)
    *rounds = *iterations = 0;
    *n_cut = 0;
    if (nn == 0) return hipSuccess;
    // cut node ids: the cover's bitmap words and their scan
    const uint32_t nwd = (nn + 63) / 64;
    CK(g.cut_id.ensure(4 * ((size_t)nwd + 64)));
    CK(g.cover_bits.ensure(8 * ((size_t)nwd + 1)));
    CK(g.scratch.ensure(std::max(scan_scratch_bytes((size_t)nwd + 1), (size_t)1024)));
    CK(g.count.ensure(64));
    uint32_t *wc = g.cut_id.as<uint32_t>();
    uint64_t *bits = g.cover_bits.as<uint64_t>();
    k_cover_words<<<blocks(nn), 256, 0, s>>>(nn, cover, bits, wc);
    CK(hipMemsetAsync(wc + nwd, 0, 4, s));
    CK(scan_exclusive_u32(wc, (size_t)nwd + 1, g.scratch.as<uint32_t>(), s));
    uint32_t nc = 0;
    CK(hipMemcpyAsync(&nc, wc + nwd, 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    *n_cut = nc;
    CK(g.txn_of.ensure(4 * ((size_t)nc + 64)));
    uint32_t *txn_of = g.txn_of.as<uint32_t>();
    k_txn_of_w<<<blocks(nwd), 256, 0, s>>>(nwd, bits, wc, txn_of);
    // edge rows over cut ids -> sorted unique CSR / CSC
    const size_t ecap = std::max<size_t>(64, (m + 63) & ~(size_t)63);
    CK(g.ew.ensure(8 * ecap));
    CK(g.et.ensure(8 * ecap));
    CK(g.eg.ensure(4 * ecap));
    CK(g.ew2.ensure(8 * ecap));
    CK(g.et2.ensure(8 * ecap));
    CK(g.eg2.ensure(4 * ecap));
    uint32_t *bad = g.count.as<uint32_t>() + 8;
    CK(hipMemsetAsync(bad, 0, 4, s));
    if (m)
        k_relabel<<<blocks(m), 256, 0, s>>>(m, nn, rows, bits, wc, g.ew.as<uint64_t>(),
                                            g.et.as<uint64_t>(), g.eg.as<uint32_t>(), bad);
    CK(hipGetLastError());
    uint32_t hbad = 0;
    if (nc <= kSccSmallNodes && m <= kSccSmallEdges) {  // the usual small cut: one workgroup
        // (the relabel's check read with the result: one sync; a row outside
        // the cover fails the call, whatever the SCC made of its ~0)
        CK(g.scc.ensure(4 * ((size_t)nc + 1)));
        k_scc_small<<<1, kSccSmallThreads, 0, s>>>(nc, m, g.ew.as<uint64_t>(), g.scc.as<uint32_t>(),
                                                   g.count.as<uint32_t>() + 4);
        CK(hipGetLastError());
        uint32_t ri[3] = {0, 0, 0};
        k_scc_out<<<blocks(nn), 256, 0, s>>>(nn, bits, wc, g.scc.as<uint32_t>(), txn_of, scc_out);
        CK(hipGetLastError());
        CK(hipMemcpyAsync(ri, g.count.as<uint32_t>() + 4, 8, hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(&ri[2], bad, 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (ri[2]) return hipErrorInvalidValue;  // a row outside the cover: not a cut of it
        *rounds = ri[0], *iterations = ri[1];
        return hipSuccess;
    }
    CK(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (hbad) return hipErrorInvalidValue;  // a row outside the cover: not a cut of it
    CK(graph_rows_csr(m, ecap, nc, g, s));
    CK(graph_scc(nc, g, rounds, iterations, s));
    // sub_scc lives in g.scc (nc entries); the caller's scc_out gets all nn
    k_scc_out<<<blocks(nn), 256, 0, s>>>(nn, bits, wc, g.scc.as<uint32_t>(), txn_of, scc_out);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
#undef CK
    return hipSuccess;
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_graph()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_gw_count);
}

}  // namespace hsc
