// hsc_ingest.hip -- packed-key window sort (gfx950).
//
// A window build sorts its rows by (gid, key words), keeps every version in
// key order (rw pairs, the delta fold) and the last version of each key
// (device_build).  The generic path (hsc_kernels.hip radix_sort_rows) moves
// whole rows -- gid, W key words and the LSN, 20+ bytes -- through one LSD
// pass per varying key byte.  When the key bits that vary across the window
// (gid and words together) plus the bits of a row index fit one 64-bit word
// -- config 2's 40-bit keys with 24 index bits, config 5's 33 + 27 -- each row
// travels as a single word instead:
//   pack     key = compress(varying bits, most significant limb first) << I
//            | row index, one pass over the varying limbs only; it also counts
//            digit 0 of its 8192-row block;
//   scatter  one stable LSD pass per varying key byte: the block's keys are
//            ranked per wave with ballots, staged in LDS in sorted order and
//            leave as coalesced runs per digit (k_pk_count counts the next
//            digit of the permuted keys);
//   unpack   every sorted key back to gid / words (expand of the kept bits
//            over row 0's constant bits) with the LSN gathered by row index
//            -- or, when the LSNs' varying bits fit beside the key bits, the
//            LSN itself rides in the low bits instead of the index (packed by
//            k_pk_pack's coalesced read, expanded here: no random gather) --
//            plus the "last version of its key" flag;
// then the usual scan + compaction (dedupe_flagged) gives the distinct rows.
// Per row and pass that is 8 B read + 8 B written instead of a whole row.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

namespace hsc {
namespace {

constexpr int kPkThreads = 512;
constexpr int kPkItems = 16;
constexpr int kPkTile = kPkThreads * kPkItems;  // rows per block (8192)
constexpr int kPkWaves = kPkThreads / 64;

__device__ __forceinline__ uint64_t pk_compress(uint64_t x, uint64_t m, const uint64_t (&mv)[6])
{
    return bits_compress(x, m, mv);
}

// inverse of pk_compress (Hacker's Delight expand: the same moves, reversed)
__device__ __forceinline__ uint64_t pk_expand(uint64_t x, uint64_t m, const uint64_t (&mv)[6])
{
    return bits_expand(x, m, mv);
}

__device__ __forceinline__ uint64_t pk_limb(const PackPlan &P, int l, size_t i, const uint32_t *gid,
                                            const uint64_t *words, size_t stride)
{
    const int id = P.limb[l];
    return id == P.W ? (uint64_t)gid[i] : words[(size_t)id * stride + i];
}

// ghist != null (the one-sweep passes): instead of pass 0's per-block counts,
// the global digit histograms of all np passes (ghist[p * 256 + digit])
constexpr int kOsMaxPasses = 8;
__global__ __launch_bounds__(kPkThreads) void k_pk_pack(PackPlan P, size_t n, const uint32_t *gid,
                                                        const uint64_t *words, size_t stride,
                                                        const uint64_t *lsn, uint64_t *keys, uint32_t *counts,
                                                        uint32_t nblocks, uint32_t *ghist, int np)
{
    __shared__ uint32_t h[256];
    __shared__ uint32_t hh[kOsMaxPasses][256];
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    if (ghist)
        for (int j = threadIdx.x; j < np * 256; j += kPkThreads) hh[j >> 8][j & 255] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kPkTile;
    uint64_t key[kPkItems];
#pragma unroll
    for (int k = 0; k < kPkItems; ++k) {  // every load in flight before the first store
        const size_t i = base + (size_t)k * kPkThreads + threadIdx.x;
        uint64_t kb = 0;
        if (i < n) {
#pragma unroll
            for (int l = 0; l < kPackLimbs; ++l) {
                if (l < P.nl) {
                    uint64_t mv[6];
#pragma unroll
                    for (int q = 0; q < 6; ++q) mv[q] = P.mv[l][q];
                    kb = (kb << P.bits[l]) |
                         pk_compress(pk_limb(P, l, i, gid, words, stride), P.mask[l], mv);
                }
            }
        }
        uint64_t low = (uint64_t)i;
        if (P.lsn_packed) {
            uint64_t lm[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) lm[q] = P.lmv[q];
            low = i < n ? pk_compress(lsn[i], P.lmask, lm) : 0;
        }
        key[k] = P.I ? (kb << P.I) | low : kb;  // (I = 0, no LSN field: the key is the whole row)
    }
#pragma unroll
    for (int k = 0; k < kPkItems; ++k) {
        const size_t i = base + (size_t)k * kPkThreads + threadIdx.x;
        if (i < n) {
            keys[i] = key[k];
            if (ghist) {
                for (int p = 0; p < np; ++p)
                    atomicAdd(&hh[p][(uint32_t)(key[k] >> (P.I + P.skip + 8 * p)) & 0xFFu], 1u);
            } else {
                atomicAdd(&h[(uint32_t)(key[k] >> (P.I + P.skip)) & 0xFFu], 1u);
            }
        }
    }
    __syncthreads();
    if (ghist) {
        for (int j = threadIdx.x; j < np * 256; j += kPkThreads)
            if (hh[j >> 8][j & 255]) atomicAdd(&ghist[j], hh[j >> 8][j & 255]);
    } else if (threadIdx.x < 256) {
        counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
    }
}

// Per-block counts of digit (key >> sh) & 255, digit-major.
__global__ __launch_bounds__(kPkThreads) void k_pk_count(int sh, size_t n, const uint64_t *keys,
                                                         uint32_t *counts, uint32_t nblocks)
{
    __shared__ uint32_t h[256];
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kPkTile;
    uint32_t d[kPkItems];
#pragma unroll
    for (int k = 0; k < kPkItems; ++k) {
        const size_t i = base + (size_t)k * kPkThreads + threadIdx.x;
        d[k] = i < n ? (uint32_t)(__builtin_nontemporal_load(keys + i) >> sh) & 0xFFu : 0x100u;
    }
#pragma unroll
    for (int k = 0; k < kPkItems; ++k)
        if (d[k] < 0x100u) atomicAdd(&h[d[k]], 1u);
    __syncthreads();
    if (threadIdx.x < 256) counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter of one digit.  Phase 1: wave w ranks keys [1024 w, 1024 w +
// 1024) of the block in index order against wave-private digit counters (16
// rounds of 64 lanes, 8 ballots per round), the per-wave counts become
// per-(wave, digit) starts and every key is written to its place of the
// block's sorted order in LDS.  Phase 2 reads LDS in order, so consecutive
// threads store consecutive addresses of each digit's run.
__global__ __launch_bounds__(kPkThreads) void k_pk_scatter(int sh, size_t n, const uint64_t *keys,
                                                           uint64_t *keys_o, const uint32_t *offsets,
                                                           uint32_t nblocks)
{
    constexpr uint32_t kWaveRows = kPkTile / kPkWaves;
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t loff[256];
    __shared__ uint32_t wcnt[kPkWaves][256];
    __shared__ uint64_t stage[kPkTile];
    __shared__ uint32_t lds16[16];
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * kPkTile;
    const uint32_t wbase = wid * kWaveRows;
    uint64_t key[kPkItems];
#pragma unroll
    for (int k = 0; k < kPkItems; ++k) {  // the block's keys first: their loads overlap the offsets'
        const size_t i = base + wbase + k * 64 + lane;
        key[k] = i < n ? __builtin_nontemporal_load(keys + i) : 0;
    }
    uint32_t cnt = 0;
    if (threadIdx.x < 256) {
        const uint32_t dg = threadIdx.x;
        const size_t at = (size_t)dg * nblocks + blockIdx.x;
        const uint32_t mine = offsets[at];
        const uint32_t nxt = at + 1 < (size_t)256 * nblocks ? offsets[at + 1] : (uint32_t)n;
        cnt = nxt - mine;
        gbase[dg] = mine;
    }
    uint32_t tot;
    const uint32_t lo = block_excl_scan<kPkThreads>(cnt, lds16, tot);
    if (threadIdx.x < 256) {
        loff[threadIdx.x] = lo;
#pragma unroll
        for (int w = 0; w < kPkWaves; ++w) wcnt[w][threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t lt_mask = (lane ? (~0ull >> (64 - lane)) : 0ull);
    uint32_t *wc = wcnt[wid];
    uint32_t dig[kPkItems], lp[kPkItems];
#pragma unroll
    for (int k = 0; k < kPkItems; ++k) {
        const size_t i = base + wbase + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t dk = (uint32_t)(key[k] >> sh) & 0xFFu;
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
    if (threadIdx.x < 256) {  // per-(wave, digit) start inside the block's sorted order
        uint32_t acc = loff[threadIdx.x];
#pragma unroll
        for (int w = 0; w < kPkWaves; ++w) {
            const uint32_t t = wcnt[w][threadIdx.x];
            wcnt[w][threadIdx.x] = acc;
            acc += t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPkItems; ++k)
        if (dig[k] != 0xFFFFFFFFu) stage[wc[dig[k]] + lp[k]] = key[k];
    __syncthreads();
    const uint32_t nrows = (uint32_t)min((size_t)kPkTile, n - base);
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < nrows; j += kPkThreads) {
        const uint64_t kj = stage[j];
        const uint32_t dj = (uint32_t)(kj >> sh) & 0xFFu;
        __builtin_nontemporal_store(kj, keys_o + gbase[dj] + (j - loff[dj]));
    }
}

// One pass of the one-sweep sort (no count pass, no scan): tiles are taken in
// ticket order; each ranks its keys as k_pk_scatter does, publishes its digit
// counts (flag 1 = this tile's count, 2 = the inclusive prefix through it) and
// looks back over the tiles before it -- one thread per digit, summing counts
// until a prefix -- for its runs' global starts (the digit's base from the
// pass's histogram, which k_pk_pack counted, + the prefix).  Earlier tickets
// are resident or done, so the look-back always ends; a look-back that spins
// past kOsSpin reads sets *err (the build fails loudly) and goes on.
constexpr uint32_t kOsAgg = 1u << 30, kOsInc = 2u << 30, kOsVal = (1u << 30) - 1;
constexpr uint32_t kOsSpin = 1u << 24;
constexpr size_t kOsMinRows = (size_t)1 << 21;
constexpr size_t kOsMinTile = (size_t)kPkThreads * 8;  // rows per one-sweep tile, at least
// LA: the look-back reads LA tiles' statuses per step, all loads in flight
// together (the status words are agent-scope: a read that misses the XCD's L2
// costs a trip to memory, so a serial walk pays one per tile)
template <int LA, int IT, int TH>
__global__ __launch_bounds__(TH) void k_pk_onesweep(int sh, size_t n, const uint64_t *keys,
                                                            uint64_t *keys_o, const uint32_t *hist,
                                                            uint32_t *status, uint32_t *ticket, uint32_t *err)
{
    constexpr int kOsTile = TH * IT;
    constexpr uint32_t kWaveRows = kOsTile / (TH / 64);
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t loff[256];
    __shared__ uint32_t wcnt[(TH / 64)][256];
    __shared__ uint64_t stage[kOsTile];
    __shared__ uint32_t lds16[16];
    __shared__ uint32_t tile_id;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) tile_id = atomicAdd(ticket, 1u);
    if (threadIdx.x < 256) {
#pragma unroll
        for (int w = 0; w < (TH / 64); ++w) wcnt[w][threadIdx.x] = 0;
    }
    __syncthreads();
    const uint32_t b = tile_id;
    const size_t base = (size_t)b * kOsTile;
    const uint32_t wbase = wid * kWaveRows;
    uint64_t key[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const size_t i = base + wbase + k * 64 + lane;
        key[k] = i < n ? __builtin_nontemporal_load(keys + i) : 0;
    }
    // the digits' global bases: the exclusive scan of the pass's histogram
    uint32_t dtot;
    const uint32_t dbase = block_excl_scan<TH>(threadIdx.x < 256 ? hist[threadIdx.x] : 0u, lds16, dtot);
    const uint64_t lt_mask = (lane ? (~0ull >> (64 - lane)) : 0ull);
    uint32_t *wc = wcnt[wid];
    uint32_t dig[IT], lp[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const size_t i = base + wbase + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t dk = (uint32_t)(key[k] >> sh) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t m = __ballot((dk >> q) & 1u);
            peers &= ((dk >> q) & 1u) ? m : ~m;
        }
        const uint32_t before = wc[dk];
        lp[k] = before + __popcll(peers & lt_mask);
        dig[k] = valid ? dk : 0xFFFFFFFFu;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && (peers & lt_mask) == 0) wc[dk] = before + __popcll(peers);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    uint32_t cnt = 0;
    if (threadIdx.x < 256) {
        const uint32_t d = threadIdx.x;
#pragma unroll
        for (int w = 0; w < (TH / 64); ++w) cnt += wcnt[w][d];
        // publish, look back, publish the prefix
        uint32_t *my = status + (size_t)b * 256 + d;
        uint32_t excl = 0;
        if (b > 0) {
            __hip_atomic_store(my, kOsAgg | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)b - 1;
            uint32_t spins = 0;
            while (j >= 0) {
                uint32_t v[LA];
#pragma unroll
                for (int q = 0; q < LA; ++q)  // (before tile 0: an inclusive 0)
                    v[q] = j - q >= 0 ? __hip_atomic_load(status + (size_t)(j - q) * 256 + d, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : kOsInc;
                int q = 0;
                bool done = false;
#pragma unroll
                for (int r = 0; r < LA; ++r) {
                    if (q != r || done) continue;
                    const uint32_t f = v[r] & ~kOsVal;
                    if (f == 0) continue;  // not published yet: the next step starts at tile j - r
                    excl += v[r] & kOsVal;
                    done = f == kOsInc;
                    ++q;
                }
                if (done) break;
                if (q < LA) {
                    j -= q;
                    if (++spins > kOsSpin) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                j -= LA;
            }
        }
        __hip_atomic_store(my, kOsInc | (excl + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gbase[d] = dbase + excl;
    }
    uint32_t tot;
    const uint32_t lo = block_excl_scan<TH>(cnt, lds16, tot);
    if (threadIdx.x < 256) {
        loff[threadIdx.x] = lo;
        uint32_t acc = lo;  // per-(wave, digit) start inside the tile's sorted order
#pragma unroll
        for (int w = 0; w < (TH / 64); ++w) {
            const uint32_t t = wcnt[w][threadIdx.x];
            wcnt[w][threadIdx.x] = acc;
            acc += t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k)
        if (dig[k] != 0xFFFFFFFFu) stage[wc[dig[k]] + lp[k]] = key[k];
    __syncthreads();
    const uint32_t nrows = base < n ? (uint32_t)min((size_t)kOsTile, n - base) : 0u;
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < nrows; j += TH) {
        const uint64_t kj = stage[j];
        const uint32_t dj = (uint32_t)(kj >> sh) & 0xFFu;
        __builtin_nontemporal_store(kj, keys_o + gbase[dj] + (j - loff[dj]));
    }
}

// ---- unpack fused with the dedupe ----
// Every version goes to (gid_o, words_o, lsn_o) in key order, and the
// last version of each key straight to its place among the distinct rows
// (gid_d, words_d, lsn_d): a block's place is the exclusive scan of the
// blocks' distinct counts (k_pk_bcount), a row's inside the block a scan in
// LDS -- no flag array, no 10M-entry scan, no compaction pass re-reading every
// version.  The distinct outputs may overwrite the input gid / words (only row
// 0's limbs are read, from r0), not the input LSNs (gathered by row index).
constexpr int kUdThreads = 256;
constexpr int kUdRows = 8;                            // rows per thread
constexpr int kUdTile = kUdThreads * kUdRows;         // rows per block

__device__ __forceinline__ bool pk_last(const uint64_t *keys, size_t n, size_t i, int I)
{
    return i + 1 >= n || (keys[i + 1] >> I) != (keys[i] >> I);
}

__global__ __launch_bounds__(kUdThreads) void k_pk_bcount(size_t n, const uint64_t *keys, int I,
                                                          uint32_t *bc)
{
    __shared__ uint32_t wsum[kUdThreads / 64];
    const size_t base = (size_t)blockIdx.x * kUdTile;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kUdRows; ++r) {
        const size_t i = base + (size_t)r * kUdThreads + threadIdx.x;
        if (i < n) c += pk_last(keys, n, i, I);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kUdThreads / 64; ++w) t += wsum[w];
        bc[blockIdx.x] = t;
    }
}

__global__ void k_pk_row0(int W, const uint32_t *gid_in, const uint64_t *words_in, size_t stride_in,
                          uint64_t *r0)
{
    const int j = threadIdx.x;
    if (j < W) r0[j] = words_in[(size_t)j * stride_in];
    if (j == W) r0[W] = gid_in[0];
}

// KO: the distinct packed keys only (no rows, no LSNs: the graph's writers)
template <int WT, bool KO>  // key words 1..3, 0 = any (<= kPackMaxWords)
__global__ __launch_bounds__(kUdThreads) void k_pk_unpack_dd(
    PackPlan P, size_t n, const uint64_t *keys, const uint64_t *r0, const uint64_t *lsn_in,
    uint32_t *gid_o, uint64_t *words_o, uint64_t *lsn_o, size_t stride_o, const uint32_t *boff,
    uint32_t *gid_d, uint64_t *words_d, uint64_t *lsn_d, size_t stride_d, uint32_t *d_count,
    uint64_t *ww, PairPack wp)
{
    __shared__ uint64_t K[kUdTile + 1];
    __shared__ uint32_t pos[kUdTile];
    __shared__ uint32_t wsum[kUdThreads / 64];
    const int W = WT ? WT : P.W;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * kUdTile;
    const uint32_t nrows = (uint32_t)min((size_t)kUdTile, n - base);
#pragma unroll
    for (int r = 0; r < kUdRows; ++r) {
        const uint32_t j = r * kUdThreads + threadIdx.x;
        if (j < nrows) K[j] = keys[base + j];
    }
    if (threadIdx.x == 0 && base + nrows < n) K[nrows] = keys[base + nrows];
    __syncthreads();
    // thread t ranks rows 8t .. 8t + 7 of the block (contiguous): last-of-key
    // flags, their count, a wave scan and a block scan
    const uint64_t lim = P.I >= 64 ? 0 : ~0ull << P.I;  // the key bits
    uint32_t fl = 0, cnt = 0;
#pragma unroll
    for (int r = 0; r < kUdRows; ++r) {
        const uint32_t j = threadIdx.x * kUdRows + r;
        const bool last = j < nrows && (base + j + 1 >= n || ((K[j] ^ K[j + 1]) & lim) != 0);
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
    for (int w = 0; w < kUdThreads / 64; ++w) {
        run += w < wv ? wsum[w] : 0;
        total += wsum[w];
    }
#pragma unroll
    for (int r = 0; r < kUdRows; ++r) {
        const uint32_t j = threadIdx.x * kUdRows + r;
        if (j < nrows) pos[j] = (fl >> r & 1u) ? run : 0xFFFFFFFFu;
        run += fl >> r & 1u;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *d_count = boff[blockIdx.x] + total;
    __syncthreads();
    const uint32_t b0 = boff[blockIdx.x];
    if (KO) {
        // ww != null: also the writers' ww rows (writer d -> d + 1 of the same
        // key, ~0 else) -- with no index bits a run is one repeated word, so
        // the next distinct writer is simply the next row (K[nrows]: the next
        // tile's first)
        uint64_t tm[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) tm[q] = wp.tmv[q];
        const uint64_t tmask = wp.tb >= 64 ? ~0ull : (1ull << wp.tb) - 1;
#pragma unroll
        for (int r = 0; r < kUdRows; ++r) {
            const uint32_t j = r * kUdThreads + threadIdx.x;
            if (j >= nrows || pos[j] == 0xFFFFFFFFu) continue;
            const uint64_t kj = K[j];
            const size_t d = (size_t)b0 + pos[j];
            lsn_d[d] = kj;
            if (ww) {
                uint64_t e = ~0ull;
                if (base + j + 1 < n) {
                    const uint64_t nx = K[j + 1];
                    if (wp.tb >= 64 || (kj >> wp.tb) == (nx >> wp.tb))
                        e = ((bits_expand(kj & tmask, wp.tm, tm) | wp.tc) << 32) |
                            (bits_expand(nx & tmask, wp.tm, tm) | wp.tc);
                }
                ww[d] = e;
            }
        }
        return;
    }
    const uint64_t imask = P.I >= 64 ? ~0ull : (1ull << P.I) - 1;
    // every row's LSN gather issued before the first store (10M random 8-byte
    // reads for config 2: two in flight per thread left the unpack
    // latency-bound)
    uint64_t lvs[kUdRows];
#pragma unroll
    for (int r = 0; r < kUdRows; ++r) {
        const uint32_t j = r * kUdThreads + threadIdx.x;
        // (no LSNs and no index bits -- the packed key is the whole row: the
        // distinct rows' "LSN" slot gets the packed key itself, which the
        // dependency graph takes as its packed writer array)
        if (P.lsn_packed) {  // the LSN rode in the key's low bits
            uint64_t lm[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) lm[q] = P.lmv[q];
            lvs[r] = j >= nrows ? 0 : pk_expand(K[j] & imask, P.lmask, lm) | P.lconst;
        } else {
            lvs[r] = j >= nrows ? 0 : lsn_in ? lsn_in[K[j] & imask] : P.I == 0 ? K[j] : 0;
        }
    }
#pragma unroll  // (whole: lvs stays in registers)
    for (int r = 0; r < kUdRows; ++r) {
        const uint32_t j = r * kUdThreads + threadIdx.x;
        if (j >= nrows) break;
        const size_t i = base + j;
        const uint64_t key = K[j];
        uint64_t kb = key >> P.I;
        const uint64_t lv = lvs[r];
        uint64_t limb[kPackMaxWords + 1];
#pragma unroll
        for (int q = 0; q <= kPackMaxWords; ++q) {
            if (q > W) break;
            limb[q] = r0[q];
        }
#pragma unroll
        for (int l = kPackLimbs - 1; l >= 0; --l) {  // least significant varying limb first
            if (l >= P.nl) continue;
            const int b = P.bits[l];
            const uint64_t part = b >= 64 ? kb : kb & ((1ull << b) - 1);
            kb = b >= 64 ? 0 : kb >> b;
            uint64_t mv[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) mv[q] = P.mv[l][q];
            const int id = P.limb[l];
            const uint64_t v = pk_expand(part, P.mask[l], mv);
#pragma unroll
            for (int q = 0; q <= kPackMaxWords; ++q)
                if (q == id) limb[q] = (limb[q] & ~P.mask[l]) | v;
        }
        if (gid_o) {  // (null: the distinct rows only)
            gid_o[i] = (uint32_t)limb[W];
#pragma unroll
            for (int q = 0; q < kPackMaxWords; ++q) {
                if (q >= W) break;
                words_o[(size_t)q * stride_o + i] = limb[q];
            }
            lsn_o[i] = lv;
        }
        const uint32_t p = pos[j];
        if (p != 0xFFFFFFFFu) {
            const size_t d = (size_t)b0 + p;
            if (gid_d) {  // (null: the distinct packed keys only)
                gid_d[d] = (uint32_t)limb[W];
#pragma unroll
                for (int q = 0; q < kPackMaxWords; ++q) {
                    if (q >= W) break;
                    words_d[(size_t)q * stride_d + d] = limb[q];
                }
            }
            lsn_d[d] = lv;
        }
    }
}

}  // namespace

// scratch: pass 0's per-block counts + their scan, the unpack's block counts
// + scan + row 0, then (16-byte aligned) the one-sweep region: the passes'
// histograms, their tickets, and kOsMaxPasses x tiles x 256 status words
static size_t packed_base_bytes(size_t n)
{
    const size_t nblocks = (n + kPkTile - 1) / kPkTile;
    const size_t ud = (n + kUdTile - 1) / kUdTile;
    return 256 * nblocks * sizeof(uint32_t) + scan_scratch_bytes(256 * nblocks) + 1024 +
           (ud + 16) * sizeof(uint32_t) + scan_scratch_bytes(ud) + 8 * (kPackMaxWords + 1) + 64;
}

static size_t os_offset(size_t n) { return (packed_base_bytes(n) + 255) & ~(size_t)255; }

size_t packed_scratch_bytes(size_t n)
{
    const size_t nblocks = (n + kOsMinTile - 1) / kOsMinTile;  // (status words for the smallest tiles)
    return os_offset(n) + 4 * ((size_t)kOsMaxPasses * 256 + 64 + (size_t)kOsMaxPasses * 256 * nblocks);
}

bool packed_plan(int W, size_t n, const uint64_t *vary, PackPlan *P, bool index, const uint64_t *lsn_bits)
{
    if (W > kPackMaxWords || n >= 0xFFFFFFFFull) return false;
    *P = PackPlan{};
    P->W = W;
    int I = 1;
    while (I < 32 && ((size_t)1 << I) < n) ++I;
    if (!index) I = 0;
    P->I = I;
    int B = 0, nl = 0;
    // limb order, most significant first: gid, then word 0 .. W - 1
    for (int k = 0; k <= W; ++k) {
        const int id = k == 0 ? W : k - 1;
        const uint64_t m = vary[id];
        if (!m) continue;
        P->limb[nl] = id;
        P->mask[nl] = m;
        P->bits[nl] = __builtin_popcountll(m);
        compress_moves(m, P->mv[nl]);
        B += P->bits[nl];
        ++nl;
    }
    P->nl = nl;
    P->B = B;
    static const bool no_lsn_pack = getenv("HSC_NO_LSN_PACK") != nullptr;  // (A/B)
    if (index && lsn_bits && !no_lsn_pack) {
        const int L = __builtin_popcountll(lsn_bits[0]);
        if (B + L <= 64) {  // the LSN itself in the low bits: no gather in the unpack
            P->I = L;
            P->lsn_packed = true;
            P->lmask = lsn_bits[0];
            P->lconst = lsn_bits[1] & ~lsn_bits[0];
            compress_moves(P->lmask, P->lmv);
            return true;
        }
    }
    return B + I <= 64;
}

// The LSD passes of the packed keys; the sorted keys end in *kf, the other
// key buffer is *kfree.
// (err != null: the one-sweep passes, their stall flag -- cleared here)
static hipError_t packed_passes(const PackPlan &P, size_t n, const uint32_t *gid,
                                const uint64_t *words, size_t stride, const uint64_t *lsn, uint64_t *k0,
                                uint64_t *k1, void *scratch, hipStream_t s, uint64_t **kf, uint64_t **kfree,
                                uint32_t *err)
{
    const uint32_t nblocks = (uint32_t)((n + kPkTile - 1) / kPkTile);
    uint32_t *counts = (uint32_t *)scratch;
    uint32_t *scan_tmp = counts + (size_t)256 * nblocks;
    if (P.lsn_packed && !lsn) return hipErrorInvalidValue;
    // (P.skip: the low bits the input is already ordered by need no pass --
    // the passes are stable)
    const int passes = (P.B - P.skip + 7) / 8;
    // one-sweep passes (HSC_NO_ONESWEEP: the count + scan + scatter passes, an A/B)
    static const bool no_os = getenv("HSC_NO_ONESWEEP") != nullptr;
    // look-back width (HSC_OS_LOOK=1: one tile per step, an A/B)
    static const int os_look = getenv("HSC_OS_LOOK") ? atoi(getenv("HSC_OS_LOOK")) : 4;
    // rows per one-sweep tile (HSC_OS_TILE = 4096 / 8192 / 16384, an A/B)
    static const size_t os_tile = [] {
        const size_t t = getenv("HSC_OS_TILE") ? (size_t)atoi(getenv("HSC_OS_TILE")) : 8192;
        return t == 4096 || t == 16384 ? t : (size_t)8192;
    }();
    if (err) {
        const hipError_t e = hipMemsetAsync(err, 0, 4, s);
        if (e != hipSuccess) return e;
    }
    // (small sorts -- a commit stream's windows and folds, < 2M rows -- keep
    // the count + scan passes: a few tiles gain nothing from the look-back)
    if (err && !no_os && passes > 0 && passes <= kOsMaxPasses && n >= kOsMinRows && n < (size_t)kOsVal) {
        uint32_t *ghist = (uint32_t *)((uint8_t *)scratch + os_offset(n));
        uint32_t *tickets = ghist + kOsMaxPasses * 256;
        uint32_t *status = tickets + 64;
        const uint32_t nbos = (uint32_t)((n + os_tile - 1) / os_tile);
        hipError_t e =
            hipMemsetAsync(ghist, 0, 4 * ((size_t)kOsMaxPasses * 256 + 64 + (size_t)passes * 256 * nbos), s);
        if (e != hipSuccess) return e;
        k_pk_pack<<<nblocks, kPkThreads, 0, s>>>(P, n, gid, words, stride, lsn, k0, counts, nblocks, ghist,
                                                 passes);
        e = hipGetLastError();
        for (int p = 0; p < passes && e == hipSuccess; ++p) {
            const int sh = P.I + P.skip + 8 * p;
            uint32_t *st = status + (size_t)p * 256 * nbos;
            if (os_tile == 4096)
                k_pk_onesweep<4, 8, 512><<<nbos, 512, 0, s>>>(sh, n, k0, k1, ghist + 256 * p, st, tickets + p, err);
            else if (os_tile == 16384)
                k_pk_onesweep<4, 16, 1024><<<nbos, 1024, 0, s>>>(sh, n, k0, k1, ghist + 256 * p, st, tickets + p, err);
            else if (os_look == 1)
                k_pk_onesweep<1, 16, 512><<<nbos, 512, 0, s>>>(sh, n, k0, k1, ghist + 256 * p, st, tickets + p, err);
            else
                k_pk_onesweep<4, 16, 512><<<nbos, 512, 0, s>>>(sh, n, k0, k1, ghist + 256 * p, st, tickets + p, err);
            e = hipGetLastError();
            std::swap(k0, k1);
        }
        *kf = k0;
        *kfree = k1;
        return e;
    }
    k_pk_pack<<<nblocks, kPkThreads, 0, s>>>(P, n, gid, words, stride, lsn, k0, counts, nblocks, nullptr, 0);
    hipError_t e = hipGetLastError();
    for (int p = 0; p < passes && e == hipSuccess; ++p) {
        const int sh = P.I + P.skip + 8 * p;
        if (p > 0) k_pk_count<<<nblocks, kPkThreads, 0, s>>>(sh, n, k0, counts, nblocks);
        e = scan_exclusive_u32(counts, (size_t)256 * nblocks, scan_tmp, s);
        if (e != hipSuccess) break;
        k_pk_scatter<<<nblocks, kPkThreads, 0, s>>>(sh, n, k0, k1, counts, nblocks);
        e = hipGetLastError();
        std::swap(k0, k1);
    }
    *kf = k0;
    *kfree = k1;
    return e;
}

hipError_t packed_sort_dedupe(const PackPlan &P, size_t n, const uint32_t *gid, const uint64_t *words,
                              const uint64_t *lsn, size_t stride, uint64_t *k0, uint64_t *k1,
                              uint32_t *gid_o, uint64_t *words_o, uint64_t *lsn_o, size_t stride_o,
                              uint32_t *gid_d, uint64_t *words_d, size_t stride_d,
                              uint64_t **lsn_d, uint32_t *d_count, void *scratch,
                              size_t scratch_bytes, hipStream_t s, uint32_t *err, uint64_t *ww_rows,
                              const PairPack *ww_pp)
{
    *lsn_d = nullptr;
    if (n == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
    if (scratch_bytes < packed_scratch_bytes(n)) return hipErrorInvalidValue;
    uint64_t *kf, *kfree;
    hipError_t e = packed_passes(P, n, gid, words, stride, lsn, k0, k1, scratch, s, &kf, &kfree, err);
    if (e != hipSuccess) return e;
    // scratch after the passes' counters: block counts, their scan, row 0
    const uint32_t nblocks = (uint32_t)((n + kPkTile - 1) / kPkTile);
    uint8_t *sp = (uint8_t *)scratch + 256 * (size_t)nblocks * sizeof(uint32_t) +
                  scan_scratch_bytes(256 * (size_t)nblocks) + 1024;
    const uint32_t ud = (uint32_t)((n + kUdTile - 1) / kUdTile);
    uint32_t *bc = (uint32_t *)sp;
    uint32_t *btmp = bc + ud + 16;
    uint64_t *r0 = (uint64_t *)(((uintptr_t)((uint8_t *)btmp + scan_scratch_bytes(ud)) + 15) & ~(uintptr_t)15);
    k_pk_row0<<<1, 64, 0, s>>>(P.W, gid, words, stride, r0);
    k_pk_bcount<<<ud, kUdThreads, 0, s>>>(n, kf, P.I, bc);
    e = hipGetLastError();
    if (e == hipSuccess) e = scan_exclusive_u32(bc, ud, btmp, s);
    if (e != hipSuccess) return e;
    const PairPack wp = ww_pp ? *ww_pp : PairPack{};
#define HSC_UNPACK_DD(WT_)                                                                          \
    k_pk_unpack_dd<WT_, false><<<ud, kUdThreads, 0, s>>>(P, n, kf, r0, lsn, gid_o, words_o, lsn_o,     \
                                                   stride_o, bc, gid_d, words_d, kfree, stride_d,  \
                                                   d_count, nullptr, wp)
    // (the distinct packed keys only -- no rows, no LSNs: a copy of the
    // last-of-key words, no expand; with ww_rows their ww rows too)
    const bool ko = !gid_o && !gid_d && !lsn && P.I == 0 && !P.lsn_packed;
    if (ww_rows && !(ko && ww_pp)) return hipErrorInvalidValue;
    if (ko)
        k_pk_unpack_dd<0, true><<<ud, kUdThreads, 0, s>>>(P, n, kf, r0, lsn, gid_o, words_o, lsn_o, stride_o, bc,
                                                          gid_d, words_d, kfree, stride_d, d_count, ww_rows, wp);
    else if (P.W == 1)
        HSC_UNPACK_DD(1);
    else if (P.W == 2)
        HSC_UNPACK_DD(2);
    else if (P.W == 3)
        HSC_UNPACK_DD(3);
    else
        HSC_UNPACK_DD(0);
#undef HSC_UNPACK_DD
    *lsn_d = kfree;
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_ingest()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_pk_count);
}

}  // namespace hsc
