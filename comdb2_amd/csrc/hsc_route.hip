// hsc_route.hip -- probe routing between the members of a multi-GPU context
// (hsc_multi.cpp).
//
// The window is cut into `world` contiguous pieces of the composite key space
// (gid, key words): member d holds the rows whose key K has
// sp[d-1] <= K < sp[d] (the S = world - 1 splitters, ascending).  A range
// probe [g || lo, g || hi] can only conflict with rows of the members whose
// piece it overlaps, i.e. d in [owner(g || lo), owner(g || hi)] with
// owner(K) = #splitters <= K, and a member holding none of its keys cannot
// report a conflict -- so routing is exact, and the verdict of a read set is
// the OR of its members' verdicts.
//
// Every member routes the probes it holds (its share of the batch, in any
// order) in two passes over the probe columns:
//   k_route_count    per 1024-probe chunk, probes per destination (one
//                    wave-aggregated LDS add per destination present in a
//                    wave) -> hist[chunk][d] and the member's totals[d]
//   k_route_scatter  per chunk, its base in every destination claimed with one
//                    global atomic per (chunk, destination) on the target's
//                    cursor, then every probe copied to its destinations'
//                    columns (the wave's lanes of one destination take
//                    consecutive rows); the read-set number is rebased to the
//                    batch-wide numbering; table-lock probes go to member 0.
// The targets are either the destinations' own probe columns (members in one
// process write each other's memory: the copy IS the exchange) or this
// member's send blocks (one block per destination, sent by RCCL), which the
// receiver turns into probe columns with k_route_unpack.
// Bytes per routed probe: read 2 x (4 + 16 W) (count, scatter) + 8 + 4,
// write 16 W + 16 per destination.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <algorithm>

namespace hsc {

constexpr int kRouteChunk = 1024;  // ~1000 workgroups per million probes
constexpr int kRouteThreads = 256;

// Composite compare of (g, x words at x[j * xs]) against splitter k (LDS:
// sg[k], sw[j * S + k]): < 0, 0, > 0.
__device__ __forceinline__ int route_cmp(uint32_t g, const uint64_t *x, size_t xs, int W,
                                         const uint32_t *sg, const uint64_t *sw, int S, int k)
{
    if (g != sg[k]) return g < sg[k] ? -1 : 1;
    for (int j = 0; j < W; ++j) {
        const uint64_t a = x[(size_t)j * xs], b = sw[(size_t)j * S + k];
        if (a != b) return a < b ? -1 : 1;
    }
    return 0;
}

// owner(K) = #splitters <= K (splitters ascending: binary search)
__device__ __forceinline__ int route_owner(uint32_t g, const uint64_t *x, size_t xs, int W,
                                           const uint32_t *sg, const uint64_t *sw, int S)
{
    int lo = 0, hi = S;  // answer in [lo, hi]
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (route_cmp(g, x, xs, W, sg, sw, S, mid) >= 0)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// The splitters into LDS: sg[S], sw[W * S] (u64 first for alignment).
__device__ __forceinline__ void route_stage(const RouteSplit &sp, uint64_t *lds_w, uint32_t *lds_g)
{
    const int S = sp.S, nw = sp.W * S;
    for (int i = threadIdx.x; i < nw; i += blockDim.x) lds_w[i] = sp.w[i];
    for (int i = threadIdx.x; i < S; i += blockDim.x) lds_g[i] = sp.gid[i];
    __syncthreads();
}

__global__ __launch_bounds__(kRouteThreads) void k_route_count(ProbeView p, RouteSplit sp, int N,
                                                              uint32_t *hist)
{
    extern __shared__ uint64_t lds_w[];
    __shared__ uint32_t cnt[kMultiMax];
    uint32_t *lds_g = (uint32_t *)(lds_w + (size_t)sp.W * sp.S);
    if (threadIdx.x < kMultiMax) cnt[threadIdx.x] = 0;
    route_stage(sp, lds_w, lds_g);
    const uint32_t c0 = blockIdx.x * (uint32_t)kRouteChunk;
    const uint32_t c1 = min(p.n, c0 + (uint32_t)kRouteChunk);
    const int lane = lane_id();
    for (uint32_t base = c0; base < c1; base += kRouteThreads) {
        const uint32_t i = base + threadIdx.x;
        int ra = N, rb = -1;  // no destination (past the chunk)
        if (i < c1) {
            const uint32_t g = p.gid[i];
            ra = route_owner(g, p.lo + i, p.n, sp.W, lds_g, lds_w, sp.S);
            rb = route_owner(g, p.hi + i, p.n, sp.W, lds_g, lds_w, sp.S);
        }
        // wave-aggregated: one LDS add per destination the wave reaches
        int dmin = ra, dmax = rb;
        for (int o = 32; o > 0; o >>= 1) {
            dmin = min(dmin, __shfl_xor(dmin, o, 64));
            dmax = max(dmax, __shfl_xor(dmax, o, 64));
        }
        for (int d = dmin; d <= dmax; ++d) {
            const uint64_t m = __ballot(ra <= d && d <= rb);
            if (lane == 0 && m) atomicAdd(&cnt[d], (uint32_t)__popcll(m));
        }
    }
    __syncthreads();
    if (threadIdx.x < N) hist[(size_t)blockIdx.x * N + threadIdx.x] = cnt[threadIdx.x];
}

// ---- keys of at most 4 words: a chunk's probes in registers ----
// Each thread loads its kRouteP probes of the chunk first (read-once inputs:
// non-temporal), then routes them against the splitters in LDS with the key
// words compared in registers (the generic kernels above re-read them from
// memory at every splitter compare and keep one probe in flight per thread).
constexpr int kRouteP = kRouteChunk / kRouteThreads;

template <int W>
__device__ __forceinline__ int route_owner_r(uint32_t g, const uint64_t (&x)[W], const uint32_t *sg,
                                             const uint64_t *sw, int S)
{
    int lo = 0, hi = S;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int c = g == sg[mid] ? 0 : (g < sg[mid] ? -1 : 1);
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const uint64_t b = sw[(size_t)j * S + mid];
            if (c == 0 && x[j] != b) c = x[j] < b ? -1 : 1;
        }
        if (c >= 0)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

template <int W>
__global__ __launch_bounds__(kRouteThreads) void k_route_count_r(ProbeView p, RouteSplit sp, int N,
                                                                uint32_t *hist)
{
    extern __shared__ uint64_t lds_w[];
    __shared__ uint32_t cnt[kMultiMax];
    uint32_t *lds_g = (uint32_t *)(lds_w + (size_t)W * sp.S);
    const uint32_t c0 = blockIdx.x * (uint32_t)kRouteChunk;
    const uint32_t c1 = min(p.n, c0 + (uint32_t)kRouteChunk);
    if (sp.S == 0) {  // one piece: every probe goes to member 0
        if (threadIdx.x < N) hist[(size_t)blockIdx.x * N + threadIdx.x] = threadIdx.x == 0 ? c1 - min(c0, c1) : 0;
        return;
    }
    uint64_t lo[kRouteP][W], hi[kRouteP][W];
    uint32_t gg[kRouteP];
#pragma unroll
    for (int k = 0; k < kRouteP; ++k) {
        const uint32_t i = c0 + (uint32_t)k * kRouteThreads + threadIdx.x;
        const uint32_t q = i < c1 ? i : 0;
        const bool v = p.n != 0;
        gg[k] = v ? __builtin_nontemporal_load(p.gid + q) : 0;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            lo[k][j] = v ? __builtin_nontemporal_load(p.lo + (size_t)j * p.n + q) : 0;
            hi[k][j] = v ? __builtin_nontemporal_load(p.hi + (size_t)j * p.n + q) : 0;
        }
    }
    if (threadIdx.x < kMultiMax) cnt[threadIdx.x] = 0;
    route_stage(sp, lds_w, lds_g);
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < kRouteP; ++k) {
        const uint32_t i = c0 + (uint32_t)k * kRouteThreads + threadIdx.x;
        int ra = N, rb = -1;
        if (i < c1) {
            ra = route_owner_r<W>(gg[k], lo[k], lds_g, lds_w, sp.S);
            rb = route_owner_r<W>(gg[k], hi[k], lds_g, lds_w, sp.S);
        }
        int dmin = ra, dmax = rb;
        for (int o = 32; o > 0; o >>= 1) {
            dmin = min(dmin, __shfl_xor(dmin, o, 64));
            dmax = max(dmax, __shfl_xor(dmax, o, 64));
        }
        for (int d = dmin; d <= dmax; ++d) {
            const uint64_t m = __ballot(ra <= d && d <= rb);
            if (lane == 0 && m) atomicAdd(&cnt[d], (uint32_t)__popcll(m));
        }
    }
    __syncthreads();
    if (threadIdx.x < N) hist[(size_t)blockIdx.x * N + threadIdx.x] = cnt[threadIdx.x];
}

template <int W>
__global__ __launch_bounds__(kRouteThreads) void k_route_scatter_r(ProbeView p, RouteSplit sp,
                                                                  RouteArgs a, const uint32_t *hist,
                                                                  uint32_t *cursor)
{
    extern __shared__ uint64_t lds_w[];
    __shared__ uint32_t cur[kMultiMax];
    uint32_t *lds_g = (uint32_t *)(lds_w + (size_t)W * sp.S);
    const int N = a.N;
    const uint32_t c0 = blockIdx.x * (uint32_t)kRouteChunk;
    const uint32_t c1 = min(p.n, c0 + (uint32_t)kRouteChunk);
    uint64_t lo[kRouteP][W], hi[kRouteP][W], sn[kRouteP];
    uint32_t gg[kRouteP], tx[kRouteP];
#pragma unroll
    for (int k = 0; k < kRouteP; ++k) {
        const uint32_t i = c0 + (uint32_t)k * kRouteThreads + threadIdx.x;
        const uint32_t q = i < c1 ? i : 0;
        const bool v = p.n != 0;
        gg[k] = v ? __builtin_nontemporal_load(p.gid + q) : 0;
        tx[k] = v ? __builtin_nontemporal_load(p.txn + q) : 0;
        sn[k] = v ? __builtin_nontemporal_load(p.snap + q) : 0;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            lo[k][j] = v ? __builtin_nontemporal_load(p.lo + (size_t)j * p.n + q) : 0;
            hi[k][j] = v ? __builtin_nontemporal_load(p.hi + (size_t)j * p.n + q) : 0;
        }
    }
    if (threadIdx.x < N) {
        const uint32_t v = hist[(size_t)blockIdx.x * N + threadIdx.x];
        cur[threadIdx.x] = v ? a.base[threadIdx.x] + atomicAdd(&cursor[threadIdx.x], v) : 0;
    }
    route_stage(sp, lds_w, lds_g);
    const int lane = lane_id();
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll
    for (int k = 0; k < kRouteP; ++k) {
        const uint32_t i = c0 + (uint32_t)k * kRouteThreads + threadIdx.x;
        int ra = N, rb = -1;
        if (i < c1) {
            if (sp.S == 0) {
                ra = rb = 0;
            } else {
                ra = route_owner_r<W>(gg[k], lo[k], lds_g, lds_w, sp.S);
                rb = route_owner_r<W>(gg[k], hi[k], lds_g, lds_w, sp.S);
            }
        }
        int dmin = ra, dmax = rb;
        for (int o = 32; o > 0; o >>= 1) {
            dmin = min(dmin, __shfl_xor(dmin, o, 64));
            dmax = max(dmax, __shfl_xor(dmax, o, 64));
        }
        for (int d = dmin; d <= dmax; ++d) {
            const bool mine = ra <= d && d <= rb;
            const uint64_t m = __ballot(mine);
            if (!m) continue;
            const int first = __ffsll((unsigned long long)m) - 1;
            uint32_t b0 = 0;
            if (lane == first) b0 = atomicAdd(&cur[d], (uint32_t)__popcll(m));
            b0 = __shfl(b0, first, 64);
            if (mine) {
                const RouteTarget &t = a.t[d];
                const size_t r = (size_t)b0 + __popcll(m & below);
#pragma unroll
                for (int j = 0; j < W; ++j) {
                    t.lo[(size_t)j * t.stride + r] = lo[k][j];
                    t.hi[(size_t)j * t.stride + r] = hi[k][j];
                }
                t.gid[r] = gg[k];
                t.snap[r] = sn[k];
                t.txn[r] = tx[k] + a.tbase;
            }
        }
    }
    const RouteTarget &t0 = a.t[0];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n_lock; i += gridDim.x * blockDim.x) {
        const size_t r = (size_t)a.lock_base + i;
        t0.lock_table[r] = p.lock_table[i];
        t0.lock_snap[r] = p.lock_snap[i];
        t0.lock_txn[r] = p.lock_txn[i] + a.tbase;
    }
}

// One workgroup after k_route_count: the column sums of hist (no per-block
// release fence or ticket: a device-scope release per workgroup is an L2
// write-back on this part), published to totals / host and the cursors zeroed.
__global__ __launch_bounds__(256) void k_route_total(const uint32_t *hist, uint32_t nb, int N,
                                                     RouteCountOut o)
{
    __shared__ uint32_t part[256 / 64][kMultiMax];
    uint32_t acc[kMultiMax];
#pragma unroll
    for (int d = 0; d < kMultiMax; ++d) acc[d] = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256)
#pragma unroll
        for (int d = 0; d < kMultiMax; ++d)
            if (d < N) acc[d] += hist[(size_t)b * N + d];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 0; d < kMultiMax; ++d) {
        uint32_t v = acc[d];
        for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
        if (lane == 0) part[w][d] = v;
    }
    __syncthreads();
    const int C = N + 2;
    if (threadIdx.x < C) {
        uint32_t v;
        if (threadIdx.x < N) {
            v = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
            o.ctl[N + 1 + threadIdx.x] = 0;  // the scatter's cursor
        } else {
            v = threadIdx.x == N ? o.n_lock : o.n_txn;
        }
        o.totals[threadIdx.x] = v;
        if (o.host) __hip_atomic_store(&o.host[threadIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    if (o.host && threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&o.host[C], o.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_route_publish(const uint32_t *src, uint32_t words, uint32_t *host, uint32_t seq)
{
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
        __hip_atomic_store(&host[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&host[words], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(kRouteThreads) void k_route_scatter(ProbeView p, RouteSplit sp,
                                                                RouteArgs a, const uint32_t *hist,
                                                                uint32_t *cursor)
{
    extern __shared__ uint64_t lds_w[];
    __shared__ uint32_t cur[kMultiMax];
    uint32_t *lds_g = (uint32_t *)(lds_w + (size_t)sp.W * sp.S);
    const int N = a.N;
    if (threadIdx.x < N) {
        const uint32_t v = hist[(size_t)blockIdx.x * N + threadIdx.x];
        cur[threadIdx.x] = v ? a.base[threadIdx.x] + atomicAdd(&cursor[threadIdx.x], v) : 0;
    }
    route_stage(sp, lds_w, lds_g);
    const uint32_t c0 = blockIdx.x * (uint32_t)kRouteChunk;
    const uint32_t c1 = min(p.n, c0 + (uint32_t)kRouteChunk);
    const int lane = lane_id();
    const uint64_t below = (1ull << lane) - 1;
    const int W = sp.W;
    for (uint32_t base = c0; base < c1; base += kRouteThreads) {
        const uint32_t i = base + threadIdx.x;
        int ra = N, rb = -1;
        uint32_t g = 0;
        if (i < c1) {
            g = p.gid[i];
            ra = route_owner(g, p.lo + i, p.n, W, lds_g, lds_w, sp.S);
            rb = route_owner(g, p.hi + i, p.n, W, lds_g, lds_w, sp.S);
        }
        int dmin = ra, dmax = rb;
        for (int o = 32; o > 0; o >>= 1) {
            dmin = min(dmin, __shfl_xor(dmin, o, 64));
            dmax = max(dmax, __shfl_xor(dmax, o, 64));
        }
        for (int d = dmin; d <= dmax; ++d) {
            const bool mine = ra <= d && d <= rb;
            const uint64_t m = __ballot(mine);
            if (!m) continue;
            uint32_t b0 = 0;
            if (lane == __ffsll((unsigned long long)m) - 1) b0 = atomicAdd(&cur[d], (uint32_t)__popcll(m));
            b0 = __shfl(b0, __ffsll((unsigned long long)m) - 1, 64);
            if (mine) {
                const RouteTarget &t = a.t[d];
                const size_t r = (size_t)b0 + __popcll(m & below);
                for (int j = 0; j < W; ++j) {
                    t.lo[(size_t)j * t.stride + r] = p.lo[(size_t)j * p.n + i];
                    t.hi[(size_t)j * t.stride + r] = p.hi[(size_t)j * p.n + i];
                }
                t.gid[r] = g;
                t.snap[r] = p.snap[i];
                t.txn[r] = p.txn[i] + a.tbase;
            }
        }
    }
    // table-lock probes: all to member 0, behind the other sources' locks
    const RouteTarget &t0 = a.t[0];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n_lock; i += gridDim.x * blockDim.x) {
        const size_t r = (size_t)a.lock_base + i;
        t0.lock_table[r] = p.lock_table[i];
        t0.lock_snap[r] = p.lock_snap[i];
        t0.lock_txn[r] = p.lock_txn[i] + a.tbase;
    }
}

// Received send blocks -> probe columns.  Block of source s at byte offset
// u.boff[s] holds u.n[s] probes as columns lo[W] hi[W] snap (u64) gid txn
// (u32) of stride u.n[s], then (from any source) u.nl[s] lock probes:
// lock_snap (u64) lock_table lock_txn (u32).  Rows land at u.roff[s] / the
// lock offset u.loff[s] of the target.
__global__ __launch_bounds__(256) void k_route_unpack(const uint8_t *raw, RouteUnpack u, RouteTarget t,
                                                     int W)
{
    const uint32_t total = u.roff[u.N];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        int s = 0;
        while (s + 1 < u.N && u.roff[s + 1] <= i) ++s;
        const uint32_t k = i - u.roff[s], n = u.n[s];
        const size_t r = (size_t)u.dst[s] + k;
        const uint64_t *c = (const uint64_t *)(raw + u.boff[s]);
        for (int j = 0; j < W; ++j) {
            t.lo[(size_t)j * t.stride + r] = c[(size_t)j * n + k];
            t.hi[(size_t)j * t.stride + r] = c[(size_t)(W + j) * n + k];
        }
        t.snap[r] = c[(size_t)2 * W * n + k];
        const uint32_t *c32 = (const uint32_t *)(c + (size_t)(2 * W + 1) * n);
        t.gid[r] = c32[k];
        t.txn[r] = c32[n + k];
    }
    const uint32_t ltotal = u.loff[u.N];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ltotal; i += gridDim.x * blockDim.x) {
        int s = 0;
        while (s + 1 < u.N && u.loff[s + 1] <= i) ++s;
        const uint32_t k = i - u.loff[s], n = u.n[s], nl = u.nl[s];
        const uint8_t *b = raw + u.boff[s] + route_block_bytes(W, n, 0);
        const size_t r = (size_t)u.ldst[s] + k;
        t.lock_snap[r] = ((const uint64_t *)b)[k];
        t.lock_table[r] = ((const uint32_t *)(b + 8 * (size_t)nl))[k];
        t.lock_txn[r] = ((const uint32_t *)(b + 12 * (size_t)nl))[k];
    }
}

// out[w] = OR over k < nparts of parts[k][w] (parts may live on peer GPUs)
__global__ void k_or_slices(RouteParts parts, size_t words, uint64_t *out)
{
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint64_t m = 0;
    for (int k = 0; k < parts.n; ++k) m |= parts.p[k][w];
    out[w] = m;
}

// out[w] = bit i set iff verdict byte 64 w + i of any part is nonzero: the
// members' verdict bytes OR-ed and packed in one pass (in-process merges:
// no per-member pack kernel)
__global__ void k_or_bytes(RouteBytes parts, size_t words, uint64_t *out)
{
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < parts.n; ++k) {
        const uint64_t *v = (const uint64_t *)(parts.p[k] + 64 * w);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] |= v[j];
    }
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b) m |= (uint64_t)(((acc[j] >> (8 * b)) & 0xFF) != 0) << (8 * j + b);
    out[w] = m;
}

hipError_t launch_or_bytes(const RouteBytes &parts, size_t words, uint64_t *out, hipStream_t s)
{
    if (!words) return hipSuccess;
    k_or_bytes<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(parts, words, out);
    return hipGetLastError();
}

static size_t route_lds(const RouteSplit &sp) { return 8 * (size_t)sp.W * sp.S + 4 * (size_t)sp.S + 8; }

uint32_t route_blocks(size_t n) { return (uint32_t)((n + kRouteChunk - 1) / kRouteChunk); }

hipError_t launch_route_count(const ProbeView &p, const RouteSplit &sp, int N, uint32_t *hist,
                              const RouteCountOut &o, hipStream_t s)
{
    if (N < 1 || N > kMultiMax) return hipErrorInvalidValue;
    // one block at least (an empty share counts 0)
    const uint32_t nb = std::max<uint32_t>(route_blocks(p.n), 1);
    const size_t lds = route_lds(sp);
    switch (sp.W) {
    case 1: k_route_count_r<1><<<nb, kRouteThreads, lds, s>>>(p, sp, N, hist); break;
    case 2: k_route_count_r<2><<<nb, kRouteThreads, lds, s>>>(p, sp, N, hist); break;
    case 3: k_route_count_r<3><<<nb, kRouteThreads, lds, s>>>(p, sp, N, hist); break;
    case 4: k_route_count_r<4><<<nb, kRouteThreads, lds, s>>>(p, sp, N, hist); break;
    default: k_route_count<<<nb, kRouteThreads, lds, s>>>(p, sp, N, hist);
    }
    k_route_total<<<1, 256, 0, s>>>(hist, nb, N, o);
    return hipGetLastError();
}

hipError_t launch_route_publish(const uint32_t *src, uint32_t words, uint32_t *host, uint32_t seq,
                                hipStream_t s)
{
    k_route_publish<<<1, 256, 0, s>>>(src, words, host, seq);
    return hipGetLastError();
}

hipError_t launch_route_scatter(const ProbeView &p, const RouteSplit &sp, const RouteArgs &a,
                                const uint32_t *hist, uint32_t *cursor, hipStream_t s)
{
    if (a.N < 1 || a.N > kMultiMax) return hipErrorInvalidValue;
    uint32_t nb = route_blocks(p.n);
    if (!nb && p.n_lock) nb = 1;
    if (!nb) return hipSuccess;
    const size_t lds = route_lds(sp);
    switch (sp.W) {
    case 1: k_route_scatter_r<1><<<nb, kRouteThreads, lds, s>>>(p, sp, a, hist, cursor); break;
    case 2: k_route_scatter_r<2><<<nb, kRouteThreads, lds, s>>>(p, sp, a, hist, cursor); break;
    case 3: k_route_scatter_r<3><<<nb, kRouteThreads, lds, s>>>(p, sp, a, hist, cursor); break;
    case 4: k_route_scatter_r<4><<<nb, kRouteThreads, lds, s>>>(p, sp, a, hist, cursor); break;
    default: k_route_scatter<<<nb, kRouteThreads, lds, s>>>(p, sp, a, hist, cursor);
    }
    return hipGetLastError();
}

hipError_t launch_route_unpack(const uint8_t *raw, const RouteUnpack &u, const RouteTarget &t, int W,
                               hipStream_t s)
{
    const uint32_t total = std::max(u.roff[u.N], u.loff[u.N]);
    if (!total) return hipSuccess;
    const uint32_t nb = std::min<uint32_t>((total + 255) / 256, 4096);
    k_route_unpack<<<nb, 256, 0, s>>>(raw, u, t, W);
    return hipGetLastError();
}

hipError_t launch_or_slices(const RouteParts &parts, size_t words, uint64_t *out, hipStream_t s)
{
    if (!words) return hipSuccess;
    k_or_slices<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(parts, words, out);
    return hipGetLastError();
}

hipError_t warm_route()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_route_scatter);
}

}  // namespace hsc
