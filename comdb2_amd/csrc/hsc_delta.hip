// hsc_delta.hip -- the incremental part of the resident write window.
//
// The reference sees every commit up to the end of the log on every check
// (bdb/serializable.c:390-539) and commits keep appending (bdb/tran.c:
// 1545-1560).  Rebuilding the main window (radix sort + summaries) per commit
// would cost milliseconds, so committed writes appended after a build go to a
// small delta run instead: rows (gid, key words, commit LSN) kept sorted by
// (gid, words) on the device, one merge launch per append (the appended rows
// are sorted on the host), plus 64-row LSN maxima.  Every probe batch checks
// the delta beside the main window (k_probe_delta: one thread per range, two
// binary searches over the delta and a range maximum), so a verdict is the
// OR of both.  When the delta outgrows its cap the host folds it into the
// main window with one device rebuild (hsc_host.cpp merge_delta).
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace hsc {

namespace {

// out = merge of the delta (d.n rows) and the appended rows a (a.n rows,
// sorted), stable: equal keys keep delta rows first.  One thread per output
// row: its co-rank (how many delta rows precede it, a binary search on its
// merge-path diagonal) names the source row, so a wave writes 64 consecutive
// rows and takes their 64-row LSN maximum with it (no second pass).  Block 0
// also copies the table maxima staged with the rows (nt of them) into place.
// kStage: a lives in the host's pinned staging (a commit's few rows, no
// upload): every block first copies it into LDS, and the searches read that.
template <bool kStage>
__global__ void k_delta_merge(DeltaView d, DeltaView a, uint32_t *ogid, uint64_t *owords,
                              uint64_t *olsn, size_t ostride, uint64_t *bmax,
                              const uint64_t *tmax_src, uint64_t *tmax_dst, uint32_t nt)
{
    if (blockIdx.x == 0)
        for (uint32_t t = threadIdx.x; t < nt; t += blockDim.x) tmax_dst[t] = tmax_src[t];
    if constexpr (kStage) {
        extern __shared__ __attribute__((aligned(16))) uint64_t sa[];  // words [W][n], lsn [n], gid [n]
        const uint32_t k = a.n;
        uint64_t *sw = sa, *sl = sa + (size_t)a.W * k;
        uint32_t *sg = (uint32_t *)(sl + k);
        for (uint32_t i = threadIdx.x; i < (uint32_t)a.W * k; i += blockDim.x)
            sw[i] = a.words[(size_t)(i / k) * a.stride + i % k];
        for (uint32_t i = threadIdx.x; i < k; i += blockDim.x) sl[i] = a.lsn[i], sg[i] = a.gid[i];
        __syncthreads();
        a.words = sw, a.lsn = sl, a.gid = sg, a.stride = k;
    }
    const uint32_t n = d.n + a.n;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t lv = 0;
    if (i < n) {
        // x = delta rows among outputs [0, i): the least x with d[x] > a[i - 1 - x]
        uint32_t lo = i > a.n ? i - a.n : 0, hi = min(i, d.n);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t y = i - 1 - mid;
            // d[mid] <= a[y]: delta row mid precedes appended row y (ties: delta first)
            if (row_cmp(d.gid, d.words, d.stride, d.W, mid, a.gid[y], a.words + y, a.stride) <= 0)
                lo = mid + 1;
            else
                hi = mid;
        }
        const uint32_t x = lo, y = i - x;
        const bool from_d = x < d.n && (y >= a.n || row_cmp(d.gid, d.words, d.stride, d.W, x, a.gid[y],
                                                             a.words + y, a.stride) <= 0);
        const DeltaView &src = from_d ? d : a;
        const uint32_t r = from_d ? x : y;
        ogid[i] = src.gid[r];
        for (int w = 0; w < d.W; ++w) owords[(size_t)w * ostride + i] = src.words[(size_t)w * src.stride + r];
        lv = src.lsn[r];
        olsn[i] = lv;
    }
    // rows [64 b, 64 b + 64) are one wave's (blocks start at multiples of 64)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t v = __shfl_xor(lv, o, 64);
        lv = v > lv ? v : lv;
    }
    if ((threadIdx.x & 63) == 0 && i < n) bmax[i >> 6] = lv;
}

// Range probes against the delta: any row of the range's group inside
// [lo, hi] committed after the snapshot -> flags[txn] = 1.
__global__ __launch_bounds__(256) void k_probe_delta(DeltaView d, ProbeView p, uint8_t *flags)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    if (delta_hit(d, p, q)) flags[p.txn[q]] = 1;
}

}  // namespace

hipError_t delta_merge(const DeltaView &d, const DeltaView &a, uint32_t *ogid, uint64_t *owords,
                       uint64_t *olsn, size_t ostride, uint64_t *bmax, hipStream_t s,
                       const uint64_t *tmax_src, uint64_t *tmax_dst, uint32_t nt, bool stage_a)
{
    const uint32_t n = d.n + a.n;
    if (n == 0 && nt == 0) return hipSuccess;
    const uint32_t blocks = std::max(1u, (n + 255) / 256);
    if (stage_a) {
        if (a.n > kDeltaStageRows) return hipErrorInvalidValue;
        const size_t lds = (8 * (size_t)a.W + 8 + 4) * a.n + 16;
        k_delta_merge<true><<<blocks, 256, lds, s>>>(d, a, ogid, owords, olsn, ostride, bmax, tmax_src,
                                                     tmax_dst, nt);
    } else {
        k_delta_merge<false><<<blocks, 256, 0, s>>>(d, a, ogid, owords, olsn, ostride, bmax, tmax_src,
                                                    tmax_dst, nt);
    }
    return hipGetLastError();
}

hipError_t launch_probe_delta(const DeltaView &d, const ProbeView &p, uint8_t *flags, hipStream_t s)
{
    if (d.n == 0 || p.n == 0) return hipSuccess;
    k_probe_delta<<<(p.n + 255) / 256, 256, 0, s>>>(d, p, flags);
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_delta()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_probe_delta);
}

}  // namespace hsc
