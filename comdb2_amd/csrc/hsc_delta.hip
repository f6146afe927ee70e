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

namespace hsc {

namespace {

// out = merge of the delta (d.n rows) and the appended rows a (a.n rows,
// sorted), stable: equal keys keep delta rows first.  One thread per row.
__global__ void k_delta_merge(DeltaView d, DeltaView a, uint32_t *ogid, uint64_t *owords,
                              uint64_t *olsn, size_t ostride)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t pos;
    const DeltaView *src;
    uint32_t r;
    if (i < d.n) {  // delta row i: + appended rows strictly below it
        uint32_t lo = 0, hi = a.n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            // a[mid] < d[i] <=> d[i] > a[mid]
            if (row_cmp(d.gid, d.words, d.stride, d.W, i, a.gid[mid], a.words + mid, a.stride) > 0)
                lo = mid + 1;
            else
                hi = mid;
        }
        pos = i + lo;
        src = &d;
        r = i;
    } else if (i < d.n + a.n) {  // appended row j: + delta rows <= it
        const uint32_t j = i - d.n;
        pos = j + delta_count(d, a.gid[j], a.words + j, a.stride, false);
        src = &a;
        r = j;
    } else {
        return;
    }
    ogid[pos] = src->gid[r];
    for (int w = 0; w < d.W; ++w) owords[(size_t)w * ostride + pos] = src->words[(size_t)w * src->stride + r];
    olsn[pos] = src->lsn[r];
}

__global__ void k_delta_bmax(const uint64_t *lsn, uint32_t n, uint64_t *bmax)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if ((size_t)b * 64 >= n) return;
    uint64_t m = 0;
    const uint32_t e = min(n, (b + 1) * 64);
    for (uint32_t i = b * 64; i < e; ++i) m = lsn[i] > m ? lsn[i] : m;
    bmax[b] = m;
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
                       uint64_t *olsn, size_t ostride, uint64_t *bmax, hipStream_t s)
{
    const uint32_t n = d.n + a.n;
    if (n == 0) return hipSuccess;
    k_delta_merge<<<(n + 255) / 256, 256, 0, s>>>(d, a, ogid, owords, olsn, ostride);
    const uint32_t nb = (n + 63) / 64;
    k_delta_bmax<<<(nb + 255) / 256, 256, 0, s>>>(olsn, n, bmax);
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
    return hipFuncGetAttributes(&a, (const void *)k_delta_bmax);
}

}  // namespace hsc
