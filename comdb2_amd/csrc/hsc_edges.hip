// hsc_edges.hip -- read/write conflict pairs before the OR-reduction
// (SURVEY.md §8(f) 4): the A0 join of bdb_osql_serial_check
// (bdb/serializable.c:571 -> serial_check_callback, db/glue.c:2926-2963)
// stops at the first committed write after the snapshot that falls in a read
// range; here every such (read set, writer commit) pair is produced -- the
// rw-antidependency edges of a Jepsen-style dependency graph.
//
// The probe side is the marshalled batch (inclusive word bounds per range,
// as for the verdict path).  The write side is every version of the window
// (the build's key-sorted rows before dedupe: one row per logged write, its
// commit LSN) committed after the batch's oldest snapshot.  Per range probe:
// two binary searches give the rows [pa, pb) of its group inside [lo, hi];
// every row there with LSN > snapshot is a pair (txn, commit LSN).  Counted, scanned and emitted in place (no atomics), then
// sorted and deduplicated with the window's own radix sort / dedupe kernels.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

namespace hsc {

namespace {

// (gid[row], words[.][row]) vs (g, b[j * bs]): <0, 0, >0
__device__ __forceinline__ int cmp_row(const EdgeView &w, uint32_t row, uint32_t g,
                                       const uint64_t *b, size_t bs)
{
    const uint32_t rg = w.gid[row];
    if (rg != g) return rg < g ? -1 : 1;
    for (int j = 0; j < w.W; ++j) {
        const uint64_t x = w.words[(size_t)j * w.stride + row], y = b[(size_t)j * bs];
        if (x != y) return x < y ? -1 : 1;
    }
    return 0;
}

// first row >= bound (upper = false) or > bound (upper = true)
__device__ uint32_t bound_row(const EdgeView &w, uint32_t g, const uint64_t *b, size_t bs,
                              bool upper)
{
    uint32_t lo = 0, len = w.n;
    while (len > 0) {
        const uint32_t half = len >> 1, mid = lo + half;
        const int c = cmp_row(w, mid, g, b, bs);
        if (upper ? c <= 0 : c < 0) {
            lo = mid + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

__global__ void k_edge_count(EdgeView w, ProbeView p, uint2 *span, uint32_t *cnt)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    const uint32_t g = p.gid[q];
    const uint32_t a = bound_row(w, g, p.lo + q, p.n, false);
    const uint32_t b = max(a, bound_row(w, g, p.hi + q, p.n, true));
    const uint64_t s = p.snap[q];
    uint32_t c = 0;
    for (uint32_t r = a; r < b; ++r) c += w.lsn[r] > s;
    span[q] = make_uint2(a, b);
    cnt[q] = c;
}

__global__ void k_edge_emit(EdgeView w, ProbeView p, const uint2 *span, const uint32_t *off,
                            uint32_t *out_txn, uint64_t *out_lsn)
{
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    const uint2 ab = span[q];
    const uint64_t s = p.snap[q];
    const uint32_t t = p.txn[q];
    uint32_t o = off[q];
    for (uint32_t r = ab.x; r < ab.y; ++r) {
        const uint64_t l = w.lsn[r];
        if (l > s) {
            out_txn[o] = t;
            out_lsn[o] = l;
            ++o;
        }
    }
}

__global__ void k_flag_after(const uint64_t *lsn, uint32_t n, uint64_t smin, uint32_t *flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = lsn[i] > smin;
}

__global__ void k_compact_after(EdgeView w, uint64_t smin, const uint32_t *pos, EdgeView o)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= w.n || !(w.lsn[i] > smin)) return;
    const uint32_t d = pos[i];
    ((uint32_t *)o.gid)[d] = w.gid[i];
    ((uint64_t *)o.lsn)[d] = w.lsn[i];
    for (int j = 0; j < w.W; ++j)
        ((uint64_t *)o.words)[(size_t)j * o.stride + d] = w.words[(size_t)j * w.stride + i];
}

}  // namespace

// The versions committed after smin (the batch's oldest snapshot), in key
// order, into o (o.stride rows per word); returns their count in *n_out.
// Only they can pair with a range probe of the batch, so the per-probe scans
// are output sensitive.
hipError_t edge_after(const EdgeView &w, uint64_t smin, uint32_t *flag, uint32_t *scratch,
                      EdgeView &o, uint32_t *n_out, hipStream_t s)
{
    const uint32_t n = w.n;
    k_flag_after<<<(n + 256) / 256, 256, 0, s>>>(w.lsn, n, smin, flag);
    hipError_t e = hipMemsetAsync(flag + n, 0, 4, s);
    if (e != hipSuccess) return e;
    e = scan_exclusive_u32(flag, (size_t)n + 1, scratch, s);
    if (e != hipSuccess) return e;
    k_compact_after<<<(n + 255) / 256, 256, 0, s>>>(w, smin, flag, o);
    e = hipMemcpyAsync(n_out, flag + n, 4, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

hipError_t launch_edge_count(const EdgeView &w, const ProbeView &p, uint2 *span, uint32_t *cnt,
                             hipStream_t s)
{
    if (p.n == 0) return hipSuccess;
    k_edge_count<<<(p.n + 255) / 256, 256, 0, s>>>(w, p, span, cnt);
    return hipGetLastError();
}

hipError_t launch_edge_emit(const EdgeView &w, const ProbeView &p, const uint2 *span,
                            const uint32_t *off, uint32_t *out_txn, uint64_t *out_lsn,
                            hipStream_t s)
{
    if (p.n == 0) return hipSuccess;
    k_edge_emit<<<(p.n + 255) / 256, 256, 0, s>>>(w, p, span, off, out_txn, out_lsn);
    return hipGetLastError();
}

// load this file's code object now (HIP loads it lazily at the first launch
// of one of its kernels: ~1 ms, which would land inside the first build or
// probe -- hsc_ctx_create calls every warm_* once)
hipError_t warm_edges()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void *)k_edge_count);
}

}  // namespace hsc
