// hsc_coalesce.hip -- the replicant's read-set coalesce on the GPU (SURVEY.md
// §8(f) 3): currangearr_coalesce (db/sqlglue.c:305-311) = qsort by
// currange_cmp (:206-242), currangearr_merge_neighbor (:247-304), again.
//
// One thread per read set runs exactly the reference's algorithm, quirks
// included: the comparator is not a consistent order (two ranges open on the
// left each sort first; a range without a lower key ties with every range),
// so the result depends on the sort algorithm -- glibc's qsort is a top-down
// merge sort (msort: halves n / 2 and n - n / 2, "cmp <= 0 takes the left
// run"), reproduced here iteratively.  merge_neighbor mutates the surviving
// range: its right flag / right key / lock bit (a right-key "swap" moves the
// key bytes but not rkeylen, :265-270), so those four fields live in working
// arrays.  Table names compare by their strcmp rank (host).  Key bytes past
// the end of the key buffer read as 0.
#include "hsc_device.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

namespace hsc {

namespace {

__device__ __forceinline__ int key_byte(const CoView &v, uint64_t off, int i)
{
    return off + (uint64_t)i < v.nkeys ? v.keys[off + (uint64_t)i] : 0;
}

__device__ int keycmp(const CoView &v, uint64_t a, uint64_t b, int n)
{
    for (int i = 0; i < n; ++i) {
        const int x = key_byte(v, a, i), y = key_byte(v, b, i);
        if (x != y) return x - y;
    }
    return 0;
}

// currange_cmp over range rows i, j
__device__ int co_cmp(const CoView &v, uint32_t i, uint32_t j)
{
    const int ti = v.tbrank[v.table[i]], tj = v.tbrank[v.table[j]];
    if (ti != tj) return ti < tj ? -1 : 1;
    const int li = v.w_islocked[i], lj = v.w_islocked[j];
    if (li || lj) return lj - li;
    if (v.idxnum[i] != v.idxnum[j]) return v.idxnum[i] - v.idxnum[j];
    if (v.lflag[i]) return -1;
    if (v.lflag[j]) return 1;
    const int ki = v.lkeylen[i], kj = v.lkeylen[j];
    if (ki > 0 && kj > 0) {
        const int rc = keycmp(v, v.lkey_off[i], v.lkey_off[j], ki < kj ? ki : kj);
        return rc ? rc : ki - kj;
    }
    return 0;
}

// glibc msort_with_tmp over ord[0 .. n) (global rows), iterative post-order
__device__ void co_msort(const CoView &v, uint32_t *ord, uint32_t *tmp, uint32_t n)
{
    struct Frame {
        uint32_t b, n, st;
    } stk[34];
    int sp = 0;
    stk[sp++] = {0, n, 0};
    while (sp) {
        Frame &f = stk[sp - 1];
        if (f.n <= 1) {
            --sp;
            continue;
        }
        const uint32_t n1 = f.n / 2, n2 = f.n - n1;
        if (f.st == 0) {
            f.st = 1;
            stk[sp++] = {f.b, n1, 0};
            continue;
        }
        if (f.st == 1) {
            f.st = 2;
            stk[sp++] = {f.b + n1, n2, 0};
            continue;
        }
        uint32_t i1 = f.b, i2 = f.b + n1, t = f.b;
        const uint32_t e1 = f.b + n1, e2 = f.b + f.n;
        while (i1 < e1 && i2 < e2) {
            if (co_cmp(v, ord[i1], ord[i2]) <= 0)
                tmp[t++] = ord[i1++];
            else
                tmp[t++] = ord[i2++];
        }
        while (i1 < e1) tmp[t++] = ord[i1++];
        for (uint32_t k = f.b; k < t; ++k) ord[k] = tmp[k];  // the right run's tail is in place
        --sp;
    }
}

// currangearr_merge_neighbor over ord[0 .. n); returns the new length
__device__ uint32_t co_merge(const CoView &v, uint32_t *ord, uint32_t n)
{
    if (!n) return 0;
    uint32_t j = 0, i = 1;
    while (i < n) {
        const uint32_t p = ord[j], q = ord[i];
        if (v.tbrank[v.table[p]] == v.tbrank[v.table[q]]) {
            if (v.idxnum[p] == v.idxnum[q]) {
                const int m = v.lkeylen[q] < v.w_rkeylen[p] ? v.lkeylen[q] : v.w_rkeylen[p];
                if (v.lflag[q] || v.w_rflag[p] || keycmp(v, v.lkey_off[q], v.w_rkey_off[p], m) <= 0) {
                    if (v.w_rflag[p] || v.w_rflag[q]) {
                        v.w_rflag[p] = 1;
                        v.w_rkey_off[p] = 0;
                        v.w_rkeylen[p] = 0;
                    } else {
                        const int pl = v.w_rkeylen[p], ql = v.w_rkeylen[q];
                        if (keycmp(v, v.w_rkey_off[p], v.w_rkey_off[q], pl < ql ? pl : ql) < 0) {
                            const uint64_t t = v.w_rkey_off[p];  // pointer swap, lengths stay
                            v.w_rkey_off[p] = v.w_rkey_off[q];
                            v.w_rkey_off[q] = t;
                        }
                    }
                    if (v.lflag[p] && v.w_rflag[p]) v.w_islocked[p] = 1;
                    ++i;
                    continue;
                }
            } else if (v.w_islocked[p]) {
                ++i;
                continue;
            }
        }
        ++j;
        if (j != i) ord[j] = ord[i];
        ++i;
    }
    return j + 1;
}

__global__ __launch_bounds__(128) void k_coalesce(CoView v)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint32_t)v.ntxn) return;
    const uint64_t b = (uint64_t)v.off[t];
    const uint32_t n = (uint32_t)(v.off[t + 1] - v.off[t]);
    uint32_t *ord = v.ord + b, *tmp = v.tmp + b;
    for (uint32_t k = 0; k < n; ++k) {
        const uint64_t r = b + k;
        ord[k] = (uint32_t)r;
        v.w_rflag[r] = v.rflag[r];
        v.w_islocked[r] = v.islocked[r];
        v.w_rkeylen[r] = v.rkeylen[r];
        v.w_rkey_off[r] = v.rkey_off[r];
    }
    co_msort(v, ord, tmp, n);
    uint32_t m = co_merge(v, ord, n);
    co_msort(v, ord, tmp, m);
    m = co_merge(v, ord, m);
    v.count[t] = m;
}

}  // namespace

hipError_t launch_coalesce(const CoView &v, hipStream_t s)
{
    if (v.ntxn <= 0) return hipSuccess;
    k_coalesce<<<(v.ntxn + 127) / 128, 128, 0, s>>>(v);
    return hipGetLastError();
}

}  // namespace hsc
