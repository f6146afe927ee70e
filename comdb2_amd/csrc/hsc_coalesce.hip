// hsc_coalesce.hip -- the replicant's read-set coalesce on the GPU (SURVEY.md
// §8(f) 3): currangearr_coalesce (db/sqlglue.c:305-311) = qsort by
// currange_cmp (:206-242), currangearr_merge_neighbor (:247-304), again.
//
// One thread per read set runs exactly the reference's algorithm (large
// sets with a consistent order sort level-parallel instead, see CoBig), quirks
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
    // the lower keys compare only when both pointers are non-NULL (a NULL one,
    // HSC_KEY_NULL, ties with every range of the index; a present empty one
    // sorts before the longer keys)
    const int ki = v.lkeylen[i], kj = v.lkeylen[j];
    if (v.lkey_off[i] != HSC_KEY_NULL && v.lkey_off[j] != HSC_KEY_NULL) {
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

// One range's merge fields.  The surviving range p lives in registers while it
// absorbs its neighbours (written back when the next survivor takes over), and
// the next q is loaded one step ahead.  (Measured and dropped: the first 8 key
// bytes of each row in registers, and a 3-stage load pipeline -- both slower.)
struct CoRow {
    uint32_t r;
    int tb, ix, lf, lkl, rf, rl, lk;
    uint64_t lko, ro;
};

__device__ __forceinline__ CoRow co_row(const CoView &v, uint32_t r)
{
    CoRow x;
    x.r = r;
    x.tb = v.tbrank[v.table[r]];
    x.ix = v.idxnum[r];
    x.lf = v.lflag[r];
    x.lkl = v.lkeylen[r];
    x.lko = v.lkey_off[r];
    x.rf = v.w_rflag[r];
    x.rl = v.w_rkeylen[r];
    x.ro = v.w_rkey_off[r];
    x.lk = v.w_islocked[r];
    return x;
}

__device__ __forceinline__ void co_put(const CoView &v, const CoRow &p)
{
    v.w_rflag[p.r] = p.rf;
    v.w_islocked[p.r] = p.lk;
    v.w_rkeylen[p.r] = p.rl;
    v.w_rkey_off[p.r] = p.ro;
}

// currangearr_merge_neighbor (db/sqlglue.c:247-304) over ord[0 .. n); returns
// the new length
// RUN: stop at the first row of another (table rank, idxnum) and return the
// survivors of ord[0 .. that row) (the level-parallel path's runs); *plock =
// the last survivor's lock bit.
template <bool RUN = false>
__device__ uint32_t co_merge(const CoView &v, uint32_t *ord, uint32_t n, int *plock = nullptr)
{
    if (!n) return 0;
    CoRow p = co_row(v, ord[0]);
    CoRow nx = n > 1 ? co_row(v, ord[1]) : p;
    const int rtb = p.tb, rix = p.ix;
    uint32_t j = 0;
    for (uint32_t i = 1; i < n; ++i) {
        const CoRow q = nx;
        if (RUN && (q.tb != rtb || q.ix != rix)) break;
        if (i + 1 < n) nx = co_row(v, ord[i + 1]);
        bool absorbed = false;
        if (p.tb == q.tb) {
            if (p.ix == q.ix) {
                const int m = q.lkl < p.rl ? q.lkl : p.rl;
                if (q.lf || p.rf || keycmp(v, q.lko, p.ro, m) <= 0) {
                    if (p.rf || q.rf) {
                        p.rf = 1;
                        p.ro = HSC_KEY_NULL;  // free(p->rkey); p->rkey = NULL
                        p.rl = 0;
                    } else if (keycmp(v, p.ro, q.ro, p.rl < q.rl ? p.rl : q.rl) < 0) {
                        v.w_rkey_off[q.r] = p.ro;  // pointer swap, lengths stay
                        p.ro = q.ro;
                    }
                    if (p.lf && p.rf) p.lk = 1;
                    absorbed = true;
                }
            } else if (p.lk) {
                absorbed = true;
            }
        }
        if (absorbed) continue;
        co_put(v, p);
        ord[++j] = q.r;
        p = q;
    }
    co_put(v, p);
    if (plock) *plock = p.lk;
    return j + 1;
}

__global__ __launch_bounds__(128) void k_coalesce(CoView v, const uint32_t *isbig)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint32_t)v.ntxn) return;
    if (isbig && isbig[t]) return;  // the level-parallel path below
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

// ---- large sets whose comparator is a consistent order ----
// currange_cmp ties a range with every other range of its (table, index) only
// through a NULL lower key (no lflag, lkey_off == HSC_KEY_NULL) on an unlocked
// range; two left-open ranges compare "first" both ways, which the merge rule
// (cmp(left, right) <= 0 takes the left run) treats exactly like equal keys.
// Without such a tie the order is a total preorder (table rank, locked first,
// idxnum, left-open first, then lexicographic key bytes + length), so glibc's
// merge sort returns the unique stable order, and any stable sort does too.
// The host sends those sets (>= kCoBig ranges) here: each bottom-up merge level
// is one launch over every element of every such set, an element's output slot
// = its index in its run + the number of the other run's elements that go
// before it (a binary search with the same tie rule).  lflag / lkey never
// change and islocked only turns on, so the check holds for the second sort.
struct CoBig {
    const uint32_t *set;  // [nbig] set ids
    const uint32_t *pre;  // [nbig + 1] element prefix
    uint32_t nbig, total;
};

__device__ __forceinline__ uint32_t co_big_of(const CoBig &bg, uint32_t g)
{
    uint32_t lo = 0, hi = bg.nbig;  // last k with pre[k] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (bg.pre[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_co_big_init(CoView v, CoBig bg)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= bg.total) return;
    const uint32_t k = co_big_of(bg, g), t = bg.set[k];
    const uint32_t i = g - bg.pre[k];
    const uint64_t r = (uint64_t)v.off[t] + i;
    v.ord[r] = (uint32_t)r;
    v.w_rflag[r] = v.rflag[r];
    v.w_islocked[r] = v.islocked[r];
    v.w_rkeylen[r] = v.rkeylen[r];
    v.w_rkey_off[r] = v.rkey_off[r];
    if (i == 0) v.count[t] = bg.pre[k + 1] - bg.pre[k];
}

__global__ __launch_bounds__(256) void k_co_big_level(CoView v, CoBig bg, uint32_t w,
                                                      const uint32_t *src, uint32_t *dst)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= bg.total) return;
    const uint32_t k = co_big_of(bg, g), t = bg.set[k];
    const uint32_t i = g - bg.pre[k], n = v.count[t];
    if (i >= n) return;
    const uint64_t b = (uint64_t)v.off[t];
    const uint32_t a0 = i / (2 * w) * (2 * w);
    const uint32_t a1 = min(a0 + w, n), b1 = min(a0 + 2 * w, n);
    const uint32_t x = src[b + i];
    uint32_t pos;
    if (i < a1) {  // left run: right elements with cmp(x, y) > 0 go first
        uint32_t lo = a1, hi = b1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (co_cmp(v, x, src[b + mid]) > 0) lo = mid + 1; else hi = mid;
        }
        pos = i + (lo - a1);
    } else {  // right run: left elements with cmp(y, x) <= 0 go first
        uint32_t lo = a0, hi = a1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (co_cmp(v, src[b + mid], x) <= 0) lo = mid + 1; else hi = mid;
        }
        pos = a0 + (i - a1) + (lo - a0);
    }
    dst[b + pos] = x;
}

__global__ __launch_bounds__(256) void k_co_big_copy(CoView v, CoBig bg)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= bg.total) return;
    const uint32_t k = co_big_of(bg, g), t = bg.set[k];
    const uint32_t i = g - bg.pre[k];
    const uint64_t b = (uint64_t)v.off[t];
    if (i < v.count[t]) v.ord[b + i] = v.tmp[b + i];
}

// Merge scan of the large sets, split into runs of equal (table rank,
// idxnum).  Rows of another table never merge; a run's first row follows the
// previous run's last survivor p, which either starts a new survivor or -- if
// p is locked -- is absorbed with everything after it in p's table (p's
// fields do not change then).  The host admits only sets whose locked ranges
// are open at both ends, so a locked survivor also absorbs the rest of its own
// run: it is always its run's last survivor.  Runs merge independently
// (k_co_big_runs: survivors compacted to the run's head, count and last lock
// bit in tmp[run head]); k_co_big_join then drops the runs a locked survivor
// of their table absorbed and packs the rest, in order (one workgroup per set).
__device__ __forceinline__ uint64_t co_runkey(const CoView &v, uint32_t r)
{
    return (uint64_t)(uint32_t)v.tbrank[v.table[r]] << 32 | (uint32_t)v.idxnum[r];
}

__global__ __launch_bounds__(256) void k_co_big_runs(CoView v, CoBig bg)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= bg.total) return;
    const uint32_t k = co_big_of(bg, g), t = bg.set[k];
    const uint32_t i = g - bg.pre[k], n = v.count[t];
    if (i >= n) return;
    const uint64_t b = (uint64_t)v.off[t];
    uint32_t *ord = v.ord + b;
    // rows keep their run while runs compact (a run writes only its own rows
    // into its own slots), so the neighbour test below is race-free
    const bool head = i == 0 || co_runkey(v, ord[i - 1]) != co_runkey(v, ord[i]);
    uint32_t info = 0;
    if (head) {
        int lk = 0;
        const uint32_t c = co_merge<true>(v, ord + i, n - i, &lk);
        info = c | (uint32_t)lk << 31;
    }
    v.tmp[b + i] = info;
}

constexpr int kJoinT = 256;

__global__ __launch_bounds__(kJoinT) void k_co_big_join(CoView v, CoBig bg, uint32_t *runpos,
                                                        uint32_t *runinfo)
{
    __shared__ uint32_t lds[kJoinT / 64];
    __shared__ uint32_t nruns, mtot;
    const uint32_t k = blockIdx.x, t = bg.set[k];
    const uint32_t n = v.count[t];
    const uint64_t b = (uint64_t)v.off[t];
    uint32_t *ord = v.ord + b, *tmp = v.tmp + b, *rp = runpos + b, *ri = runinfo + 2 * b;
    // run heads, in order
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += kJoinT) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t info = i < n ? tmp[i] : 0;
        uint32_t tot;
        const uint32_t pre = block_excl_scan<kJoinT>(info != 0, lds, tot);
        if (info) {
            rp[base + pre] = i;
            ri[base + pre] = info;
        }
        base += tot;
    }
    __syncthreads();
    // sequential over runs: drop the absorbed ones, output offsets of the rest
    if (threadIdx.x == 0) {
        int64_t locked_tb = -1;
        uint32_t acc = 0;
        for (uint32_t r = 0; r < base; ++r) {
            const uint32_t info = ri[r];
            const int64_t tb = v.tbrank[v.table[ord[rp[r]]]];
            if (tb == locked_tb) {
                ri[r] = ~0u;
                continue;
            }
            ri[r] = acc;
            acc += info & 0x7FFFFFFFu;
            if (info >> 31) locked_tb = tb;
            tmp[rp[r]] = info & 0x7FFFFFFFu;  // survivors of the run, for the copy
        }
        nruns = base;
        mtot = acc;
    }
    __syncthreads();
    const uint32_t R = nruns, m = mtot;
    // survivors staged in the second half of the set's scratch [2b, 2b + 2n)
    uint32_t *out = ri + n;
    for (uint32_t i = threadIdx.x; i < n; i += kJoinT) {
        uint32_t lo = 0, hi = R;  // last run with head <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (rp[mid] <= i) lo = mid; else hi = mid;
        }
        const uint32_t h = rp[lo], dst = ri[lo];
        if (dst == ~0u) continue;
        if (i - h < tmp[h]) out[dst + (i - h)] = ord[i];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += kJoinT) ord[i] = out[i];
    if (threadIdx.x == 0) v.count[t] = m;
}

hipError_t co_big_sort(const CoView &v, const CoBig &bg, uint32_t maxn, hipStream_t s)
{
    const uint32_t nb = (bg.total + 255) / 256;
    bool in_tmp = false;
    for (uint32_t w = 1; w < maxn; w *= 2) {
        k_co_big_level<<<nb, 256, 0, s>>>(v, bg, w, in_tmp ? v.tmp : v.ord, in_tmp ? v.ord : v.tmp);
        in_tmp = !in_tmp;
    }
    if (in_tmp) k_co_big_copy<<<nb, 256, 0, s>>>(v, bg);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_coalesce(const CoView &v, const uint32_t *isbig, const uint32_t *big_set,
                           const uint32_t *big_pre, uint32_t nbig, uint32_t big_total,
                           uint32_t big_maxn, uint32_t *big_runpos, uint32_t *big_scratch,
                           hipStream_t s)
{
    if (v.ntxn <= 0) return hipSuccess;
    k_coalesce<<<(v.ntxn + 127) / 128, 128, 0, s>>>(v, nbig ? isbig : nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nbig == 0 || big_total == 0) return e;
    const CoBig bg{big_set, big_pre, nbig, big_total};
    const uint32_t nb = (big_total + 255) / 256;
    k_co_big_init<<<nb, 256, 0, s>>>(v, bg);
    for (int pass = 0; pass < 2; ++pass) {
        if ((e = co_big_sort(v, bg, big_maxn, s)) != hipSuccess) return e;
        k_co_big_runs<<<nb, 256, 0, s>>>(v, bg);
        k_co_big_join<<<nbig, kJoinT, 0, s>>>(v, bg, big_runpos, big_scratch);
    }
    return hipGetLastError();
}

}  // namespace hsc
