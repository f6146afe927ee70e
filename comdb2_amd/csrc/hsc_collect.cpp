// hsc_collect.cpp -- batching collector for concurrent callers of the drop-in.
//
// comdb2 runs bdb_osql_serial_check once per transaction, from whichever
// block-processor thread handles that transaction's commit (db/toblock.c:
// 4779-4836 -> bdb/serializable.c:571), so the calls arrive one read set at a
// time from many threads at once.  One device pass costs about the same for
// 1 read set as for a few thousand, so the collector turns those calls into
// batches, group-commit style: every caller pushes its request; a caller that
// finds no leader becomes the leader, takes every pushed request (after an
// optional gather window of max_wait_us), runs them as hip_serial_check_batch
// passes of at most max_batch and hands each caller its verdict.  Requests
// that arrive while a batch runs form the next batch, led by one of their own
// callers -- there is no collector thread, and a lone caller pays one
// ordinary single-set check.
//
// Each request keeps bdb_osql_serial_check's contract: ranges == NULL -> 0
// (no queueing), regop_only requests get the commit-after-snapshot verdict,
// full requests get *file,*offset := end LSN, errors count as 1.
//
// No lock on the request path.  The pending requests and the leader flag
// share one atomic word (a Treiber stack of requests, bit 0 = a leader is
// gathering): a push that finds the bit clear sets it in the same CAS and
// makes its caller the leader, and the leader takes the whole stack and
// clears the bit with one exchange -- so no request is ever left without a
// leader, and no election, queue lock or wake-up is needed to hand the role
// on.  Up to max_inflight batches run at once (hip_serial_check_batch
// releases the context lock while a small batch's kernel runs, so the next
// leader marshals and launches meanwhile); a leader that finds the device
// full sleeps on the gate word until a batch ends, gathering meanwhile.
// Callers sleep on their own request word.  The leader stores the verdicts,
// cuts the batch into about sqrt(n) wake chains and wakes each chain's head,
// which wakes the rest of its chain: the wakes run in parallel instead of one
// thread's 1-2 µs futex call per request.  A done store is the last touch of
// a request (its caller may return right after, so a chain's next link is
// read before it); a wake of a stale stack address is at worst spurious for
// its thread, whose waits all re-check.
//
// r03's collector queued under a mutex and elected leaders by waking
// waiters: with 256 caller threads on a host whose cgroup grants 16 CPUs but
// lets threads run on all 256, the mutex handoffs (a futex wake per queued
// call, serialised) and elections took 120 µs of kernel time per call, the
// quota ran out early in every 100 ms period and every thread stalled for the
// rest of it (p99 77 ms, `scripts/collector_diag.py`: 8 of 8 periods
// throttled, 12 s of system time for 100k calls).
#include "../../include/hip_serial.h"
#include "hsc_internal.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kDone = 1u;       // Req::word: the verdict is ready
constexpr uintptr_t kLead = 1u;      // hsc_collector::state: a leader is gathering

void futex_wait(std::atomic<uint32_t> *w, uint32_t seen)
{
    syscall(SYS_futex, (uint32_t *)w, FUTEX_WAIT_PRIVATE, seen, nullptr, nullptr, 0);
}

void futex_wake(std::atomic<uint32_t> *w, int n)
{
    syscall(SYS_futex, (uint32_t *)w, FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

uint64_t ns_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b)
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
}

}  // namespace

struct hsc_collector {
    hsc_ctx *ctx = nullptr;
    int max_batch = 0;
    int max_wait_us = 0;
    std::atomic<int> max_inflight{4};
    bool premarshal = true;  // callers marshal their own read set before queueing
    struct alignas(64) Req {
        void *ranges;
        unsigned int *file, *offset;
        int regop_only;
        int rc;
        hsc::PreMarshal *pm;  // the caller's marshalled rows, or null
        Req *next;            // the stack below it
        Req *chain;           // (set by the leader) the next request of its wake chain
        bool head;            // (set by the leader) this one wakes the rest of its chain
        std::atomic<uint32_t> word{0};
    };
    // pending requests (a stack of Req*, aligned) | kLead
    alignas(64) std::atomic<uintptr_t> state{0};
    alignas(64) std::atomic<int> running{0};     // batches on the device
    std::atomic<uint32_t> gate{0};               // bumped when a batch ends
    std::atomic<int> gate_waiting{0};            // a leader sleeps on gate
    alignas(64) std::atomic<int> inside{0};      // callers inside hsc_collector_check (last touch: the decrement)
    std::atomic<uint64_t> st_calls{0}, st_batches{0}, st_max_batch{0}, st_pass_ns{0}, st_gate_ns{0},
        st_handout_ns{0};
    // busy = the union of the in-flight passes' intervals: the clock runs from
    // the moment the first of them starts until none is left
    std::mutex busy_mu;
    int busy_depth = 0;
    std::chrono::steady_clock::time_point busy_t0;
    uint64_t st_busy_ns = 0;
};

namespace {

using Req = hsc_collector::Req;

// one device pass over a group of requests that share regop_only
void run_group(hsc_collector *k, Req *const *g, int n, int regop_only)
{
    if (!n) return;
    std::vector<void *> ranges(n);
    std::vector<hsc::PreMarshal *> pm(n);
    std::vector<unsigned int> file(n), offset(n);
    std::vector<int> rc_out(n, 1);
    for (int i = 0; i < n; ++i) {
        ranges[i] = g[i]->ranges;
        pm[i] = g[i]->pm;
        file[i] = *g[i]->file;
        offset[i] = *g[i]->offset;
    }
    const int rc = regop_only ? hip_serial_check_batch(k->ctx, ranges.data(), file.data(),
                                                       offset.data(), 1, n, rc_out.data())
                              : hsc::check_batch_pre(k->ctx, ranges.data(), pm.data(), file.data(),
                                                     offset.data(), n, rc_out.data());
    for (int i = 0; i < n; ++i) {
        *g[i]->file = file[i];  // full mode wrote curlsn back; regop_only left it
        *g[i]->offset = offset[i];
        g[i]->rc = rc ? 1 : rc_out[i];
    }
}

void max_into(std::atomic<uint64_t> &a, uint64_t v)
{
    uint64_t cur = a.load(std::memory_order_relaxed);
    while (v > cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
    }
}

// The leader (holding kLead): wait for room on the device, take every
// pending request, run them, hand out the verdicts.  `me` is the leader's own
// request (in the stack it takes: it pushed before it led).
void lead(hsc_collector *k, Req *me)
{
    using clk = std::chrono::steady_clock;
    const auto tg = clk::now();
    for (;;) {  // the in-flight bound: requests keep piling up on the stack meanwhile
        const uint32_t seen = k->gate.load(std::memory_order_acquire);
        if (k->running.load(std::memory_order_acquire) < k->max_inflight.load(std::memory_order_relaxed))
            break;
        k->gate_waiting.store(1, std::memory_order_seq_cst);
        if (k->running.load(std::memory_order_seq_cst) >= k->max_inflight.load(std::memory_order_relaxed))
            futex_wait(&k->gate, seen);
        k->gate_waiting.store(0, std::memory_order_relaxed);
    }
    if (k->max_wait_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(k->max_wait_us));
    k->running.fetch_add(1, std::memory_order_acq_rel);
    {
        std::lock_guard<std::mutex> g(k->busy_mu);
        if (k->busy_depth++ == 0) k->busy_t0 = clk::now();
    }
    // take the stack and give up the lead in one exchange: the next push
    // becomes the next leader
    const uintptr_t taken = k->state.exchange(0, std::memory_order_acq_rel);
    std::vector<Req *> all;
    for (Req *q = (Req *)(taken & ~kLead); q; q = q->next) all.push_back(q);
    std::reverse(all.begin(), all.end());  // arrival order
    const auto t0 = clk::now();
    k->st_gate_ns.fetch_add(ns_between(tg, t0), std::memory_order_relaxed);
    // regop_only and full requests run as separate passes, max_batch each
    std::stable_partition(all.begin(), all.end(), [](const Req *q) { return q->regop_only != 0; });
    const int nreg = (int)std::count_if(all.begin(), all.end(), [](const Req *q) { return q->regop_only != 0; });
    const int n = (int)all.size();
    for (int a = 0; a < n;) {
        const int end_grp = a < nreg ? nreg : n;
        const int b = std::min(end_grp, a + k->max_batch);
        run_group(k, all.data() + a, b - a, a < nreg ? 1 : 0);
        k->st_batches.fetch_add(1, std::memory_order_relaxed);
        max_into(k->st_max_batch, (uint64_t)(b - a));
        a = b;
    }
    const auto t1 = clk::now();
    k->st_pass_ns.fetch_add(ns_between(t0, t1), std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(k->busy_mu);
        if (--k->busy_depth == 0) k->st_busy_ns += ns_between(k->busy_t0, t1);
    }
    k->running.fetch_sub(1, std::memory_order_seq_cst);
    k->gate.fetch_add(1, std::memory_order_seq_cst);
    if (k->gate_waiting.load(std::memory_order_seq_cst)) futex_wake(&k->gate, 1);
    // hand out in about sqrt(n) chains: the leader wakes each chain's head,
    // every woken head wakes its chain (a futex wake costs a microsecond or
    // two; one thread waking a batch of 50 made its last caller wait ~100 µs)
    std::vector<Req *> &out = all;
    out.erase(std::remove(out.begin(), out.end(), me), out.end());
    const size_t m = out.size();
    size_t L = 1;
    while (L * L < m) ++L;  // chain length
    for (size_t h = 0; h < m; h += L)
        for (size_t i = h; i < std::min(m, h + L); ++i) {
            out[i]->chain = i + 1 < std::min(m, h + L) ? out[i + 1] : nullptr;
            out[i]->head = i == h;
        }
    for (size_t h = 0; h < m; h += L) {  // each store is the last touch of its request
        out[h]->word.store(kDone, std::memory_order_release);
        futex_wake(&out[h]->word, 1);
    }
    k->st_handout_ns.fetch_add(ns_between(t1, clk::now()), std::memory_order_relaxed);
}

}  // namespace

extern "C" {

int hsc_collector_create(hsc_ctx *ctx, int max_batch, int max_wait_us, hsc_collector **out)
{
    if (!ctx || !out || max_batch < 0 || max_wait_us < 0) return HSC_EINVAL;
    hsc_collector *k = new (std::nothrow) hsc_collector;
    if (!k) return HSC_ENOMEM;
    k->ctx = ctx;
    k->max_batch = max_batch ? max_batch : 65536;
    k->max_wait_us = max_wait_us;
    *out = k;
    return HSC_OK;
}

int hsc_collector_set_inflight(hsc_collector *k, int n)
{
    if (!k || n < 1 || n > 8) return HSC_EINVAL;
    k->max_inflight.store(n, std::memory_order_relaxed);
    k->gate.fetch_add(1, std::memory_order_seq_cst);
    futex_wake(&k->gate, INT_MAX);
    return HSC_OK;
}

void hsc_collector_destroy(hsc_collector *k)
{
    if (!k) return;
    // callers still inside hsc_collector_check are a caller bug; drain them
    // anyway (a returning caller's last touch of k is its decrement)
    while (k->inside.load(std::memory_order_acquire) != 0)
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    delete k;
}

int hsc_collector_check(hsc_collector *k, void *ranges, unsigned int *file, unsigned int *offset,
                        int regop_only)
{
    if (!ranges) return 0;  // bdb_osql_serial_check: nothing read -> serializable
    if (!k) return 1;
    // regop_only: answered from the context's published snapshot in the
    // caller's thread, never queued behind full passes (db/toblock.c:4779-4785
    // holds the commit_lock write lock around it)
    if (regop_only) return hsc::ctx_regop_probe(k->ctx, ranges, file, offset);
    hsc_currangearr *a = (hsc_currangearr *)ranges;
    Req r;
    r.ranges = ranges;
    r.file = file ? file : &a->file;
    r.offset = offset ? offset : &a->offset;
    r.regop_only = regop_only;
    r.rc = 1;
    r.pm = nullptr;
    r.chain = nullptr;  // before the push: a leader may set them right after
    r.head = false;
    // Marshal this caller's own read set now, in its own thread, against the
    // context's dictionary snapshot: the leader then copies rows instead of
    // walking every caller's CurRanges.  The object is the thread's own and
    // stays untouched by it until this call returns.
    static thread_local std::unique_ptr<hsc::PreMarshal, void (*)(hsc::PreMarshal *)> tl_pm(
        hsc::premarshal_new(), hsc::premarshal_free);
    if (!regop_only && k->premarshal && tl_pm &&
        hsc::premarshal(k->ctx, a, ((uint64_t)*r.file << 32) | *r.offset, tl_pm.get()))
        r.pm = tl_pm.get();
    k->inside.fetch_add(1, std::memory_order_relaxed);
    k->st_calls.fetch_add(1, std::memory_order_relaxed);
    // push; a push onto a stack with no leader makes this caller the leader
    uintptr_t old = k->state.load(std::memory_order_relaxed);
    bool leader;
    for (;;) {
        r.next = (Req *)(old & ~kLead);
        leader = !(old & kLead);
        if (k->state.compare_exchange_weak(old, (uintptr_t)&r | kLead, std::memory_order_acq_rel,
                                           std::memory_order_relaxed))
            break;
    }
    if (leader) {
        lead(k, &r);  // r was taken with the rest (it is in the stack the leader took)
    } else {
        while (!(r.word.load(std::memory_order_acquire) & kDone)) futex_wait(&r.word, 0);
        // a chain's head wakes the rest of it (each link read before its
        // done store: the request may return right after it)
        for (Req *q = r.head ? r.chain : nullptr; q;) {
            Req *nx = q->chain;
            q->word.store(kDone, std::memory_order_release);
            futex_wake(&q->word, 1);
            q = nx;
        }
    }
    const int rc = r.rc;
    k->inside.fetch_sub(1, std::memory_order_release);  // last touch of k
    return rc;
}

int hsc_collector_get_stats(hsc_collector *k, hsc_collector_stats *out)
{
    if (!k || !out) return HSC_EINVAL;
    out->calls = k->st_calls.load(std::memory_order_relaxed);
    out->batches = k->st_batches.load(std::memory_order_relaxed);
    out->max_batch = k->st_max_batch.load(std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(k->busy_mu);
        out->busy_ns = k->st_busy_ns;
    }
    out->pass_ns = k->st_pass_ns.load(std::memory_order_relaxed);
    out->gate_ns = k->st_gate_ns.load(std::memory_order_relaxed);
    out->handout_ns = k->st_handout_ns.load(std::memory_order_relaxed);
    return HSC_OK;
}

}  // extern "C"
