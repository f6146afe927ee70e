// hsc_collect.cpp -- batching collector for concurrent callers of the drop-in.
//
// comdb2 runs bdb_osql_serial_check once per transaction, from whichever
// block-processor thread handles that transaction's commit (db/toblock.c:
// 4779-4836 -> bdb/serializable.c:571), so the calls arrive one read set at a
// time from many threads at once.  One device pass costs about the same for
// 1 read set as for a few thousand, so the collector turns those calls into
// batches, group-commit style: every caller queues its request; the first
// caller that finds no leader elected becomes the leader, takes everything
// queued (up to max_batch, after an optional gather window of max_wait_us),
// runs it as one hip_serial_check_batch and hands each caller its verdict.
// Requests that arrive while a batch runs form the next batch, led by one of
// their own callers -- there is no collector thread, and a lone caller pays
// one ordinary single-set check.
//
// Each request keeps bdb_osql_serial_check's contract: ranges == NULL -> 0
// (no queueing), regop_only requests get the commit-after-snapshot verdict,
// full requests get *file,*offset := end LSN, errors count as 1.
//
// Up to max_inflight batches run at once: hip_serial_check_batch releases the
// context lock while a small batch's kernel runs, so the next leader marshals
// and launches its batch meanwhile (the kernels queue on the context's
// stream).  Callers sleep on the futex word of their batch (a request takes
// the id of the batch open when it queues); a finished batch sets its
// callers' done bits after dropping the collector lock (the set is the last
// touch of a request: its caller may return right after), then wakes the
// whole batch with one futex call, and the woken callers return without
// taking the collector lock.
//
// The next leader is designated, not raced for: when a leader takes its
// batch (or a batch ends with requests queued and none elected), the oldest
// queued request is marked to lead and only waiters whose wake bit matches
// its (FUTEX_WAKE_BITSET, one of 32 bits per request) are woken -- waking the
// whole queue to elect one of them made every election a thundering herd of
// lock acquisitions, which on a CPU-quota'd host (256 caller threads, 16 CPUs
// of quota) burnt the quota and stalled every thread for the rest of the
// period (p99 77 ms in r03).
#include "../../include/hip_serial.h"
#include "hsc_internal.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kDone = 1u;  // Req::word: the verdict is ready
constexpr uint32_t kChans = 16;  // batch wait words (more than batches alive at once: <= 4 + 1)

// wait on w while it holds `seen`, for a wake whose bitset meets `bits`
void futex_wait(std::atomic<uint32_t> *w, uint32_t seen, uint32_t bits = FUTEX_BITSET_MATCH_ANY)
{
    syscall(SYS_futex, (uint32_t *)w, FUTEX_WAIT_BITSET_PRIVATE, seen, nullptr, nullptr, bits);
}

void futex_wake(std::atomic<uint32_t> *w, uint32_t bits = FUTEX_BITSET_MATCH_ANY)
{
    syscall(SYS_futex, (uint32_t *)w, FUTEX_WAKE_BITSET_PRIVATE, INT_MAX, nullptr, nullptr, bits);
}

}  // namespace

struct hsc_collector {
    hsc_ctx *ctx = nullptr;
    int max_batch = 0;
    int max_wait_us = 0;
    int max_inflight = 2;
    bool premarshal = true;  // callers marshal their own read set before queueing
    std::mutex m;
    struct Req {
        void *ranges;
        unsigned int *file, *offset;
        int regop_only;
        int rc;
        hsc::PreMarshal *pm;  // the caller's marshalled rows, or null
        bool queued;    // in q (under m): not yet taken into a batch
        bool lead;      // (under m) designated to lead the next batch
        uint32_t bit;   // its futex wake bit (leader designation wakes only that bit)
        uint32_t chan;  // the batch id open when it queued (its wait word: chan % kChans)
        std::atomic<uint32_t> word{0};
    };
    std::deque<Req *> q;
    bool elected = false;  // a leader is waiting to take the next batch
    int running = 0;       // batches on the device
    uint32_t open_id = 0;  // the batch queued requests will join
    uint32_t next_bit = 0;  // round-robin wake bits
    std::atomic<uint32_t> chan[kChans];  // per-batch wait words (bumped at each wake)
    std::condition_variable run_cv;     // a batch finished (the elected leader waits)
    std::condition_variable arrive_cv;  // a request queued (a gathering leader waits)
    std::atomic<int> inside{0};         // callers inside hsc_collector_check (last touch: the decrement)
    hsc_collector_stats st{};           // (under m, but handout_ns:)
    std::atomic<uint64_t> st_handout_ns{0};
    hsc_collector()
    {
        for (auto &c : chan) c.store(0, std::memory_order_relaxed);
    }
};

namespace {

// wake the callers sleeping on batch word `id` (bits: only those whose wake
// bit is among them) to re-check
void wake(hsc_collector *k, uint32_t id, uint32_t bits = FUTEX_BITSET_MATCH_ANY)
{
    std::atomic<uint32_t> &w = k->chan[id % kChans];
    w.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&w, bits);
}

// (under m) the oldest queued request leads the next batch: mark it and wake
// the waiters of its word that share its bit.  Returns the (word, bit) to
// wake once the lock is dropped, or bit 0 when there is nothing to do.
std::pair<uint32_t, uint32_t> designate(hsc_collector *k)
{
    if (k->elected || k->q.empty()) return {0, 0};
    hsc_collector::Req *q = k->q.front();
    q->lead = true;
    k->elected = true;
    return {q->chan, q->bit};
}

// one device pass over a group of requests that share regop_only
void run_group(hsc_collector *k, std::vector<hsc_collector::Req *> &g, int regop_only)
{
    const int n = (int)g.size();
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
    if (!k || n < 1 || n > 4) return HSC_EINVAL;
    std::lock_guard<std::mutex> g(k->m);
    k->max_inflight = n;
    k->run_cv.notify_all();
    return HSC_OK;
}

void hsc_collector_destroy(hsc_collector *k)
{
    if (!k) return;
    // callers still inside hsc_collector_check are a caller bug; drain them
    // anyway (a returning caller's last touch of k is its decrement)
    while (k->inside.load(std::memory_order_acquire) != 0)
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    { std::lock_guard<std::mutex> g(k->m); }  // a leader still unlocking
    delete k;
}

int hsc_collector_check(hsc_collector *k, void *ranges, unsigned int *file, unsigned int *offset,
                        int regop_only)
{
    if (!ranges) return 0;  // bdb_osql_serial_check: nothing read -> serializable
    if (!k) return 1;
    hsc_currangearr *a = (hsc_currangearr *)ranges;
    hsc_collector::Req r;
    r.ranges = ranges;
    r.file = file ? file : &a->file;
    r.offset = offset ? offset : &a->offset;
    r.regop_only = regop_only;
    r.rc = 1;
    r.queued = true;
    r.pm = nullptr;
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
    std::unique_lock<std::mutex> lk(k->m);
    r.chan = k->open_id;
    r.bit = 1u << (k->next_bit++ & 31);
    r.lead = false;
    k->q.push_back(&r);
    k->st.calls++;
    if (k->max_wait_us > 0) k->arrive_cv.notify_one();
    if (!k->elected) {  // nobody leads the next batch yet: this caller does
        k->elected = true;
        r.lead = true;
    }
    for (;;) {  // under lk
        if (!r.queued) {
            // in a batch: wait for the done bit without the lock (the batch's
            // leader sets it, then bumps and wakes the batch word)
            std::atomic<uint32_t> &w = k->chan[r.chan % kChans];
            lk.unlock();
            for (;;) {
                const uint32_t seen = w.load(std::memory_order_acquire);
                if (r.word.load(std::memory_order_acquire) & kDone) break;
                futex_wait(&w, seen);
            }
            break;
        }
        if (!r.lead) {  // queued: sleep until taken into a batch or designated
            std::atomic<uint32_t> &w = k->chan[r.chan % kChans];
            const uint32_t seen = w.load(std::memory_order_acquire);
            lk.unlock();
            futex_wait(&w, seen, r.bit);
            if (r.word.load(std::memory_order_acquire) & kDone) break;  // taken and answered meanwhile
            lk.lock();
            continue;
        }
        // this caller leads the next batch
        const auto tg = std::chrono::steady_clock::now();
        k->run_cv.wait(lk, [k] { return k->running < k->max_inflight; });
        k->st.gate_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(
                             std::chrono::steady_clock::now() - tg).count();
        if (k->max_wait_us > 0 && (int)k->q.size() < k->max_batch)
            k->arrive_cv.wait_for(lk, std::chrono::microseconds(k->max_wait_us),
                                  [k] { return (int)k->q.size() >= k->max_batch; });
        const size_t take = std::min(k->q.size(), (size_t)k->max_batch);
        std::vector<hsc_collector::Req *> full, regop;
        std::vector<uint32_t> ids;  // batch words of the taken requests (one, or two after a max_batch cut)
        bool mine = false;  // max_batch may leave this caller's own request queued
        for (size_t i = 0; i < take; ++i) {
            hsc_collector::Req *q = k->q.front();
            k->q.pop_front();
            q->queued = false;
            q->lead = false;
            mine |= q == &r;
            if (std::find(ids.begin(), ids.end(), q->chan) == ids.end()) ids.push_back(q->chan);
            (q->regop_only ? regop : full).push_back(q);
        }
        r.lead = false;
        k->open_id++;  // later arrivals form the next batch
        k->running++;
        k->elected = false;
        // requests max_batch left queued join the next batch
        for (hsc_collector::Req *q : k->q) q->chan = k->open_id;
        // the next batch's leader: designated now, it gathers while this one runs
        const auto nl = designate(k);
        lk.unlock();
        if (nl.second) wake(k, nl.first, nl.second);
        const auto t0 = std::chrono::steady_clock::now();
        run_group(k, regop, 1);
        run_group(k, full, 0);
        const auto t1 = std::chrono::steady_clock::now();
        lk.lock();
        k->running--;
        k->st.busy_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        k->st.batches++;
        k->st.max_batch = std::max<uint64_t>(k->st.max_batch, take);
        k->run_cv.notify_one();
        const auto nl2 = designate(k);
        lk.unlock();
        if (nl2.second) wake(k, nl2.first, nl2.second);
        // hand out the verdicts: each done bit is the last touch of its
        // request, then one wake per batch word
        for (auto *g : {&regop, &full})
            for (hsc_collector::Req *q : *g)
                if (q != &r) q->word.fetch_or(kDone, std::memory_order_release);
        for (uint32_t id : ids) wake(k, id);
        k->st_handout_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                       std::chrono::steady_clock::now() - t1).count(),
                                   std::memory_order_relaxed);
        if (mine) break;
        lk.lock();
    }
    const int rc = r.rc;
    k->inside.fetch_sub(1, std::memory_order_release);  // last touch of k
    return rc;
}

int hsc_collector_get_stats(hsc_collector *k, hsc_collector_stats *out)
{
    if (!k || !out) return HSC_EINVAL;
    std::lock_guard<std::mutex> g(k->m);
    *out = k->st;
    out->handout_ns = k->st_handout_ns.load(std::memory_order_relaxed);
    return HSC_OK;
}

}  // extern "C"
