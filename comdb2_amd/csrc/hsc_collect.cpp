// hsc_collect.cpp -- batching collector for concurrent callers of the drop-in.
//
// comdb2 runs bdb_osql_serial_check once per transaction, from whichever
// block-processor thread handles that transaction's commit (db/toblock.c:
// 4779-4836 -> bdb/serializable.c:571), so the calls arrive one read set at a
// time from many threads at once.  One device pass costs about the same for
// 1 read set as for a few thousand, so the collector turns those calls into
// batches, group-commit style: every caller queues its request; the first
// caller that finds no batch running becomes the leader, takes everything
// queued (up to max_batch, after an optional gather window of max_wait_us),
// runs it as one hip_serial_check_batch and hands each caller its verdict.
// Requests that arrive while a batch runs form the next batch, led by one of
// their own callers -- there is no collector thread, and a lone caller pays
// one ordinary single-set check.
//
// Each request keeps bdb_osql_serial_check's contract: ranges == NULL -> 0
// (no queueing), regop_only requests get the commit-after-snapshot verdict,
// full requests get *file,*offset := end LSN, errors count as 1.
#include "../../include/hip_serial.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>

struct hsc_collector {
    hsc_ctx *ctx = nullptr;
    int max_batch = 0;
    int max_wait_us = 0;
    std::mutex m;
    struct Req {
        void *ranges;
        unsigned int *file, *offset;
        int regop_only;
        int rc;
        bool done;
        std::condition_variable cv;  // this caller's wake-up: done, or elected leader
    };
    std::deque<Req *> q;
    bool elected = false;  // a leader is waiting to take the next batch
    bool running = false;  // a batch is on the device
    std::condition_variable run_cv;     // the running batch finished (elected leader waits)
    std::condition_variable arrive_cv;  // a request queued (gathering leader waits)
    int inside = 0;                     // callers inside hsc_collector_check
    std::condition_variable idle_cv;    // inside dropped to 0 (destroy waits)
    hsc_collector_stats st{};
};

namespace {

// one device pass over a group of requests that share regop_only
void run_group(hsc_collector *k, std::vector<hsc_collector::Req *> &g, int regop_only)
{
    const int n = (int)g.size();
    if (!n) return;
    std::vector<void *> ranges(n);
    std::vector<unsigned int> file(n), offset(n);
    std::vector<int> rc_out(n, 1);
    for (int i = 0; i < n; ++i) {
        ranges[i] = g[i]->ranges;
        file[i] = *g[i]->file;
        offset[i] = *g[i]->offset;
    }
    const int rc = hip_serial_check_batch(k->ctx, ranges.data(), file.data(), offset.data(),
                                          regop_only, n, rc_out.data());
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

void hsc_collector_destroy(hsc_collector *k)
{
    if (!k) return;
    {  // callers still inside hsc_collector_check are a caller bug; drain them anyway
        std::unique_lock<std::mutex> lk(k->m);
        k->idle_cv.wait(lk, [k] { return k->inside == 0; });
    }
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
    r.done = false;
    std::unique_lock<std::mutex> lk(k->m);
    k->q.push_back(&r);
    k->st.calls++;
    k->inside++;
    k->arrive_cv.notify_one();
    // Waiters sleep on their own condition variable: a finished batch wakes
    // exactly its callers, and the next leader is elected (and waiting for the
    // device) while the current batch still runs, so its wake-up latency hides
    // behind the device pass.
    while (!r.done) {
        if (k->elected) {
            r.cv.wait(lk);
            continue;
        }
        k->elected = true;  // this caller leads the next batch
        k->run_cv.wait(lk, [k] { return !k->running; });
        if (k->max_wait_us > 0 && (int)k->q.size() < k->max_batch)
            k->arrive_cv.wait_for(lk, std::chrono::microseconds(k->max_wait_us),
                                  [k] { return (int)k->q.size() >= k->max_batch; });
        const size_t take = std::min(k->q.size(), (size_t)k->max_batch);
        std::vector<hsc_collector::Req *> full, regop;
        for (size_t i = 0; i < take; ++i) {
            hsc_collector::Req *q = k->q.front();
            k->q.pop_front();
            (q->regop_only ? regop : full).push_back(q);
        }
        k->running = true;
        k->elected = false;
        if (!k->q.empty()) k->q.front()->cv.notify_one();  // elect the next leader now
        lk.unlock();
        const auto t0 = std::chrono::steady_clock::now();
        run_group(k, regop, 1);
        run_group(k, full, 0);
        const auto t1 = std::chrono::steady_clock::now();
        lk.lock();
        k->running = false;
        k->st.busy_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        k->st.batches++;
        k->st.max_batch = std::max<uint64_t>(k->st.max_batch, take);
        for (auto *g : {&regop, &full})
            for (hsc_collector::Req *q : *g) {
                q->done = true;
                if (q != &r) q->cv.notify_one();
            }
        k->run_cv.notify_one();
        if (!k->elected && !k->q.empty()) k->q.front()->cv.notify_one();
    }
    if (--k->inside == 0) k->idle_cv.notify_all();
    return r.rc;
}

int hsc_collector_get_stats(hsc_collector *k, hsc_collector_stats *out)
{
    if (!k || !out) return HSC_EINVAL;
    std::lock_guard<std::mutex> g(k->m);
    *out = k->st;
    return HSC_OK;
}

}  // extern "C"
