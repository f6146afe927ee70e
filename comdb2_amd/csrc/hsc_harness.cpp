// hsc_harness.cpp -- harness support, not on the check path: CurRangeArr
// objects laid out the way comdb2 holds a read set on the master, built from
// flat read sets, so that tests and the bench can drive the drop-in entry
// (hip_serial_check_batch) with what a caller would pass it.
//
// Each read set becomes a CurRangeArr (db/comdb2.h:1117-1124, size / cap /
// snapshot LSN / NULL hash / an array of CurRange pointers) whose CurRange's
// (:1105-1115) are separate heap objects with a strdup'd table name and
// malloc'd key bytes, as serial_readset_get leaves them (db/osqlcomm.c:948-993;
// a key the message carries is malloc'd even when empty, an absent one is
// NULL: HSC_KEY_NULL in the flat form).
#include "../../include/hip_serial.h"

#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

void free_arr(hsc_currangearr *a)
{
    if (!a) return;
    for (int k = 0; k < a->size; ++k) {
        hsc_currange *r = a->ranges[k];
        if (!r) continue;
        free(r->tbname);
        free(r->lkey);
        free(r->rkey);
        free(r);
    }
    free(a->ranges);
    free(a);
}

// p-quantile of v (sorted in place); 0 for an empty v
double quant(std::vector<float> &v, double p)
{
    if (v.empty()) return 0;
    const size_t k = std::min(v.size() - 1, (size_t)(p * (double)v.size()));
    std::nth_element(v.begin(), v.begin() + (long)k, v.end());
    return v[k];
}

void *dup_key(const uint8_t *keys, uint64_t off, int len)
{
    if (off == HSC_KEY_NULL) return nullptr;
    void *p = malloc(len > 0 ? (size_t)len : 1);
    if (p && len > 0) memcpy(p, keys + off, (size_t)len);
    return p;
}

}  // namespace

extern "C" {

int hsc_currangearrs_build(const hsc_readsets *rs, void ***out)
{
    if (!rs || !out || rs->ntxn < 0) return HSC_EINVAL;
    *out = nullptr;
    void **arrs = (void **)calloc((size_t)rs->ntxn + 1, sizeof(void *));
    if (!arrs) return HSC_ENOMEM;
    for (int t = 0; t < rs->ntxn; ++t) {
        const int64_t r0 = rs->txn_off[t];
        const int n = (int)(rs->txn_off[t + 1] - r0);
        hsc_currangearr *a = (hsc_currangearr *)calloc(1, sizeof *a);
        if (!a) goto oom;
        arrs[t] = a;
        a->cap = n < 2 ? 2 : n;  // CURRANGEARR_INIT_CAP 2 (db/sql.h:275), doubled as needed
        a->file = (unsigned)(rs->snap[t] >> 32);
        a->offset = (unsigned)rs->snap[t];
        a->ranges = (hsc_currange **)calloc((size_t)a->cap, sizeof(hsc_currange *));
        if (!a->ranges) goto oom;
        for (int k = 0; k < n; ++k) {
            const int64_t r = r0 + k;
            hsc_currange *c = (hsc_currange *)calloc(1, sizeof *c);
            if (!c) goto oom;
            a->ranges[a->size++] = c;
            const int32_t tb = rs->table[r];
            if (tb < 0 || tb >= rs->ntbnames || !rs->tbnames[tb]) {
                free_arr(a);
                arrs[t] = nullptr;
                for (int q = 0; q < t; ++q) free_arr((hsc_currangearr *)arrs[q]);
                free(arrs);
                return HSC_EINVAL;
            }
            c->tbname = strdup(rs->tbnames[tb]);
            c->idxnum = rs->idxnum[r];
            c->lflag = rs->lflag[r];
            c->rflag = rs->rflag[r];
            c->islocked = rs->islocked[r];
            c->lkeylen = rs->lkeylen[r];
            c->rkeylen = rs->rkeylen[r];
            c->lkey = dup_key(rs->keys, rs->lkey_off[r], c->lkeylen);
            c->rkey = dup_key(rs->keys, rs->rkey_off[r], c->rkeylen);
            if (!c->tbname) goto oom;
        }
    }
    *out = arrs;
    return HSC_OK;
oom:
    for (int q = 0; q < rs->ntxn; ++q) free_arr((hsc_currangearr *)arrs[q]);
    free(arrs);
    return HSC_ENOMEM;
}

void hsc_currangearrs_free(void **arrs, int n)
{
    if (!arrs) return;
    for (int t = 0; t < n; ++t) free_arr((hsc_currangearr *)arrs[t]);
    free(arrs);
}

int hsc_harness_concurrent(hsc_ctx *ctx, hsc_collector *col, void *const *arrs, int n,
                           int nthreads, int rounds, int regop_only, int *rc_out,
                           hsc_concurrent_result *res)
{
    if (!ctx || n < 0 || (n && (!arrs || !rc_out)) || nthreads < 1 || rounds < 1 || !res)
        return HSC_EINVAL;
    using clk = std::chrono::steady_clock;
    std::vector<std::vector<float>> lat(nthreads);
    auto body = [&](int t) {
        for (int r = 0; r < rounds; ++r)
            for (int i = t; i < n; i += nthreads) {
                const hsc_currangearr *a = (const hsc_currangearr *)arrs[i];
                unsigned int file = a ? a->file : 0, offset = a ? a->offset : 0;
                const auto t0 = clk::now();
                const int rc = col ? hsc_collector_check(col, arrs[i], &file, &offset, regop_only)
                                   : hip_bdb_osql_serial_check(ctx, arrs[i], &file, &offset,
                                                               regop_only);
                lat[t].push_back(std::chrono::duration<float, std::micro>(clk::now() - t0).count());
                rc_out[i] = rc;
            }
    };
    const auto w0 = clk::now();
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(body, t);
    body(0);
    for (auto &x : th) x.join();
    res->seconds = std::chrono::duration<double>(clk::now() - w0).count();
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    res->calls = all.size();
    res->lat_mean_us = res->lat_p50_us = res->lat_p99_us = 0;
    if (!all.empty()) {
        double s = 0;
        for (float x : all) s += x;
        res->lat_mean_us = s / all.size();
        std::sort(all.begin(), all.end());
        res->lat_p50_us = all[all.size() / 2];
        res->lat_p99_us = all[std::min(all.size() - 1, all.size() * 99 / 100)];
    }
    return HSC_OK;
}

int hsc_harness_commit_protocol(hsc_ctx *ctx, const hsc_protocol_txn *txns, int ntxn, const int *events,
                                int nevents, int nthreads, int *rc_out, int64_t *commit_seq, uint64_t *snap_out,
                                uint64_t *check_end_out, hsc_protocol_result *res)
{
    if (!ctx || ntxn < 0 || nevents < 0 || (ntxn && !txns) || (nevents && !events) || nthreads < 1 || !res ||
        (ntxn && (!rc_out || !commit_seq || !snap_out || !check_end_out)))
        return HSC_EINVAL;
    for (int k = 0; k < nevents; ++k) {
        const int t = events[k] >= 0 ? events[k] : ~events[k];
        if (t >= ntxn || !txns[t].arr) return HSC_EINVAL;
    }
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<float, std::micro>(b - a).count();
    };
    pthread_rwlock_t commit_lock;  // db/toblock.c's commit_lock
    if (pthread_rwlock_init(&commit_lock, nullptr)) return HSC_ENOMEM;
    std::vector<std::atomic<int>> begun(ntxn);
    for (auto &b : begun) b.store(0, std::memory_order_relaxed);
    for (int t = 0; t < ntxn; ++t) rc_out[t] = 0, commit_seq[t] = -1, snap_out[t] = 0, check_end_out[t] = 0;
    std::atomic<int> next{0};
    std::atomic<int> err{HSC_OK};
    int64_t ncommit = 0;  // under the write lock
    struct Lat {
        std::vector<float> regop, full, hold, commit;
        uint64_t commits = 0, aborts = 0;
    };
    std::vector<Lat> lat(nthreads);
    auto body = [&](int th) {
        Lat &L = lat[th];
        std::vector<hsc_write> w;
        for (;;) {
            const int k = next.fetch_add(1, std::memory_order_relaxed);
            if (k >= nevents || err.load(std::memory_order_relaxed)) return;
            const int e = events[k];
            if (e >= 0) {  // begin: the snapshot is the end of the log now
                hsc_currangearr *a = (hsc_currangearr *)txns[e].arr;
                const uint64_t S = hsc_window_end(ctx);
                a->file = (unsigned int)(S >> 32), a->offset = (unsigned int)S;
                snap_out[e] = S;
                begun[e].store(1, std::memory_order_release);
                continue;
            }
            const int t = ~e;
            while (!begun[t].load(std::memory_order_acquire)) std::this_thread::yield();
            const hsc_protocol_txn &x = txns[t];
            if (x.nwrites <= 0) continue;  // read-only: never checked (db/sqloffload.c:280-287)
            hsc_currangearr *a = (hsc_currangearr *)x.arr;
            const auto c0 = clk::now();
            pthread_rwlock_rdlock(&commit_lock);
            pthread_rwlock_unlock(&commit_lock);
            pthread_rwlock_wrlock(&commit_lock);
            auto held = clk::now();
            bool aborted = false;
            for (;;) {
                const auto r0 = clk::now();
                const int busy = hip_bdb_osql_serial_check(ctx, a, &a->file, &a->offset, 1);
                L.regop.push_back(us(r0, clk::now()));
                if (!busy) break;
                L.hold.push_back(us(held, clk::now()));
                pthread_rwlock_unlock(&commit_lock);
                const auto f0 = clk::now();
                const int rc = hip_bdb_osql_serial_check(ctx, a, &a->file, &a->offset, 0);
                L.full.push_back(us(f0, clk::now()));
                check_end_out[t] = ((uint64_t)a->file << 32) | a->offset;
                if (rc) {
                    aborted = true;
                    break;
                }
                pthread_rwlock_wrlock(&commit_lock);
                held = clk::now();
            }
            if (aborted) {
                rc_out[t] = 1;
                L.aborts++;
                L.commit.push_back(us(c0, clk::now()));
                continue;
            }
            // commit: the txn's writes logged behind everything before it
            const uint64_t lsn = hsc_window_end(ctx) + 1;
            w.assign(x.writes, x.writes + x.nwrites);
            for (hsc_write &y : w) y.commit_lsn = lsn;
            const int rc = hsc_window_append(ctx, w.data(), w.size());
            commit_seq[t] = ncommit++;
            L.hold.push_back(us(held, clk::now()));
            pthread_rwlock_unlock(&commit_lock);
            L.commit.push_back(us(c0, clk::now()));
            L.commits++;
            if (rc) {
                rc_out[t] = 1;
                int z = HSC_OK;
                err.compare_exchange_strong(z, rc);
            }
        }
    };
    const auto w0 = clk::now();
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(body, t);
    body(0);
    for (auto &x : th) x.join();
    pthread_rwlock_destroy(&commit_lock);
    res->seconds = std::chrono::duration<double>(clk::now() - w0).count();
    Lat all;
    for (Lat &L : lat) {
        all.regop.insert(all.regop.end(), L.regop.begin(), L.regop.end());
        all.full.insert(all.full.end(), L.full.begin(), L.full.end());
        all.hold.insert(all.hold.end(), L.hold.begin(), L.hold.end());
        all.commit.insert(all.commit.end(), L.commit.begin(), L.commit.end());
        all.commits += L.commits, all.aborts += L.aborts;
    }
    res->commits = all.commits;
    res->aborts = all.aborts;
    res->regop_probes = all.regop.size();
    res->full_checks = all.full.size();
    res->regop_p50_us = quant(all.regop, 0.5);
    res->regop_p99_us = quant(all.regop, 0.99);
    res->regop_p999_us = quant(all.regop, 0.999);
    res->regop_max_us = all.regop.empty() ? 0 : *std::max_element(all.regop.begin(), all.regop.end());
    res->full_p50_us = quant(all.full, 0.5);
    res->full_p99_us = quant(all.full, 0.99);
    res->hold_p50_us = quant(all.hold, 0.5);
    res->hold_p99_us = quant(all.hold, 0.99);
    res->commit_p50_us = quant(all.commit, 0.5);
    res->commit_p99_us = quant(all.commit, 0.99);
    return err.load();
}

}  // extern "C"
