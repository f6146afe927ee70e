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

#include <algorithm>
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

}  // extern "C"
