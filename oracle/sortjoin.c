/*
 * sortjoin.c -- CPU BASELINE / TEST INFRASTRUCTURE ONLY.
 *
 * The build's own multi-threaded sort-join on the CPU (the
 * second CPU line "to separate algorithmic gain from hardware gain").  It
 * evaluates the same marshalled probes as the HIP path (comdb2_amd's
 * marshaller: lo/hi padded to L^ bytes as big-endian u64 words, snap, txn,
 * group; table-lock probes) against the same write window, with the
 * set-formula of SURVEY.md §8(a) A0 instead of the reference's per-txn log
 * rescan (oracle/serial_oracle.c):
 *
 *   verdict(t) = OR over probes q of t:
 *       max{ lsn(row) : row in group(q), lo(q) <= key(row) <= hi(q) } > snap(q)
 *     OR over lock probes: table_max(table) > snap
 *
 * Window build: LSD radix sort of (group, key words) rows, skipping byte
 * digits that are constant over the window; duplicates keep the max LSN;
 * 64-row block maxima plus a sparse table over the blocks.  Probe: two
 * binary searches per range inside its group, then the range maximum.
 * Parallel over probes with pthreads.  Only bench.py's cpu_baseline leg and
 * tests/ call this; comdb2_amd/ never does.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sortjoin.h"

#define BLK 64

struct sj_window {
    size_t n;
    int W;
    uint32_t ngroups;
    uint64_t *key;      /* [n][W] row-major, sorted by (gid, key) */
    uint64_t *lsn;      /* [n] */
    uint32_t *gstart;   /* [ngroups] */
    uint32_t *gend;
    size_t nblk;
    int levels;
    uint64_t *sparse;   /* [levels][nblk]: max over 2^l blocks */
};

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* byte d of a row's sort key: d = 0 is the least significant byte of the
 * last key word; the group id occupies the most significant 4 bytes */
static inline unsigned digit(const uint32_t *gid, const uint64_t *words, size_t n, int W,
                             size_t r, int d)
{
    const int wi = W - 1 - d / 8;
    if (wi >= 0) return (unsigned)(words[(size_t)wi * n + r] >> (8 * (d % 8))) & 0xFF;
    return (gid[r] >> (8 * (d - 8 * W))) & 0xFF;
}

sj_window *sj_build(size_t n, int W, uint32_t ngroups, const uint32_t *gid,
                    const uint64_t *words, const uint64_t *lsn, double *secs)
{
    const double t0 = now_s();
    sj_window *w = calloc(1, sizeof *w);
    uint32_t *perm = malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t *tmp = malloc(sizeof(uint32_t) * (n ? n : 1));
    uint8_t *dig = malloc(n ? n : 1);
    if (!w || !perm || !tmp || !dig) goto fail;
    for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
    /* LSD over bytes, least significant first; stable counting sort */
    for (int d = 0; d < 8 * W + 4; ++d) {
        size_t cnt[256] = {0};
        for (size_t i = 0; i < n; ++i) {
            dig[i] = (uint8_t)digit(gid, words, n, W, perm[i], d);
            cnt[dig[i]]++;
        }
        int constant = 0;
        for (int b = 0; b < 256; ++b) constant |= cnt[b] == n;
        if (constant) continue;
        size_t off = 0;
        for (int b = 0; b < 256; ++b) {
            size_t c = cnt[b];
            cnt[b] = off;
            off += c;
        }
        for (size_t i = 0; i < n; ++i) tmp[cnt[dig[i]]++] = perm[i];
        uint32_t *x = perm;
        perm = tmp;
        tmp = x;
    }
    /* dedupe equal (gid, key): keep the max lsn */
    w->W = W;
    w->ngroups = ngroups;
    w->key = malloc(sizeof(uint64_t) * (n ? n : 1) * W);
    w->lsn = malloc(sizeof(uint64_t) * (n ? n : 1));
    w->gstart = calloc(ngroups ? ngroups : 1, sizeof(uint32_t));
    w->gend = calloc(ngroups ? ngroups : 1, sizeof(uint32_t));
    uint32_t *rg = malloc(sizeof(uint32_t) * (n ? n : 1));
    if (!w->key || !w->lsn || !w->gstart || !w->gend || !rg) goto fail;
    size_t m = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t r = perm[i];
        int same = m > 0 && rg[m - 1] == gid[r];
        for (int j = 0; same && j < W; ++j) same = w->key[(m - 1) * W + j] == words[(size_t)j * n + r];
        if (same) {
            if (lsn[r] > w->lsn[m - 1]) w->lsn[m - 1] = lsn[r];
            continue;
        }
        rg[m] = gid[r];
        for (int j = 0; j < W; ++j) w->key[m * W + j] = words[(size_t)j * n + r];
        w->lsn[m] = lsn[r];
        ++m;
    }
    w->n = m;
    for (size_t i = 0; i < m; ++i) {
        if (rg[i] >= ngroups) continue;
        if (i == 0 || rg[i - 1] != rg[i]) w->gstart[rg[i]] = (uint32_t)i;
        w->gend[rg[i]] = (uint32_t)i + 1;
    }
    free(rg);
    /* block maxima + sparse table */
    w->nblk = (m + BLK - 1) / BLK;
    w->levels = 1;
    while (((size_t)1 << w->levels) <= w->nblk) w->levels++;
    w->sparse = malloc(sizeof(uint64_t) * (w->nblk ? w->nblk : 1) * w->levels);
    if (!w->sparse) goto fail;
    for (size_t b = 0; b < w->nblk; ++b) {
        uint64_t mx = 0;
        for (size_t i = b * BLK; i < m && i < (b + 1) * BLK; ++i) mx = w->lsn[i] > mx ? w->lsn[i] : mx;
        w->sparse[b] = mx;
    }
    for (int l = 1; l < w->levels; ++l) {
        const uint64_t *p = w->sparse + (size_t)(l - 1) * w->nblk;
        uint64_t *q = w->sparse + (size_t)l * w->nblk;
        const size_t h = (size_t)1 << (l - 1);
        for (size_t b = 0; b < w->nblk; ++b)
            q[b] = b + h < w->nblk && p[b + h] > p[b] ? p[b + h] : p[b];
    }
    free(perm);
    free(tmp);
    free(dig);
    if (secs) *secs = now_s() - t0;
    return w;
fail:
    free(perm);
    free(tmp);
    free(dig);
    sj_free(w);
    return NULL;
}

void sj_free(sj_window *w)
{
    if (!w) return;
    free(w->key);
    free(w->lsn);
    free(w->gstart);
    free(w->gend);
    free(w->sparse);
    free(w);
}

size_t sj_rows(const sj_window *w) { return w ? w->n : 0; }

/* sign(row key - probe key) with the probe key in SoA words */
static inline int cmp_row(const sj_window *w, size_t row, const uint64_t *pk, size_t ks)
{
    const uint64_t *rk = w->key + row * w->W;
    for (int j = 0; j < w->W; ++j) {
        const uint64_t b = pk[(size_t)j * ks];
        if (rk[j] != b) return rk[j] < b ? -1 : 1;
    }
    return 0;
}

static uint64_t range_max(const sj_window *w, size_t a, size_t b) /* [a, b) */
{
    uint64_t mx = 0;
    size_t ba = (a + BLK - 1) / BLK, bb = b / BLK;
    if (ba >= bb) {
        for (size_t i = a; i < b; ++i) mx = w->lsn[i] > mx ? w->lsn[i] : mx;
        return mx;
    }
    for (size_t i = a; i < ba * BLK; ++i) mx = w->lsn[i] > mx ? w->lsn[i] : mx;
    for (size_t i = bb * BLK; i < b; ++i) mx = w->lsn[i] > mx ? w->lsn[i] : mx;
    const size_t len = bb - ba;
    int l = 63 - __builtin_clzll(len);
    const uint64_t *lv = w->sparse + (size_t)l * w->nblk;
    const uint64_t x = lv[ba], y = lv[bb - ((size_t)1 << l)];
    mx = x > mx ? x : mx;
    return y > mx ? y : mx;
}

typedef struct {
    const sj_window *w;
    const sj_probes *p;
    uint8_t *verdict;
    size_t q0, q1;
} job;

static void *probe_range(void *arg)
{
    job *j = arg;
    const sj_window *w = j->w;
    const sj_probes *p = j->p;
    const size_t ks = p->n;
    for (size_t q = j->q0; q < j->q1; ++q) {
        const uint32_t t = p->txn[q];
        if (__atomic_load_n(&j->verdict[t], __ATOMIC_RELAXED)) continue; /* early exit */
        const uint32_t g = p->gid[q];
        if (g >= w->ngroups) continue;
        size_t lo = w->gstart[g], hi = w->gend[g];
        while (lo < hi) { /* first row >= lo(q) */
            size_t m = (lo + hi) / 2;
            if (cmp_row(w, m, p->lo + q, ks) < 0) lo = m + 1; else hi = m;
        }
        const size_t a = lo;
        hi = w->gend[g];
        while (lo < hi) { /* first row > hi(q) */
            size_t m = (lo + hi) / 2;
            if (cmp_row(w, m, p->hi + q, ks) <= 0) lo = m + 1; else hi = m;
        }
        if (a < lo && range_max(w, a, lo) > p->snap[q])
            __atomic_store_n(&j->verdict[t], 1, __ATOMIC_RELAXED);
    }
    return NULL;
}

double sj_probe(const sj_window *w, const sj_probes *p, int nthreads, uint8_t *verdict)
{
    const double t0 = now_s();
    for (size_t i = 0; i < p->n_lock; ++i) {
        const uint32_t t = p->lock_table[i];
        if (t < p->ntables && p->table_max[t] > p->lock_snap[i]) verdict[p->lock_txn[i]] = 1;
    }
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    job jobs[256];
    if (nthreads > 256) nthreads = 256;
    const size_t per = (p->n + nthreads - 1) / nthreads;
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].w = w;
        jobs[i].p = p;
        jobs[i].verdict = verdict;
        jobs[i].q0 = i * per < p->n ? i * per : p->n;
        jobs[i].q1 = (i + 1) * per < p->n ? (i + 1) * per : p->n;
        if (nthreads == 1)
            probe_range(&jobs[i]);
        else
            pthread_create(&th[i], NULL, probe_range, &jobs[i]);
    }
    if (nthreads > 1)
        for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    return now_s() - t0;
}
