/*
 * serial_oracle.c -- TEST INFRASTRUCTURE ONLY (see serial_oracle.h).
 *
 * A literal CPU restatement of comdb2's SERIALIZABLE read-set check over an
 * in-memory, already-decoded log (or_log).  Per check it re-walks the log
 * window record by record, walks every committed write txn's logical chain
 * backwards, and scans the read ranges of the written index linearly, exiting
 * at the first conflict -- the reference's cost model, minus log I/O.
 */
#define _GNU_SOURCE
#include "serial_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum {
    REC_TXN_REGOP = 10,
    REC_TXN_REGOP_ROWLOCKS = 15,
    REC_TXN_REGOP_GEN = 16,
    REC_UNDO_ADD_DTA = 10003,
    REC_UNDO_ADD_IX = 10004,
    REC_LTRAN_COMMIT = 10005,
    REC_LTRAN_START = 10006,
    REC_LTRAN_COMPREC = 10007,
    REC_UNDO_DEL_DTA = 10008,
    REC_UNDO_DEL_IX = 10009,
    REC_UNDO_UPD_DTA = 10010,
    REC_UNDO_UPD_IX = 10011,
    REC_UNDO_ADD_DTA_LK = 10013,
    REC_UNDO_ADD_IX_LK = 10014,
    REC_UNDO_DEL_DTA_LK = 10015,
    REC_UNDO_DEL_IX_LK = 10016,
    REC_UNDO_UPD_DTA_LK = 10017,
    REC_UNDO_UPD_IX_LK = 10018
};

/* berkdb DB_NOTFOUND; any other failing cursor op is restated as OR_EIO. */
#define OR_NOTFOUND (-30988)
#define OR_EIO 5
#define OR_ABORT (-999) /* reference calls abort() (bdb/serializable.c:283) */

/* ---- the span "hash" (db/comdb2.h:1126-1140, db/sqlglue.c:312-351) ------ */
typedef struct or_ih {
    int idxnum;
    int begin, end;
} or_ih;

typedef struct or_th {
    const char *tbname;
    int islocked;
    int begin, end;
    int nidx, capidx;
    or_ih *idx;
} or_th;

typedef struct or_hash {
    int ntab, captab;
    or_th *tab;
} or_hash;

static or_th *find_table(or_hash *h, const char *name)
{
    for (int i = 0; i < h->ntab; i++)
        if (strcmp(h->tab[i].tbname, name) == 0)
            return &h->tab[i];
    return NULL;
}

static or_ih *find_idx(or_th *th, int idxnum)
{
    for (int i = 0; i < th->nidx; i++)
        if (th->idx[i].idxnum == idxnum)
            return &th->idx[i];
    return NULL;
}

static void add_idx(or_th *th, int idxnum, int i)
{
    if (th->nidx == th->capidx) {
        th->capidx = th->capidx ? 2 * th->capidx : 4;
        th->idx = realloc(th->idx, sizeof(or_ih) * th->capidx);
    }
    th->idx[th->nidx].idxnum = idxnum;
    th->idx[th->nidx].begin = i;
    th->idx[th->nidx].end = i;
    th->nidx++;
}

/* currangearr_build_hash: per table the islocked of its FIRST range in array
 * order and the [first,last] array span; per (table, idxnum) the span. */
void or_prepare(or_rangearr *arr)
{
    if (arr->size == 0)
        return;
    or_hash *h = calloc(1, sizeof(or_hash));
    for (int i = 0; i < arr->size; i++) {
        or_range *r = arr->ranges[i];
        or_th *th = find_table(h, r->tbname);
        if (th == NULL) {
            if (h->ntab == h->captab) {
                h->captab = h->captab ? 2 * h->captab : 4;
                h->tab = realloc(h->tab, sizeof(or_th) * h->captab);
            }
            th = &h->tab[h->ntab++];
            memset(th, 0, sizeof(*th));
            th->tbname = r->tbname;
            th->islocked = r->islocked;
            th->begin = th->end = i;
            add_idx(th, r->idxnum, i);
        } else {
            th->end = i;
            or_ih *ih = find_idx(th, r->idxnum);
            if (ih == NULL)
                add_idx(th, r->idxnum, i);
            else
                ih->end = i;
        }
    }
    arr->hash = h;
}

void or_unprepare(or_rangearr *arr)
{
    or_hash *h = arr->hash;
    if (!h)
        return;
    for (int i = 0; i < h->ntab; i++)
        free(h->tab[i].idx);
    free(h->tab);
    free(h);
    arr->hash = NULL;
}

static int mc(const void *a, const void *b, int n)
{
    return n > 0 ? memcmp(a, b, (size_t)n) : 0;
}

/* serial_check_callback, db/glue.c:2926-2963. */
static int callback(const char *tbname, int idxnum, const void *key,
                    int keylen, or_rangearr *arr)
{
    if (arr->size == 0)
        return 0;
    or_th *th = find_table((or_hash *)arr->hash, tbname);
    if (th == NULL)
        return 0;
    if (th->islocked)
        return 1;
    if (!key)
        return 0;
    or_ih *ih = find_idx(th, idxnum);
    if (ih == NULL)
        return 0;
    for (int i = ih->begin; i <= ih->end; i++) {
        or_range *r = arr->ranges[i];
        int ll = r->lkeylen < keylen ? r->lkeylen : keylen;
        int rl = r->rkeylen < keylen ? r->rkeylen : keylen;
        if ((r->lflag || mc(r->lkey, key, ll) <= 0) &&
            (r->rflag || mc(key, r->rkey, rl) <= 0))
            return 1;
    }
    return 0;
}

/* DB_LOGC->get(DB_SET): exact LSN lookup.  Past the end -> DB_NOTFOUND,
 * inside the log but not a record boundary -> an I/O error. */
static long find_rec(const or_log *log, uint64_t lsn, int *rc)
{
    size_t lo = 0, hi = log->nrec;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (log->lsn[mid] < lsn)
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo < log->nrec && log->lsn[lo] == lsn) {
        *rc = 0;
        return (long)lo;
    }
    *rc = (lsn >= log->end_lsn) ? OR_NOTFOUND : OR_EIO;
    return -1;
}

static const char *tbl(const or_log *log, size_t i)
{
    return log->tbnames[log->table[i]];
}

static const void *keyp(const or_log *log, size_t i)
{
    return log->keys + log->key_off[i];
}

/* serial_check_this_txn, bdb/serializable.c:60-332: walk one committed txn's
 * logical chain back to ltran_start, one callback per write record. */
static int check_txn(const or_log *log, uint64_t lsn, or_rangearr *arr)
{
    int rc;
    long i = find_rec(log, lsn, &rc);
    if (rc)
        return 1;
    uint32_t rectype = log->rectype[i];
    while (rc == 0 && rectype != REC_LTRAN_START) {
        switch (rectype) {
        case REC_UNDO_ADD_DTA:
        case REC_UNDO_DEL_DTA:
        case REC_UNDO_UPD_DTA:
        case REC_UNDO_ADD_DTA_LK:
        case REC_UNDO_DEL_DTA_LK:
        case REC_UNDO_UPD_DTA_LK:
            rc = callback(tbl(log, i), -2, NULL, 0, arr);
            lsn = log->prev[i];
            break;
        case REC_UNDO_ADD_IX:      /* key via bdb_reconstruct_add (rc ignored) */
        case REC_UNDO_DEL_IX:      /* key via bdb_reconstruct_delete          */
        case REC_UNDO_DEL_IX_LK:   /* key via bdb_reconstruct_delete          */
        case REC_UNDO_UPD_IX:      /* key carried in the record               */
        case REC_UNDO_ADD_IX_LK:
        case REC_UNDO_UPD_IX_LK:
            rc = callback(tbl(log, i), (int)log->ix[i], keyp(log, i),
                          log->keylen[i], arr);
            lsn = log->prev[i];
            break;
        case REC_LTRAN_COMMIT:
        case REC_LTRAN_COMPREC:
            lsn = log->prev[i];
            break;
        default:
            return OR_ABORT;
        }
        if (rc)
            return rc;
        if ((uint32_t)(lsn >> 32) == 0)
            break;
        i = find_rec(log, lsn, &rc);
        if (rc)
            return 1;
        rectype = log->rectype[i];
    }
    return 0;
}

static int is_regop(uint32_t t)
{
    return t == REC_TXN_REGOP || t == REC_TXN_REGOP_GEN ||
           t == REC_TXN_REGOP_ROWLOCKS;
}

/* osql_serial_check, bdb/serializable.c:341-569. */
static int osql_check(const or_log *log, or_rangearr *ranges,
                      unsigned int *file, unsigned int *offset, int regop_only)
{
    int rc;
    uint32_t sfile = *file, soff = *offset;
    uint64_t cur = log->end_lsn;
    uint32_t cfile = (uint32_t)(cur >> 32), coff = (uint32_t)cur;
    if (!regop_only) {
        *file = cfile;
        *offset = coff;
    }
    rc = 0;
    while (sfile < cfile || soff <= coff) {
        uint64_t slsn = ((uint64_t)sfile << 32) | soff;
        long i = find_rec(log, slsn, &rc);
        if (rc == OR_NOTFOUND) {
            rc = 0;
            break;
        } else if (rc) {
            goto done;
        }
        long commit = -1;
        for (;;) {
            i++; /* DB_NEXT */
            if ((size_t)i >= log->nrec) {
                rc = OR_NOTFOUND;
                break;
            }
            sfile = (uint32_t)(log->lsn[i] >> 32);
            soff = (uint32_t)log->lsn[i];
            if (is_regop(log->rectype[i])) {
                long p = find_rec(log, log->prev[i], &rc);
                if (rc)
                    goto done;
                if (log->rectype[p] == REC_LTRAN_COMMIT) {
                    commit = p;
                    break;
                }
            }
        }
        if (rc == OR_NOTFOUND) {
            rc = 0;
            goto done;
        } else if (rc) {
            goto done;
        }
        /* found a committed transaction */
        if ((uint32_t)(log->prev[commit] >> 32) == 0) /* not a write txn */
            continue;
        if (log->isabort[commit])
            continue;
        rc = regop_only ? 1 : check_txn(log, log->prev[commit], ranges);
        if (rc)
            goto done;
    }
done:
    return rc;
}

int or_serial_check(const or_log *log, or_rangearr *arr, unsigned int *file,
                    unsigned int *offset, int regop_only)
{
    if (!arr)
        return 0;
    return osql_check(log, arr, file, offset, regop_only);
}

/* ---- batch driver (CPU baseline: one read set per task, all cores) ------ */
typedef struct job {
    const or_log *log;
    or_rangearr **arrs;
    int n, regop_only;
    int *rc_out;
    int next;
    pthread_mutex_t mu;
} job;

static void *worker(void *p)
{
    job *j = p;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int i = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->n)
            break;
        or_rangearr *a = j->arrs[i];
        j->rc_out[i] = a ? or_serial_check(j->log, a, &a->file, &a->offset,
                                           j->regop_only)
                         : 0;
    }
    return NULL;
}

double or_serial_check_many(const or_log *log, or_rangearr **arrs, int n,
                            int regop_only, int nthreads, int *rc_out)
{
    struct timespec t0, t1;
    job j = {log, arrs, n, regop_only, rc_out, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1)
        nthreads = 1;
    pthread_t *th = malloc(sizeof(pthread_t) * (size_t)nthreads);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- flat read sets -> heap arrays -------------------------------------- */
static void *dupbytes(const uint8_t *p, int n)
{
    if (n <= 0)
        return NULL;
    void *q = malloc((size_t)n);
    memcpy(q, p, (size_t)n);
    return q;
}

or_rangearr **or_build_arrs(int ntxn, const int64_t *txn_off,
                            const uint64_t *snap, const int32_t *table,
                            const int32_t *idxnum, const int32_t *lflag,
                            const int32_t *rflag, const int32_t *islocked,
                            const int32_t *lkeylen, const int32_t *rkeylen,
                            const uint64_t *lkey_off, const uint64_t *rkey_off,
                            const uint8_t *keys, const char *const *tbnames)
{
    or_rangearr **arrs = calloc((size_t)ntxn, sizeof(or_rangearr *));
    for (int t = 0; t < ntxn; t++) {
        or_rangearr *a = calloc(1, sizeof(or_rangearr));
        int n = (int)(txn_off[t + 1] - txn_off[t]);
        a->size = n;
        a->cap = n > 2 ? n : 2;
        a->file = (unsigned int)(snap[t] >> 32);
        a->offset = (unsigned int)snap[t];
        a->ranges = calloc((size_t)a->cap, sizeof(or_range *));
        for (int k = 0; k < n; k++) {
            int64_t r = txn_off[t] + k;
            or_range *c = calloc(1, sizeof(or_range));
            c->tbname = strdup(tbnames[table[r]]);
            c->idxnum = idxnum[r];
            c->lflag = lflag[r];
            c->rflag = rflag[r];
            c->islocked = islocked[r];
            c->lkeylen = lkeylen[r];
            c->rkeylen = rkeylen[r];
            c->lkey = dupbytes(keys + lkey_off[r], lkeylen[r]);
            c->rkey = dupbytes(keys + rkey_off[r], rkeylen[r]);
            a->ranges[k] = c;
        }
        or_prepare(a);
        arrs[t] = a;
    }
    return arrs;
}

void or_free_arrs(or_rangearr **arrs, int ntxn)
{
    for (int t = 0; t < ntxn; t++) {
        or_rangearr *a = arrs[t];
        if (!a)
            continue;
        or_unprepare(a);
        for (int k = 0; k < a->size; k++) {
            free(a->ranges[k]->tbname);
            free(a->ranges[k]->lkey);
            free(a->ranges[k]->rkey);
            free(a->ranges[k]);
        }
        free(a->ranges);
        free(a);
    }
    free(arrs);
}
