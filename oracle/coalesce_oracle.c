/*
 * coalesce_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker for
 * hsc_coalesce_readsets; never linked into comdb2_amd/).
 *
 * CPU restatement of the replicant's read-set coalesce,
 * reference db/sqlglue.c:
 *   currange_cmp               :206-242
 *   currangearr_sort           :243-246   qsort -> glibc msort (top-down merge
 *                                          sort, n1 = n / 2, "cmp <= 0 takes
 *                                          the left run"; glibc <= 2.36)
 *   currangearr_merge_neighbor :247-304
 *   currangearr_coalesce       :305-311   sort, merge, sort, merge
 * over the flat read-set layout of include/hip_serial.h (hsc_readsets):
 *   - tbname = tbnames[table] compared with strcmp (table must be valid: a
 *     NULL tbname would crash merge_neighbor's strcmp in the reference);
 *   - a key pointer is NULL iff its offset is HSC_KEY_NULL (~0); any other
 *     offset is a present key, also when empty (include/hip_serial.h);
 *   - the right-key pointer swap of :265-270 moves only the key (offset),
 *     never rkeylen: p keeps its own length over q's key bytes (reading past
 *     the end of the keys buffer yields 0 bytes here; heap bytes there).
 * Parity: unpinned by the reference (it has no test of currangearr_coalesce);
 * tests/ cross-check this file against an independent Python model
 * (tests/coalesce_model.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CO_KEY_NULL UINT64_MAX /* HSC_KEY_NULL of include/hip_serial.h */

struct co_rng {
    int32_t table, idxnum, lflag, rflag, islocked, lkeylen, rkeylen;
    uint64_t lkey_off, rkey_off;
};

struct co_ctx {
    const uint8_t *keys;
    uint64_t nkeys;
    const char *const *tbnames;
    int ntb;
};

static int key_byte(const struct co_ctx *c, uint64_t off, int i)
{
    return off + (uint64_t)i < c->nkeys ? c->keys[off + (uint64_t)i] : 0;
}

/* memcmp(a, b, n) over the keys buffer */
static int keycmp(const struct co_ctx *c, uint64_t a, uint64_t b, int n)
{
    for (int i = 0; i < n; ++i) {
        int x = key_byte(c, a, i), y = key_byte(c, b, i);
        if (x != y) return x - y;
    }
    return 0;
}

/* currange_cmp (db/sqlglue.c:206-242) */
static int co_cmp(const struct co_ctx *c, const struct co_rng *l, const struct co_rng *r)
{
    int rc;
    rc = strcmp(c->tbnames[l->table], c->tbnames[r->table]);
    if (rc) return rc;
    if (l->islocked || r->islocked) return r->islocked - l->islocked;
    if (l->idxnum != r->idxnum) return l->idxnum - r->idxnum;
    if (l->lflag) return -1;
    if (r->lflag) return 1;
    if (l->lkey_off != CO_KEY_NULL && r->lkey_off != CO_KEY_NULL) { /* l->lkey && r->lkey */
        rc = keycmp(c, l->lkey_off, r->lkey_off, l->lkeylen < r->lkeylen ? l->lkeylen : r->lkeylen);
        if (rc) return rc;
        return l->lkeylen - r->lkeylen;
    }
    return 0;
}

/* glibc msort_with_tmp over an array of range indices */
static void co_msort(const struct co_ctx *c, const struct co_rng *a, uint32_t *b, uint32_t *tmp,
                     size_t n)
{
    if (n <= 1) return;
    size_t n1 = n / 2, n2 = n - n1;
    uint32_t *b1 = b, *b2 = b + n1;
    co_msort(c, a, b1, tmp, n1);
    co_msort(c, a, b2, tmp, n2);
    uint32_t *t = tmp;
    while (n1 > 0 && n2 > 0) {
        if (co_cmp(c, &a[*b1], &a[*b2]) <= 0) {
            *t++ = *b1++;
            --n1;
        } else {
            *t++ = *b2++;
            --n2;
        }
    }
    if (n1 > 0) memcpy(t, b1, n1 * sizeof *b1);
    memcpy(b, tmp, (n - n2) * sizeof *b);
}

/* currangearr_merge_neighbor (db/sqlglue.c:247-304) over ord[0 .. n): the
 * records a[ord[k]] are mutated like the CurRange's behind the pointers */
static size_t co_merge(const struct co_ctx *c, struct co_rng *a, uint32_t *ord, size_t n)
{
    size_t i = 1, j = 0;
    if (!n) return 0;
    while (i < n) {
        struct co_rng *p = &a[ord[j]], *q = &a[ord[i]];
        if (strcmp(c->tbnames[p->table], c->tbnames[q->table]) == 0) {
            if (p->idxnum == q->idxnum) {
                int m = q->lkeylen < p->rkeylen ? q->lkeylen : p->rkeylen;
                if (q->lflag || p->rflag || keycmp(c, q->lkey_off, p->rkey_off, m) <= 0) {
                    if (p->rflag || q->rflag) {
                        p->rflag = 1;
                        p->rkey_off = CO_KEY_NULL; /* free(p->rkey); p->rkey = NULL */
                        p->rkeylen = 0;
                    } else if (keycmp(c, p->rkey_off, q->rkey_off,
                                      p->rkeylen < q->rkeylen ? p->rkeylen : q->rkeylen) < 0) {
                        p->rkey_off = q->rkey_off;  /* pointer swap: rkeylen stays */
                    }
                    if (p->lflag && p->rflag) p->islocked = 1;
                    ++i;
                    continue;
                }
            } else if (p->islocked) {
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

/* Coalesces every read set.  Output rows (in coalesced order) go to out_*
 * (capacity = input ranges), out_off[ntxn + 1] delimits them.  Returns the
 * number of output ranges, or -1 if a range names no table. */
long co_coalesce(int ntxn, const int64_t *txn_off, const int32_t *table, const int32_t *idxnum,
                 const int32_t *lflag, const int32_t *rflag, const int32_t *islocked,
                 const int32_t *lkeylen, const int32_t *rkeylen, const uint64_t *lkey_off,
                 const uint64_t *rkey_off, const uint8_t *keys, uint64_t nkeys,
                 const char *const *tbnames, int ntb, int64_t *out_off, int32_t *o_table,
                 int32_t *o_idxnum, int32_t *o_lflag, int32_t *o_rflag, int32_t *o_islocked,
                 int32_t *o_lkeylen, int32_t *o_rkeylen, uint64_t *o_lkey_off,
                 uint64_t *o_rkey_off)
{
    struct co_ctx c = {keys, nkeys, tbnames, ntb};
    long total = 0;
    out_off[0] = 0;
    for (int t = 0; t < ntxn; ++t) {
        size_t b = (size_t)txn_off[t], n = (size_t)(txn_off[t + 1] - txn_off[t]);
        struct co_rng *a = malloc((n ? n : 1) * sizeof *a);
        uint32_t *ord = malloc((n ? n : 1) * sizeof *ord), *tmp = malloc((n ? n : 1) * sizeof *tmp);
        if (!a || !ord || !tmp) {
            free(a), free(ord), free(tmp);
            return -1;
        }
        for (size_t k = 0; k < n; ++k) {
            size_t r = b + k;
            if (table[r] < 0 || table[r] >= ntb) {
                free(a), free(ord), free(tmp);
                return -1;
            }
            a[k] = (struct co_rng){table[r], idxnum[r], lflag[r], rflag[r], islocked[r],
                                   lkeylen[r], rkeylen[r], lkey_off[r], rkey_off[r]};
            ord[k] = (uint32_t)k;
        }
        co_msort(&c, a, ord, tmp, n);
        size_t m = co_merge(&c, a, ord, n);
        co_msort(&c, a, ord, tmp, m);
        m = co_merge(&c, a, ord, m);
        for (size_t k = 0; k < m; ++k) {
            const struct co_rng *r = &a[ord[k]];
            size_t o = (size_t)total + k;
            o_table[o] = r->table, o_idxnum[o] = r->idxnum, o_lflag[o] = r->lflag;
            o_rflag[o] = r->rflag, o_islocked[o] = r->islocked, o_lkeylen[o] = r->lkeylen;
            o_rkeylen[o] = r->rkeylen, o_lkey_off[o] = r->lkey_off, o_rkey_off[o] = r->rkey_off;
        }
        total += (long)m;
        out_off[t + 1] = total;
        free(a), free(ord), free(tmp);
    }
    return total;
}
