/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement of comdb2's index-key
 * reconstruction from the physical log, the parity checker for the product's
 * walk in comdb2_amd/csrc/hsc_logdec.cpp.  Nothing in comdb2_amd/ links it.
 *
 * Reference (read as text; none of it is compiled here):
 *   get_next_addrem_buffer   bdb/rowlocks.c:209-426
 *   bdb_reconstruct_add      bdb/rowlocks.c:428-456
 *   bdb_reconstruct_delete   bdb/rowlocks.c:535-617
 *   call sites               bdb/serializable.c:120-133 (undo_add_ix),
 *                            :170-184 (undo_del_ix), :242-258 (undo_del_ix_lk)
 *   record layouts           berkdb/db/db.src:47-57 (addrem 41), :73-83 (big 43),
 *                            :131 (debug 47), :177-184 (pg_free 50),
 *                            :206-214 (pg_freedata 52); encoding
 *                            berkdb/dist/gen_rec_endian.awk:895-958 (readers:
 *                            u32 fields and LSNs big-endian, DBT = u32 BE size
 *                            + bytes, no bounds checks)
 *   page items               berkdb/dbinc/db_page.h:606-679 (BKEYDATA
 *                            {u16 len, u8 type, data}, BOVERFLOW {u16, u8 type,
 *                            u8, u32 pgno, u32 tlen}, native little-endian;
 *                            B_TYPE masks B_DELETE|B_PFX|B_RLE)
 *
 * The log is an in-memory array of records sorted by LSN; the "log cursor"
 * DB_SET is a binary search (DB_NOTFOUND when absent).
 *
 * Where the reference's result depends on memory it does not own, this
 * restatement reports it instead of guessing:
 *  - the key buffer is malloc'd uninitialised (bdb/serializable.c:125,175,248)
 *    and the reconstruct rc is ignored, so a key byte no walk wrote is
 *    garbage: `defined` tells whether every byte [0, keylen) was written;
 *  - reads past the record (the generated readers and the BKEYDATA /
 *    BOVERFLOW casts never check sizes), an abort() (bdb/rowlocks.c:352), a
 *    copy past the buffer (the __db_big memcpy, :391-393) or a chain that does
 *    not go strictly back in LSN (the reference would loop) return RO_BAD.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DB___db_addrem 41
#define DB___db_big 43
#define DB___db_debug 47
#define DB___db_pg_free 50
#define DB___db_pg_freedata 52
#define DB_ADD_DUP 1
#define B_KEYDATA 1
#define B_OVERFLOW 3
#define B_DELETE 0x80
#define B_PFX 0x40
#define B_RLE 0x20
#define BDBERR_NO_LOG 1000 /* any value distinct from 0 / -1 / 1 */
#define RO_BAD (-2)

typedef struct ro_log {
    size_t nrec;
    const uint64_t *lsn; /* file << 32 | offset, ascending */
    const uint64_t *off;
    const uint32_t *len;
    const uint8_t *buf;
} ro_log;

typedef struct {
    const uint8_t *data; /* record bytes of the cursor's current record */
    uint32_t size;
} ro_dbt;

/* DB_LOGC->get(DB_SET) */
static int log_get(const ro_log *lg, uint64_t lsn, ro_dbt *out)
{
    size_t lo = 0, hi = lg->nrec;
    while (lo < hi) {
        size_t m = (lo + hi) / 2;
        if (lg->lsn[m] < lsn)
            lo = m + 1;
        else
            hi = m;
    }
    if (lo == lg->nrec || lg->lsn[lo] != lsn) return -1; /* DB_NOTFOUND */
    out->data = lg->buf + lg->off[lo];
    out->size = lg->len[lo];
    return 0;
}

static uint32_t be32(const uint8_t *p)
{
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

/* A bounded reader over one record (the generated readers read blindly;
 * running past the record is reported). */
typedef struct {
    const uint8_t *p, *end;
    int bad;
} rd;
static uint32_t rd32(rd *r)
{
    if (r->end - r->p < 4) {
        r->bad = 1;
        return 0;
    }
    uint32_t v = be32(r->p);
    r->p += 4;
    return v;
}
static uint64_t rdlsn(rd *r)
{
    uint64_t f = rd32(r);
    return f << 32 | rd32(r);
}
static void rddbt(rd *r, uint32_t *size, const uint8_t **data)
{
    *size = rd32(r);
    *data = r->p;
    if (r->bad || (size_t)(r->end - r->p) < *size) {
        r->bad = 1;
        return;
    }
    r->p += *size;
}

/* __db_addrem_args / __db_big_args (the parts the walk reads). */
typedef struct {
    uint32_t type;
    uint64_t prev_lsn;
    uint32_t opcode, fileid, pgno, indx, nbytes;
    uint32_t hdr_size, dbt_size;
    const uint8_t *hdr_data, *dbt_data;
    uint64_t pagelsn;
} addrem_args;
typedef struct {
    uint32_t type;
    uint64_t prev_lsn;
    uint32_t opcode, fileid, pgno, prev_pgno, next_pgno;
    uint32_t dbt_size;
    const uint8_t *dbt_data;
    uint64_t pagelsn, prevlsn, nextlsn;
} big_args;

static int addrem_read(const ro_dbt *rec, addrem_args *a)
{
    rd r = {rec->data, rec->data + rec->size, 0};
    a->type = rd32(&r);
    (void)rd32(&r); /* txnid */
    a->prev_lsn = rdlsn(&r);
    a->opcode = rd32(&r);
    a->fileid = rd32(&r);
    a->pgno = rd32(&r);
    a->indx = rd32(&r);
    a->nbytes = rd32(&r);
    rddbt(&r, &a->hdr_size, &a->hdr_data);
    rddbt(&r, &a->dbt_size, &a->dbt_data);
    a->pagelsn = rdlsn(&r);
    return r.bad ? -1 : 0;
}

static int big_read(const ro_dbt *rec, big_args *a)
{
    rd r = {rec->data, rec->data + rec->size, 0};
    a->type = rd32(&r);
    (void)rd32(&r);
    a->prev_lsn = rdlsn(&r);
    a->opcode = rd32(&r);
    a->fileid = rd32(&r);
    a->pgno = rd32(&r);
    a->prev_pgno = rd32(&r);
    a->next_pgno = rd32(&r);
    rddbt(&r, &a->dbt_size, &a->dbt_data);
    a->pagelsn = rdlsn(&r);
    a->prevlsn = rdlsn(&r);
    a->nextlsn = rdlsn(&r);
    return r.bad ? -1 : 0;
}

/* A caller buffer that remembers which bytes were written (the reference's
 * buffers are uninitialised). */
typedef struct {
    uint8_t *b, *w;
    int len;
} wbuf;
static int wput(wbuf *buf, long at, const uint8_t *src, size_t n)
{
    if (at < 0 || (size_t)at + n > (size_t)buf->len) return -1;
    memcpy(buf->b + at, src, n);
    memset(buf->w + at, 1, n);
    return 0;
}

/* Byte k of the item the record's hdr.data points at (kd / ov casts). */
static int item_byte(const ro_dbt *rec, const uint8_t *item, size_t k, uint8_t *out)
{
    if (item + k >= rec->data + rec->size) return -1;
    *out = item[k];
    return 0;
}

#define LSN_FILE(l) ((uint32_t)((l) >> 32))

/* get_next_addrem_buffer (bdb/rowlocks.c:209-426).  buf NULL = the caller
 * passed NULL.  Returns 0, BDBERR_NO_LOG or RO_BAD. */
static int get_next_addrem_buffer(const ro_log *lg, uint64_t *lsn, wbuf *buf, int len,
                                  int *have_record, uint64_t *nextlsn)
{
    ro_dbt logent;
    uint32_t rectype = 0;
    uint64_t prevlsn = 0;
    int last_was_pgfree = 0;
    long off = 0;
    int stopped = 0;
    while (LSN_FILE(*lsn) != 0) {
        const uint64_t cur = *lsn; /* lsn and nextlsn may alias (reconstruct_add) */
        if (log_get(lg, cur, &logent)) return BDBERR_NO_LOG;
        if (logent.size < 16) return RO_BAD; /* :262-267 (< 4) / LOGCOPY_TOLSN past the record */
        rectype = be32(logent.data);
        prevlsn = (uint64_t)be32(logent.data + 8) << 32 | be32(logent.data + 12);
        *nextlsn = prevlsn;
        if (prevlsn >= cur && LSN_FILE(prevlsn) != 0) return RO_BAD; /* would not terminate */

        if (rectype == DB___db_pg_free || rectype == DB___db_pg_freedata)
            last_was_pgfree = 1;
        else if (rectype != DB___db_addrem && rectype != DB___db_debug)
            last_was_pgfree = 0;

        if (rectype == DB___db_addrem) {
            addrem_args a;
            if (addrem_read(&logent, &a)) return RO_BAD;
            if (!last_was_pgfree) {
                const uint8_t *kd = a.hdr_size > 0 ? a.hdr_data : NULL;
                uint8_t t = 0;
                if (kd && item_byte(&logent, kd, 2, &t)) return RO_BAD;
                if (a.opcode == DB_ADD_DUP && (kd == NULL || (t & ~(B_DELETE | B_PFX | B_RLE)) == 0)) {
                    if (buf && a.dbt_size > (uint32_t)len) {
                        *have_record = 0;
                    } else {
                        *have_record = 1;
                        if (buf && wput(buf, 0, a.dbt_data, a.dbt_size)) return RO_BAD;
                    }
                    stopped = 1;
                    break;
                } else {
                    kd = a.hdr_data; /* hdr.data: never NULL from the reader */
                    if (item_byte(&logent, kd, 2, &t)) return RO_BAD;
                    const int bt = t & ~(B_DELETE | B_PFX | B_RLE);
                    if (bt == B_OVERFLOW) {
                        uint8_t b[4];
                        for (int k = 0; k < 4; ++k)
                            if (item_byte(&logent, kd, 8 + k, &b[k])) return RO_BAD;
                        const uint32_t tlen = (uint32_t)b[0] | (uint32_t)b[1] << 8 |
                                              (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
                        if (tlen > 0x7FFFFFFFu) return RO_BAD;
                        off = (long)tlen;
                    } else if (bt == B_KEYDATA) {
                        uint8_t b0, b1;
                        if (item_byte(&logent, kd, 0, &b0) || item_byte(&logent, kd, 1, &b1))
                            return RO_BAD;
                        const uint32_t klen = (uint32_t)b0 | (uint32_t)b1 << 8;
                        if (buf && (int)klen > len) return RO_BAD; /* abort(), :352 */
                        if (buf && klen && item_byte(&logent, kd, 3 + klen - 1, &t)) return RO_BAD;
                        *have_record = 1;
                        if (buf && wput(buf, 0, kd + 3, klen)) return RO_BAD;
                        stopped = 1;
                        break;
                    } else {
                        *have_record = 0; /* "Unexpected type" */
                    }
                }
            }
        } else if (rectype == DB___db_big) {
            big_args b;
            if (big_read(&logent, &b)) return RO_BAD;
            off -= (long)b.dbt_size;
            if (off < 0) {
                *have_record = 0; /* "huh?" */
            } else {
                if (buf && wput(buf, off, b.dbt_data, b.dbt_size)) return RO_BAD;
                if (off == 0) {
                    *have_record = 1;
                    stopped = 1;
                    break;
                }
            }
        }
        *lsn = prevlsn;
    }
    if (stopped) *lsn = prevlsn; /* :419-420 */
    return 0;
}

/* bdb_reconstruct_add (bdb/rowlocks.c:428-456) as serial_check_this_txn calls
 * it: data = NULL. */
static int reconstruct_add(const ro_log *lg, uint64_t startlsn, wbuf *key, int keylen,
                           int datalen)
{
    int have_record = 0;
    uint64_t nextlsn = (uint64_t)1 << 32; /* {1, 0} */
    uint64_t lsn = startlsn;
    int rc = get_next_addrem_buffer(lg, &lsn, NULL, datalen, &have_record, &nextlsn);
    if (rc) return rc;
    key->len = keylen;
    rc = get_next_addrem_buffer(lg, &nextlsn, key, keylen, &have_record, &nextlsn);
    return rc;
}

/* bdb_reconstruct_delete (bdb/rowlocks.c:535-617) with page, index and data
 * NULL: the key is the buffer of the last (first in log order) of the two
 * records found. */
static int reconstruct_delete(const ro_log *lg, uint64_t startlsn, wbuf *key, int keylen,
                              int datalen)
{
    if (LSN_FILE(startlsn) == 0) return RO_BAD; /* nextlsn would stay uninitialised */
    const int alloclen = keylen > datalen ? keylen : datalen;
    wbuf bufs[2];
    int haveit[2] = {0, 0};
    uint64_t lsn = startlsn, nextlsn = 0;
    int i = 0, rc = 0;
    for (int k = 0; k < 2; ++k) {
        bufs[k].len = alloclen > 0 ? alloclen : 0;
        bufs[k].b = calloc((size_t)bufs[k].len + 1, 1);
        bufs[k].w = calloc((size_t)bufs[k].len + 1, 1);
    }
    do {
        i++;
        rc = get_next_addrem_buffer(lg, &lsn, alloclen > 0 ? &bufs[i % 2] : NULL, alloclen,
                                    &haveit[i % 2], &nextlsn);
        if (rc) break;
    } while (LSN_FILE(nextlsn) != 0 && (!haveit[0] || !haveit[1]));
    if (!rc) {
        if (haveit[0] && haveit[1]) {
            for (int k = 0; k < keylen; ++k) {
                key->b[k] = bufs[i % 2].b[k];
                key->w[k] = bufs[i % 2].w[k];
            }
        } else {
            rc = 1;
        }
    }
    free(bufs[0].b), free(bufs[0].w), free(bufs[1].b), free(bufs[1].w);
    return rc;
}

/* One keyless index record's key: kind 0 = undo_add_ix (reconstruct_add),
 * 1 = undo_del_ix / undo_del_ix_lk (reconstruct_delete); undolsn = the
 * record's header prev_lsn (bdb/serializable.c:126,176,249).  key_out gets
 * keylen bytes; *defined = every byte was written by the walk.  Returns the
 * reconstruct rc (ignored by the reference: 0, 1, BDBERR_NO_LOG) or RO_BAD. */
int ro_reconstruct(const ro_log *lg, int kind, uint64_t undolsn, int keylen, int datalen,
                   uint8_t *key_out, int *defined)
{
    if (keylen < 0) return RO_BAD;
    wbuf key;
    key.len = keylen;
    key.b = key_out;
    key.w = calloc((size_t)keylen + 1, 1);
    memset(key_out, 0, (size_t)keylen);
    int rc = kind == 0 ? reconstruct_add(lg, undolsn, &key, keylen, datalen)
                       : reconstruct_delete(lg, undolsn, &key, keylen, datalen);
    int all = 1;
    for (int k = 0; k < keylen; ++k) all &= key.w[k] != 0;
    *defined = rc != RO_BAD && all;
    free(key.w);
    return rc;
}

int ro_no_log_rc(void) { return BDBERR_NO_LOG; }
