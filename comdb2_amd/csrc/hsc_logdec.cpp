// Raw log-record decoder: the byte layouts of bdb/llog.src:26-225 and the
// txn regop records (berkdb/dbinc_auto/txn_auto.h:6-86) as the
// gen_rec_endian.awk encoders write them on a little-endian host
// (berkdb/dist/gen_rec_endian.awk:550-630, berkdb/dbinc/db_swap.amd64.h):
//   header   type u32 BE | txnid u32 BE | prev_lsn (file u32 BE, offset u32 BE)
//   ARG int/short     u32 BE (shorts widened)
//   ARG genid_t       8 bytes memcpy (native little-endian)
//   ARG u_int64_t     u64 BE (LOGCOPY_64)
//   POINTER DB_LSN    file u32 BE, offset u32 BE
//   DBT               size u32 BE + size bytes
// Output is the decoded struct-of-arrays hsc_llog that hsc_window_ingest_log
// consumes: for logical records prev = prevllsn, for regops prev = the header
// prev_lsn (-> ltran_commit, bdb/serializable.c:453-456), for every other
// record the header prev_lsn.
//
// Keys of undo_add_ix / undo_del_ix / undo_del_ix_lk are not in the record:
// the reference rebuilds them from the physical log at undolsn = the header
// prev_lsn (bdb/serializable.c:123-130,174-181,248-252) with
// bdb_reconstruct_add / bdb_reconstruct_delete (bdb/rowlocks.c:428-617),
// which walk the header prev_lsn chain over __db_addrem / __db_big records
// (get_next_addrem_buffer, :209-426; layouts berkdb/db/db.src:47-83, page
// items berkdb/dbinc/db_page.h:606-679).  recon_walk below restates that walk
// over a PhysStore of every record decoded since the last ingest; a caller
// side table (hsc_raw_log.recon_*) still takes precedence when it names the
// record's undolsn.
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/hip_serial.h"
#include "hsc_internal.h"

namespace hsc {
namespace {

struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    bool need(size_t n)
    {
        if ((size_t)(end - p) < n) ok = false;
        return ok;
    }
    uint32_t u32()  // LOGCOPY_32: big-endian on disk
    {
        if (!need(4)) return 0;
        uint32_t v = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
        p += 4;
        return v;
    }
    uint64_t lsn()  // LOGCOPY_TOLSN
    {
        uint64_t f = u32();
        return f << 32 | u32();
    }
    uint64_t genid()  // genid_t: memcpy, native order
    {
        if (!need(8)) return 0;
        uint64_t v;
        memcpy(&v, p, 8);
        p += 8;
        return v;
    }
    void dbt(const uint8_t **data, uint32_t *size)
    {
        const uint32_t n = u32();
        if (!need(n)) return;
        *data = p;
        *size = n;
        p += n;
    }
    void skip_dbt()
    {
        const uint8_t *d;
        uint32_t n;
        dbt(&d, &n);
    }
};

// Field programs of the logical records, in llog.src order:
//   T table DBT   D other DBT   K key DBT   I ix (short)   i other int/short
//   G genid_t     P prevllsn    L other DB_LSN   k keylen   A isabort (short)
struct Layout {
    uint32_t type;
    const char *prog;
};
//   d dtalen (the int after keylen in the keyless index records)
constexpr Layout kLayouts[] = {
    {HSC_REC_UNDO_ADD_DTA, "TiiGGPD"},      // llog.src:26-34
    {HSC_REC_UNDO_ADD_IX, "TIGGPkd"},       // :36-44
    {HSC_REC_LTRAN_COMMIT, "GPGA"},         // :46-51
    {HSC_REC_LTRAN_START, "Gi"},            // :54-59
    {HSC_REC_LTRAN_COMPREC, "GPL"},         // :65-69
    {HSC_REC_UNDO_DEL_DTA, "TGGPiiiD"},     // :73-82
    {HSC_REC_UNDO_DEL_IX, "TGIGPDkd"},      // :84-93
    {HSC_REC_UNDO_UPD_DTA, "TGGGPiiDDi"},   // :95-106
    {HSC_REC_UNDO_UPD_IX, "TGGGPIKi"},      // :108-117
    {HSC_REC_UNDO_ADD_DTA_LK, "TiiGGP"},    // :139-146
    {HSC_REC_UNDO_ADD_IX_LK, "TIGGPKi"},    // :152-160
    {HSC_REC_UNDO_DEL_DTA_LK, "TGGPiii"},   // :167-175
    {HSC_REC_UNDO_DEL_IX_LK, "TGIGPkd"},    // :183-191
    {HSC_REC_UNDO_UPD_DTA_LK, "TGGGPiii"},  // :199-208
    {HSC_REC_UNDO_UPD_IX_LK, "TGGGPIKi"},   // :216-225
};

const char *layout_of(uint32_t type)
{
    for (const Layout &l : kLayouts)
        if (l.type == type) return l.prog;
    return nullptr;
}

bool keyless_ix(uint32_t t)
{
    return t == HSC_REC_UNDO_ADD_IX || t == HSC_REC_UNDO_DEL_IX || t == HSC_REC_UNDO_DEL_IX_LK;
}


// ---------------------------------------------------------------------------
// Index-key reconstruction from the physical log (bdb/rowlocks.c:209-617)
// ---------------------------------------------------------------------------
constexpr uint32_t kDbAddDup = 1;             // berkdb/dbinc/db_am.h:23
constexpr uint8_t kBKeyData = 1, kBOverflow = 3;  // db_page.h:606-608
constexpr uint8_t kBTypeMask = (uint8_t)~(0x80 | 0x40 | 0x20);  // B_TYPE: ~(B_DELETE|B_PFX|B_RLE)

enum WalkRc { kWalkOk = 0, kWalkNoLog = 1, kWalkBad = 2 };

// A reconstruct buffer (malloc'd / alloca'd uninitialised in the reference)
// and which of its bytes a walk wrote.
struct KeyBuf {
    std::vector<uint8_t> b, w;
    void init(int n)
    {
        b.assign(n > 0 ? (size_t)n : 0, 0);
        w.assign(b.size(), 0);
    }
    bool put(int64_t at, const uint8_t *src, size_t n)
    {
        if (at < 0 || (size_t)at + n > b.size()) return false;  // the reference writes past it
        if (n) memcpy(b.data() + at, src, n);
        std::fill(w.begin() + at, w.begin() + at + (long)n, 1);
        return true;
    }
};

// A stored record's bytes and a bounded view of the item its hdr DBT points
// at (the BKEYDATA / BOVERFLOW casts of :293-338 read without size checks; a
// read outside the record is reported instead).
struct PhysRec {
    const uint8_t *p;
    uint32_t n;
    bool byte(size_t at, uint8_t *out) const
    {
        if (at >= n) return false;
        *out = p[at];
        return true;
    }
};

struct Addrem {  // __db_addrem_args, the fields the walk reads (db.src:47-57)
    uint32_t opcode;
    uint32_t hdr_size, dbt_size;
    size_t hdr_at, dbt_at;  // offsets of the DBT data in the record
};

static bool parse_addrem(const PhysRec &r, Addrem *a)
{
    Reader rd{r.p + 16, r.p + r.n};
    a->opcode = rd.u32();
    for (int k = 0; k < 4; ++k) (void)rd.u32();  // fileid, pgno, indx, nbytes
    const uint8_t *d = nullptr;
    a->hdr_size = 0;
    const uint32_t hs = rd.u32();
    a->hdr_at = (size_t)(rd.p - r.p);
    if (!rd.need(hs)) return false;
    rd.p += hs;
    a->hdr_size = hs;
    rd.dbt(&d, &a->dbt_size);
    if (!rd.ok) return false;
    a->dbt_at = (size_t)(d - r.p);
    (void)rd.lsn();  // pagelsn: the generated reader reads it too
    return rd.ok;
}

static bool parse_big(const PhysRec &r, uint32_t *size, size_t *at)
{
    Reader rd{r.p + 16, r.p + r.n};
    for (int k = 0; k < 5; ++k) (void)rd.u32();  // opcode, fileid, pgno, prev_pgno, next_pgno
    const uint8_t *d = nullptr;
    rd.dbt(&d, size);
    if (!rd.ok) return false;
    *at = (size_t)(d - r.p);
    for (int k = 0; k < 3; ++k) (void)rd.lsn();  // pagelsn, prevlsn, nextlsn
    return rd.ok;
}

// get_next_addrem_buffer (bdb/rowlocks.c:209-426): from *lsn back along the
// header prev_lsn chain to the first addrem that yields an item (a DB_ADD_DUP
// with no or a type-0 header: its dbt; a B_KEYDATA header item: its bytes) or
// to the __db_big record that completes an overflow item (B_OVERFLOW header:
// tlen, then the big records' dbts copied back to front).  An addrem seen
// after a pg_free / pg_freedata (walking back) is skipped, and so is every
// addrem or debug record after it until another record type.  lsn and
// nextlsn may alias (bdb_reconstruct_add passes &nextlsn for both).
static int addrem_walk(const PhysStore &ps, uint64_t *lsn, KeyBuf *buf, int len, int *have,
                       uint64_t *nextlsn)
{
    int64_t off = 0;
    bool pgfree = false, stopped = false;
    uint64_t prevlsn = 0;
    while ((*lsn >> 32) != 0) {
        const uint64_t cur = *lsn;  // lsn and nextlsn may alias
        const long i = ps.find(cur);
        if (i < 0) return kWalkNoLog;  // DB_NOTFOUND -> BDBERR_NO_LOG
        const uint32_t type = ps.type[i];
        prevlsn = ps.prev[i];
        *nextlsn = prevlsn;
        // a chain that does not go back would not terminate in the reference
        if ((prevlsn >> 32) != 0 && prevlsn >= cur) return kWalkBad;
        if (type == HSC_REC_DB_PG_FREE || type == HSC_REC_DB_PG_FREEDATA)
            pgfree = true;
        else if (type != HSC_REC_DB_ADDREM && type != HSC_REC_DB_DEBUG)
            pgfree = false;
        if (type == HSC_REC_DB_ADDREM) {
            const PhysRec r{ps.bytes.data() + ps.off[i], ps.len[i]};
            Addrem a;
            if (!parse_addrem(r, &a)) return kWalkBad;
            if (!pgfree) {
                uint8_t t = 0;
                if (a.hdr_size > 0 && !r.byte(a.hdr_at + 2, &t)) return kWalkBad;
                if (a.opcode == kDbAddDup && (a.hdr_size == 0 || (t & kBTypeMask) == 0)) {
                    // an add: the item is the record's dbt
                    if (buf && a.dbt_size > (uint32_t)len) {
                        *have = 0;
                    } else {
                        *have = 1;
                        if (buf && !buf->put(0, r.p + a.dbt_at, a.dbt_size)) return kWalkBad;
                    }
                    stopped = true;
                    break;
                }
                // hdr.data points into the record even when hdr.size is 0
                if (!r.byte(a.hdr_at + 2, &t)) return kWalkBad;
                const uint8_t bt = t & kBTypeMask;
                if (bt == kBOverflow) {
                    uint8_t b[4];
                    for (int k = 0; k < 4; ++k)
                        if (!r.byte(a.hdr_at + 8 + k, &b[k])) return kWalkBad;
                    const uint32_t tlen = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 |
                                          (uint32_t)b[3] << 24;  // BOVERFLOW.tlen, native
                    if (tlen > 0x7FFFFFFFu) return kWalkBad;
                    off = tlen;
                } else if (bt == kBKeyData) {
                    uint8_t b0, b1;
                    if (!r.byte(a.hdr_at, &b0) || !r.byte(a.hdr_at + 1, &b1)) return kWalkBad;
                    const uint32_t klen = (uint32_t)b0 | (uint32_t)b1 << 8;  // BKEYDATA.len, native
                    if (buf) {
                        if ((int)klen > len) return kWalkBad;  // abort(), :342-352
                        if (a.hdr_at + 3 + klen > r.n) return kWalkBad;
                        if (!buf->put(0, r.p + a.hdr_at + 3, klen)) return kWalkBad;
                    }
                    *have = 1;
                    stopped = true;
                    break;
                } else {
                    *have = 0;  // "Unexpected type"
                }
            }
        } else if (type == HSC_REC_DB_BIG) {
            const PhysRec r{ps.bytes.data() + ps.off[i], ps.len[i]};
            uint32_t size = 0;
            size_t at = 0;
            if (!parse_big(r, &size, &at)) return kWalkBad;
            off -= (int64_t)size;
            if (off < 0) {
                *have = 0;  // "huh?"
            } else {
                if (buf && !buf->put(off, r.p + at, size)) return kWalkBad;
                if (off == 0) {
                    *have = 1;
                    stopped = true;
                    break;
                }
            }
        }
        *lsn = prevlsn;
    }
    if (stopped) *lsn = prevlsn;  // :419-420
    return kWalkOk;
}

// bdb_reconstruct_add (:428-456) with data = NULL (bdb/serializable.c:127):
// the first walk passes the data item (logged after the key), the second one
// fills the key.
static int recon_add(const PhysStore &ps, uint64_t start, int keylen, int dtalen, KeyBuf &key)
{
    int have = 0;
    uint64_t lsn = start, nextlsn = (uint64_t)1 << 32;  // {1, 0}
    int rc = addrem_walk(ps, &lsn, nullptr, dtalen, &have, &nextlsn);
    if (rc) return rc;
    key.init(keylen);
    return addrem_walk(ps, &nextlsn, &key, keylen, &have, &nextlsn);
}

// bdb_reconstruct_delete (:535-617) with page, index and data NULL: walks in
// turn into two alternating buffers until both hold an item; the key is the
// buffer of the last walk (the first of the pair in log order).
static int recon_delete(const PhysStore &ps, uint64_t start, int keylen, int dtalen, KeyBuf &key)
{
    if ((start >> 32) == 0) return kWalkBad;  // nextlsn would stay uninitialised
    const int alloclen = std::max(keylen, dtalen);
    KeyBuf buf[2];
    buf[0].init(alloclen);
    buf[1].init(alloclen);
    int haveit[2] = {0, 0};
    uint64_t lsn = start, nextlsn = 0;
    int i = 0;
    do {
        i++;
        const int rc = addrem_walk(ps, &lsn, alloclen > 0 ? &buf[i % 2] : nullptr, alloclen,
                                   &haveit[i % 2], &nextlsn);
        if (rc) return rc;
    } while ((nextlsn >> 32) != 0 && (!haveit[0] || !haveit[1]));
    if (!(haveit[0] && haveit[1])) return 1;
    key.init(keylen);
    for (int k = 0; k < keylen; ++k) {
        key.b[k] = buf[i % 2].b[k];
        key.w[k] = buf[i % 2].w[k];
    }
    return kWalkOk;
}

}  // namespace

long PhysStore::find(uint64_t l) const
{
    auto p = std::lower_bound(lsn.begin(), lsn.end(), l);
    return (p != lsn.end() && *p == l) ? (long)(p - lsn.begin()) : -1;
}

// The records of raw (already in ps) into out.
static int decode_records(const hsc_raw_log *raw, DecodedLog &out, const PhysStore &ps,
                          std::string &err)
{
    const size_t n = raw->nrec;
    out = DecodedLog();
    out.lsn.resize(n);
    out.rectype.resize(n);
    out.prev.resize(n);
    out.isabort.assign(n, 0);
    out.table.assign(n, -1);
    out.ix.assign(n, 0);
    out.key_off.assign(n, 0);
    out.keylen.assign(n, 0);
    std::unordered_map<std::string, int> tids;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t off = raw->off[i];
        const uint32_t len = raw->len[i];
        Reader r{raw->buf + off, raw->buf + off + len};
        out.lsn[i] = raw->lsn[i];
        const uint32_t type = r.u32();
        (void)r.u32();  // txnid
        const uint64_t hdr_prev = r.lsn();
        if (!r.ok) {
            err = "truncated record header at record " + std::to_string(i);
            return HSC_ELOG;
        }
        out.rectype[i] = type;
        out.prev[i] = hdr_prev;  // regops and non-logical records
        const char *prog = layout_of(type);
        if (!prog) continue;
        out.prev[i] = 0;
        const uint8_t *key = nullptr;
        uint32_t keylen = 0, dtalen = 0;
        bool has_key = false;
        for (const char *f = prog; *f; ++f) {
            switch (*f) {
            case 'T': {
                const uint8_t *d = nullptr;
                uint32_t sz = 0;
                r.dbt(&d, &sz);
                if (!r.ok) break;
                // the table DBT carries the NUL-terminated name
                size_t l = 0;
                while (l < sz && d[l]) ++l;
                std::string name((const char *)d, l);
                auto it = tids.find(name);
                int t;
                if (it == tids.end()) {
                    t = (int)out.names.size();
                    tids.emplace(name, t);
                    out.names.push_back(name);
                } else {
                    t = it->second;
                }
                out.table[i] = t;
                break;
            }
            case 'D': r.skip_dbt(); break;
            case 'K':
                r.dbt(&key, &keylen);
                has_key = r.ok;
                break;
            case 'I': out.ix[i] = (int16_t)r.u32(); break;
            case 'i': (void)r.u32(); break;
            case 'G': (void)r.genid(); break;
            case 'P': out.prev[i] = r.lsn(); break;
            case 'L': (void)r.lsn(); break;
            case 'k': keylen = r.u32(); break;
            case 'd': dtalen = r.u32(); break;
            case 'A': out.isabort[i] = (int16_t)r.u32(); break;
            }
            if (!r.ok) {
                err = "truncated record body at record " + std::to_string(i);
                return HSC_ELOG;
            }
        }
        KeyBuf rk;
        if (keyless_ix(type)) {
            // bdb_reconstruct_add/delete at undolsn = header prev_lsn: the
            // caller's side table if it names undolsn, else the log walk
            const uint64_t *b = raw->recon_lsn, *e = raw->recon_lsn + raw->nrecon;
            const uint64_t *hit = raw->nrecon ? std::lower_bound(b, e, hdr_prev) : e;
            if (hit != e && *hit == hdr_prev) {
                const size_t k = (size_t)(hit - b);
                if ((uint32_t)raw->recon_len[k] != keylen) {
                    err = "reconstructed key length differs from the record's keylen at record " +
                          std::to_string(i);
                    return HSC_ELOG;
                }
                key = raw->recon_keys + raw->recon_off[k];
            } else {
                if (keylen > 0x7FFFFFFFu || dtalen > 0x7FFFFFFFu) {
                    err = "key or data length out of range at record " + std::to_string(i);
                    return HSC_ELOG;
                }
                const int rc = type == HSC_REC_UNDO_ADD_IX
                                   ? recon_add(ps, hdr_prev, (int)keylen, (int)dtalen, rk)
                                   : recon_delete(ps, hdr_prev, (int)keylen, (int)dtalen, rk);
                bool full = rc == kWalkOk && rk.b.size() == keylen;
                for (size_t k = 0; full && k < rk.w.size(); ++k) full = rk.w[k] != 0;
                if (!full) {
                    err = "index key of record " + std::to_string(i) +
                          " not reconstructed from the physical log (" +
                          (rc == kWalkNoLog ? "a record of the walk is missing"
                           : rc == kWalkBad ? "malformed physical record"
                                            : "no complete key item") + ")";
                    return HSC_ELOG;
                }
                key = rk.b.data();
            }
            has_key = true;
        }
        if (has_key) {
            out.key_off[i] = out.keys.size();
            out.keylen[i] = (int32_t)keylen;
            out.keys.insert(out.keys.end(), key, key + keylen);
        }
    }
    out.end_lsn = raw->end_lsn;
    out.view();
    return HSC_OK;
}

int decode_raw_log(const hsc_raw_log *raw, DecodedLog &out, PhysStore &ps, bool reset,
                   std::string &err)
{
    const size_t n = raw->nrec;
    for (size_t i = 1; i < raw->nrecon; ++i)
        if (raw->recon_lsn[i] <= raw->recon_lsn[i - 1]) {
            err = "reconstructed keys not sorted by undolsn";
            return HSC_EINVAL;
        }
    for (size_t i = 1; i < n; ++i)
        if (raw->lsn[i] <= raw->lsn[i - 1]) {
            err = "record LSNs not increasing at record " + std::to_string(i);
            return HSC_EINVAL;
        }
    // every record joins the store first: a walk may visit any earlier one
    if (reset || (n && !ps.lsn.empty() && raw->lsn[0] <= ps.lsn.back())) ps.clear();
    const size_t base = ps.lsn.size(), bytes_base = ps.bytes.size();
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = raw->buf + raw->off[i];
        const uint32_t len = raw->len[i];
        if (len < 16) {
            ps.truncate(base, bytes_base);
            err = "truncated record header at record " + std::to_string(i);
            return HSC_ELOG;
        }
        Reader r{p, p + len};
        const uint32_t type = r.u32();
        (void)r.u32();
        const uint64_t prev = r.lsn();
        ps.lsn.push_back(raw->lsn[i]);
        ps.prev.push_back(prev);
        ps.type.push_back(type);
        ps.len.push_back(len);
        ps.off.push_back(ps.bytes.size());
        if (type == HSC_REC_DB_ADDREM || type == HSC_REC_DB_BIG) ps.bytes.insert(ps.bytes.end(), p, p + len);
    }
    const int rc = decode_records(raw, out, ps, err);
    if (rc) ps.truncate(base, bytes_base);  // a failed decode leaves the store as it was
    return rc;
}


void DecodedLog::view()
{
    name_ptrs.clear();
    for (const std::string &s : names) name_ptrs.push_back(s.c_str());
    if (keys.empty()) keys.push_back(0);
    llog.nrec = lsn.size();
    llog.lsn = lsn.data();
    llog.rectype = rectype.data();
    llog.prev = prev.data();
    llog.isabort = isabort.data();
    llog.table = table.data();
    llog.ix = ix.data();
    llog.key_off = key_off.data();
    llog.keylen = keylen.data();
    llog.keys = keys.data();
    llog.tbnames = name_ptrs.data();
    llog.ntbnames = (int)names.size();
    llog.end_lsn = end_lsn;
}

}  // namespace hsc
