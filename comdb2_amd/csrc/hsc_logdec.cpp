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
// record the header prev_lsn.  Keys of undo_add_ix / undo_del_ix /
// undo_del_ix_lk are not in the record: the reference rebuilds them from the
// physical log at undolsn = the header prev_lsn (bdb/serializable.c:123-130,
// 174-181 -> bdb/rowlocks.c:428-617); here the caller supplies them as a
// side table keyed by undolsn (hsc_raw_log.recon_*).
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
constexpr Layout kLayouts[] = {
    {HSC_REC_UNDO_ADD_DTA, "TiiGGPD"},      // llog.src:26-34
    {HSC_REC_UNDO_ADD_IX, "TIGGPki"},       // :36-44
    {HSC_REC_LTRAN_COMMIT, "GPGA"},         // :46-51
    {HSC_REC_LTRAN_START, "Gi"},            // :54-59
    {HSC_REC_LTRAN_COMPREC, "GPL"},         // :65-69
    {HSC_REC_UNDO_DEL_DTA, "TGGPiiiD"},     // :73-82
    {HSC_REC_UNDO_DEL_IX, "TGIGPDki"},      // :84-93
    {HSC_REC_UNDO_UPD_DTA, "TGGGPiiDDi"},   // :95-106
    {HSC_REC_UNDO_UPD_IX, "TGGGPIKi"},      // :108-117
    {HSC_REC_UNDO_ADD_DTA_LK, "TiiGGP"},    // :139-146
    {HSC_REC_UNDO_ADD_IX_LK, "TIGGPKi"},    // :152-160
    {HSC_REC_UNDO_DEL_DTA_LK, "TGGPiii"},   // :167-175
    {HSC_REC_UNDO_DEL_IX_LK, "TGIGPki"},    // :183-191
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

}  // namespace

int decode_raw_log(const hsc_raw_log *raw, DecodedLog &out, std::string &err)
{
    const size_t n = raw->nrec;
    for (size_t i = 1; i < raw->nrecon; ++i)
        if (raw->recon_lsn[i] <= raw->recon_lsn[i - 1]) {
            err = "reconstructed keys not sorted by undolsn";
            return HSC_EINVAL;
        }
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
        uint32_t keylen = 0;
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
            case 'A': out.isabort[i] = (int16_t)r.u32(); break;
            }
            if (!r.ok) {
                err = "truncated record body at record " + std::to_string(i);
                return HSC_ELOG;
            }
        }
        if (keyless_ix(type)) {
            // bdb_reconstruct_add/delete at undolsn = header prev_lsn
            const uint64_t *b = raw->recon_lsn, *e = raw->recon_lsn + raw->nrecon;
            const uint64_t *hit = std::lower_bound(b, e, hdr_prev);
            if (hit == e || *hit != hdr_prev) {
                err = "no reconstructed key for keyless index record at record " + std::to_string(i);
                return HSC_ELOG;
            }
            const size_t k = (size_t)(hit - b);
            if ((uint32_t)raw->recon_len[k] != keylen) {
                err = "reconstructed key length differs from the record's keylen at record " +
                      std::to_string(i);
                return HSC_ELOG;
            }
            key = raw->recon_keys + raw->recon_off[k];
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
