// OSQL_SERIAL read-set decoder: payloads straight into the hsc_readsets SoA,
// skipping the reference's per-range heap CurRange objects
// (SURVEY.md §8(f) row 2).
//
// Wire format, as written by osql_send_serial (db/osqlcomm.c:4306-4440):
//   osql_serial_t (db/osqlcomm.c:748-753, osqlcomm_serial_type_get :809-826)
//       buf_size i32 | arr_size i32 | file u32 | offset u32
//   arr_size ranges (serial_readset_put / _get, db/osqlcomm.c:909-993):
//       tblen i32 | tbname[tblen] (NUL included) | islocked i32
//       if !islocked: idxnum i32 | lflag i32 | [lkeylen i32 | lkey] if !lflag
//                                | rflag i32 | [rkeylen i32 | rkey] if !rflag
//       if islocked: the receiver sets lflag = rflag = 1 and idxnum stays
//       currange_new's -2 (db/sqlglue.c:163-176)
// Every field goes through buf_put / buf_get (bbinc/endian_core.h:30-34,
// bbinc/endian_core.amd64.h:17-44), which byte-swap ANY 2-, 4- or 8-byte
// item -- the integers, but also a table name of 1, 3 or 7 characters and a
// key of 2, 4 or 8 bytes.  Decoding therefore reverses every 2/4/8-byte item.
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/hip_serial.h"
#include "hsc_internal.h"

namespace hsc {
namespace {

struct WireReader {
    const uint8_t *p, *end;
    bool ok = true;
    // buf_get of `n` bytes into dst (2/4/8-byte items arrive byte-reversed)
    bool get(void *dst, size_t n)
    {
        if (!ok || (size_t)(end - p) < n) return ok = false;
        uint8_t *d = (uint8_t *)dst;
        if (n == 2 || n == 4 || n == 8)
            for (size_t i = 0; i < n; ++i) d[i] = p[n - 1 - i];
        else if (n)  // an empty key lands in an empty buffer (dst may be null)
            memcpy(d, p, n);
        p += n;
        return true;
    }
    int32_t i32()
    {
        int32_t v = 0;
        get(&v, 4);
        return v;
    }
};

}  // namespace

int decode_serial_msgs(const hsc_serial_msgs *m, DecodedReadSets &out, std::string &err)
{
    out = DecodedReadSets();
    std::unordered_map<std::string, int> tids;
    out.txn_off.push_back(0);
    std::vector<uint8_t> tmp;
    for (size_t i = 0; i < m->nmsg; ++i) {
        WireReader r{m->buf + m->off[i], m->buf + m->off[i] + m->len[i]};
        const int32_t buf_size = r.i32();
        const int32_t arr_size = r.i32();
        const uint32_t file = (uint32_t)r.i32();
        const uint32_t offset = (uint32_t)r.i32();
        if (!r.ok || buf_size < 0 || arr_size < 0 || (size_t)(r.end - r.p) < (size_t)buf_size) {
            err = "malformed OSQL_SERIAL header in message " + std::to_string(i);
            return HSC_EINVAL;
        }
        r.end = r.p + buf_size;  // p_buf_end = p_buf + dt.buf_size (:6884)
        out.snap.push_back((uint64_t)file << 32 | offset);
        for (int32_t k = 0; k < arr_size; ++k) {
            const int32_t tblen = r.i32();
            if (!r.ok || tblen <= 0 || (size_t)(r.end - r.p) < (size_t)tblen) {
                r.ok = false;
                break;
            }
            tmp.resize(tblen);
            r.get(tmp.data(), (size_t)tblen);
            size_t l = 0;
            while (l < tmp.size() && tmp[l]) ++l;
            std::string name((const char *)tmp.data(), l);
            auto it = tids.find(name);
            int tid;
            if (it == tids.end()) {
                tid = (int)out.names.size();
                tids.emplace(name, tid);
                out.names.push_back(name);
            } else {
                tid = it->second;
            }
            const int32_t islocked = r.i32();
            int32_t idxnum = -2, lflag = 1, rflag = 1, lkeylen = 0, rkeylen = 0;
            // keys the message does not carry stay NULL (currange_new,
            // db/sqlglue.c:163-175); carried ones are malloc'd, even when empty
            uint64_t lkey_off = HSC_KEY_NULL, rkey_off = HSC_KEY_NULL;
            if (!islocked) {
                idxnum = r.i32();
                lflag = r.i32();
                if (!lflag) {
                    lkeylen = r.i32();
                    if (!r.ok || lkeylen < 0 || (size_t)(r.end - r.p) < (size_t)lkeylen) {
                        r.ok = false;
                        break;
                    }
                    lkey_off = out.keys.size();
                    out.keys.resize(out.keys.size() + lkeylen);
                    r.get(out.keys.data() + lkey_off, (size_t)lkeylen);
                }
                rflag = r.i32();
                if (!rflag) {
                    rkeylen = r.i32();
                    if (!r.ok || rkeylen < 0 || (size_t)(r.end - r.p) < (size_t)rkeylen) {
                        r.ok = false;
                        break;
                    }
                    rkey_off = out.keys.size();
                    out.keys.resize(out.keys.size() + rkeylen);
                    r.get(out.keys.data() + rkey_off, (size_t)rkeylen);
                }
            }
            if (!r.ok) break;
            out.table.push_back(tid);
            out.idxnum.push_back(idxnum);
            out.lflag.push_back(lflag);
            out.rflag.push_back(rflag);
            out.islocked.push_back(islocked);
            out.lkeylen.push_back(lkeylen);
            out.rkeylen.push_back(rkeylen);
            out.lkey_off.push_back(lkey_off);
            out.rkey_off.push_back(rkey_off);
        }
        if (!r.ok) {
            err = "truncated OSQL_SERIAL read set in message " + std::to_string(i);
            return HSC_EINVAL;
        }
        out.txn_off.push_back((int64_t)out.table.size());
    }
    out.view();
    return HSC_OK;
}

void DecodedReadSets::view()
{
    name_ptrs.clear();
    for (const std::string &s : names) name_ptrs.push_back(s.c_str());
    if (keys.empty()) keys.push_back(0);
    rs.ntxn = (int)snap.size();
    rs.txn_off = txn_off.data();
    rs.snap = snap.data();
    rs.table = table.data();
    rs.idxnum = idxnum.data();
    rs.lflag = lflag.data();
    rs.rflag = rflag.data();
    rs.islocked = islocked.data();
    rs.lkeylen = lkeylen.data();
    rs.rkeylen = rkeylen.data();
    rs.lkey_off = lkey_off.data();
    rs.rkey_off = rkey_off.data();
    rs.keys = keys.data();
    rs.tbnames = name_ptrs.data();
    rs.ntbnames = (int)names.size();
}

}  // namespace hsc
