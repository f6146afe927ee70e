// hsc_host.cpp -- host side of the MI355X serializable conflict validator.
//
// Implements include/hip_serial.h:
//   * the write window: decoded from the log stream the way
//     osql_serial_check / serial_check_this_txn walk it
//     (bdb/serializable.c:390-539 and 60-332), kept resident on the GPU;
//   * the marshaller: CurRangeArr (db/comdb2.h:1105-1124) or flat read sets
//     -> device probe struct-of-arrays, applying the span and lock rules of
//     currangearr_build_hash + serial_check_callback (db/sqlglue.c:312-351,
//     db/glue.c:2926-2963) and the min-length memcmp padding lemma;
//   * the drop-in entry points bdb_osql_serial_check / check_batch.
// There is no CPU verdict path: every range verdict comes from the GPU join.
#include "../../include/hip_serial.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

using namespace hsc;

#include "hsc_ctx.h"


// probe scratch that moves with a lane (hsc_ctx::Lane::b holds at most 20)
static DBuf hsc_ctx::*const kLaneBufs[] = {
    &hsc_ctx::w_code,      &hsc_ctx::w_hist,      &hsc_ctx::w_counts, &hsc_ctx::w_bucket,
    &hsc_ctx::w_cursor,    &hsc_ctx::w_items,     &hsc_ctx::w_item_tile, &hsc_ctx::w_item_desc,
    &hsc_ctx::w_recs,      &hsc_ctx::w_tcode,     &hsc_ctx::w_tcode2, &hsc_ctx::w_trecs,
    &hsc_ctx::w_vflags,    &hsc_ctx::d_done,      &hsc_ctx::p_code_lo, &hsc_ctx::p_code_hi};
static_assert(sizeof kLaneBufs / sizeof kLaneBufs[0] <= 20, "Lane::b size");

// Make the lane of c->stream active (the least recently used lane if the
// stream has none).
static hipError_t select_lane(hsc_ctx *c)
{
    int want = -1;
    for (int i = 0; i < hsc_ctx::kLanes; ++i)
        if (c->lanes[i].stream == c->stream && c->lanes[i].tick) want = i;
    if (want < 0) {
        want = 0;
        for (int i = 1; i < hsc_ctx::kLanes; ++i)
            if (c->lanes[i].tick < c->lanes[want].tick) want = i;
    }
    if (want != c->lane) {
        int k = 0;
        for (DBuf hsc_ctx::*m : kLaneBufs) {
            std::swap(c->*m, c->lanes[c->lane].b[k]);  // park the active lane's buffer
            std::swap(c->*m, c->lanes[want].b[k]);     // take the wanted lane's
            ++k;
        }
        c->lane = want;
    }
    hsc_ctx::Lane &L = c->lanes[want];
    if (L.stream != c->stream) {
        if (L.done && L.tick) {
            hipError_t e = hipStreamWaitEvent(c->stream, L.done, 0);
            if (e != hipSuccess) return e;
        }
        L.stream = c->stream;
    }
    L.tick = ++c->lane_tick;
    return hipSuccess;
}

// After a batch: the lane's done event marks the end of its scratch use.
static hipError_t lane_done(hsc_ctx *c)
{
    hsc_ctx::Lane &L = c->lanes[c->lane];
    if (!L.done) {
        hipError_t e = hipEventCreateWithFlags(&L.done, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    L.pend = false;
    return hipEventRecord(L.done, c->stream);
}

// A batch of the active lane went onto c->stream: its done event is recorded
// when the context leaves the stream (lane_leave) -- a take-over of the lane
// or a window change from another stream happens only after that.
static void lane_mark(hsc_ctx *c) { c->lanes[c->lane].pend = true; }

static hipError_t lane_leave(hsc_ctx *c)
{
    hsc_ctx::Lane &L = c->lanes[c->lane];
    return L.pend && L.stream == c->stream ? lane_done(c) : hipSuccess;
}

hipError_t hsc::ctx_switch_stream(hsc_ctx *c, hipStream_t s)
{
    if (s == c->stream) return hipSuccess;
    const hipError_t e = lane_leave(c);
    c->stream = s;
    return e;
}

// Small batches (k_small_narrow) run on the stream current at their launch
// without a probe lane, and their callers read the verdicts without c->mu:
// before the window changes or the stream switches, the host waits until no
// small slot is in flight (a slot is released by its caller once its kernel's
// done word is seen, which needs no c->mu).  Called under c->mu.
static hipError_t wait_small(hsc_ctx *c)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (auto &sl : c->small)
        while (sl.busy.load(std::memory_order_acquire)) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                return hipErrorLaunchTimeOut;  // a slot whose kernel never finished
        }
    return hipSuccess;
}

// Before the window changes: c->stream waits for every lane's last batch
// (and the host for every small batch in flight).
static hipError_t wait_lanes(hsc_ctx *c)
{
    if (const hipError_t e = wait_small(c); e != hipSuccess) return e;
    for (auto &L : c->lanes)
        if (L.done && L.tick && L.stream != c->stream) {
            hipError_t e = hipStreamWaitEvent(c->stream, L.done, 0);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

static int fail(hsc_ctx *c, int code, const char *what, hipError_t e = hipSuccess);

// the next append staging buffer of the ring (waits only if the copies that
// read it two appends ago have not run yet)
// HSC_FOLD_TRACE: fold events with a steady-clock stamp (diagnostics)
static bool fold_trace()
{
    static const bool on = getenv("HSC_FOLD_TRACE") != nullptr;
    return on;
}
static double trace_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int app_stage(hsc_ctx *c, size_t bytes)
{
    const int i = c->app_i;
    if (c->app_ev[i] && hipEventSynchronize(c->app_ev[i]) != hipSuccess)
        return fail(c, HSC_EDEVICE, "append staging event");
    // fine-grained and mapped: a commit's few rows are read in place by the merge
    if (c->h_appq[i].ensure(bytes, true, true)) return fail(c, HSC_ENOMEM, "append staging");
    c->h_app = &c->h_appq[i];
    return HSC_OK;
}

// the staged buffer's copies (and the work behind them) are on stream s
static int app_staged(hsc_ctx *c, hipStream_t s)
{
    const int i = c->app_i;
    if (!c->app_ev[i] && hipEventCreateWithFlags(&c->app_ev[i], hipEventDisableTiming) != hipSuccess)
        return fail(c, HSC_EDEVICE, "append event");
    if (hipEventRecord(c->app_ev[i], s) != hipSuccess) return fail(c, HSC_EDEVICE, "append event");
    c->app_last = c->app_ev[i];
    c->app_seq++;
    c->app_i ^= 1;
    return HSC_OK;
}

static int fail(hsc_ctx *c, int code, const char *what, hipError_t e)
{
    char buf[256];
    if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof buf, "%s", what);
    c->err = buf;
    return code;
}

#define HIPCHK(c, call)                                          \
    do {                                                         \
        hipError_t e_ = (call);                                  \
        if (e_ != hipSuccess) return fail((c), HSC_EDEVICE, #call, e_); \
    } while (0)

// the bits of x under mask m, packed to the low end (MSB order kept)
static uint64_t host_compress(uint64_t x, uint64_t m)
{
    uint64_t r = 0;
    for (int b = 63; b >= 0; --b)
        if ((m >> b) & 1) r = (r << 1) | ((x >> b) & 1);
    return r;
}

static int table_id_or_add(hsc_ctx *c, const char *name)
{
    auto it = c->table_ids.find(name);
    if (it != c->table_ids.end()) return it->second;
    int tid = (int)c->table_names.size();
    c->dict_epoch++;
    c->table_ids.emplace(name, tid);
    c->table_names.emplace_back(name);
    c->h_table_max.push_back(0);
    return tid;
}

static void set_words(hsc_ctx *c, int W)
{
    if (c->W != W) c->dict_epoch++;
    c->W = W;
}

static int group_id_or_add(hsc_ctx *c, int tid, int ix, int klen)
{
    uint64_t k = ((uint64_t)(uint32_t)tid << 40) ^ ((uint64_t)(uint16_t)ix << 24) ^ (uint32_t)klen;
    // disambiguate collisions by scanning (keys are tiny; collisions impossible
    // for tid < 2^24, |ix| < 2^15, klen < 2^24)
    auto it = c->group_ids.find(k);
    if (it != c->group_ids.end()) return it->second;
    int g = (int)c->groups.size();
    c->dict_epoch++;
    c->groups.push_back({tid, ix, klen});
    c->group_ids.emplace(k, g);
    c->ix_groups[ixkey(tid, ix)].push_back(g);
    return g;
}

static void fold_discard(hsc_ctx *c);

// The pending tail's rows and table entries are all in app_* / the uploaded
// table maxima now (or dropped with them): the next append mirrors into the
// other buffer, this one is refilled once the launches queued so far ran.
static void pend_retire(hsc_ctx *c)
{
    c->app_tchg.clear();
    if (!c->pend_n && !c->pend_t) return;
    (void)wait_small(c);  // small batches on side streams read the tail too
    const int i = c->pend_i;
    if ((!c->pend_ev[i] && hipEventCreateWithFlags(&c->pend_ev[i], hipEventDisableTiming) != hipSuccess) ||
        hipEventRecord(c->pend_ev[i], c->stream) != hipSuccess) {
        if (c->pend_ev[i]) (void)hipEventDestroy(c->pend_ev[i]);
        c->pend_ev[i] = nullptr;
        (void)hipStreamSynchronize(c->stream);  // no event: nothing may still read the buffer
    }
    c->pend_i ^= 1;
    c->pend_n = c->pend_t = 0;
}

static void clear_window(hsc_ctx *c)
{
    fold_discard(c);
    c->h_gid.clear();
    c->h_keyoff.clear();
    c->h_keys.clear();
    c->h_lsn.clear();
    std::fill(c->h_table_max.begin(), c->h_table_max.end(), 0);
    c->max_commit = 0;
    c->poison_regop = c->poison_chain = 0;
    c->lg.clear();
    c->lg_rule = false;
    c->last_append_lsn = 0;
    c->host_staged = true;
    c->dirty = true;
    c->live = false;
    c->merge_pending = false;
    c->dn = 0;
    c->app_gid.clear(), c->app_keys.clear(), c->app_koff.clear(), c->app_lsn.clear();
    c->app_tmax = false;
    pend_retire(c);
    c->n = 0;
}

// A write committed at lsn to table tid: its maximum rises (the pending
// tail mirrors the tables whose maximum rose since its last mirror).
static void raise_table_max(hsc_ctx *c, int tid, uint64_t lsn)
{
    if (lsn > c->h_table_max[tid]) {
        c->h_table_max[tid] = lsn;
        c->app_tmax = true;
        if (c->live && !c->host_only && (c->app_tchg.empty() || c->app_tchg.back() != (uint32_t)tid))
            c->app_tchg.push_back((uint32_t)tid);
    }
}

static void add_write(hsc_ctx *c, int tid, int ix, const uint8_t *key, int keylen, bool has_key,
                      uint64_t lsn)
{
    raise_table_max(c, tid, lsn);
    if (lsn > c->max_commit) c->max_commit = lsn;
    if (!has_key) return;
    if (keylen < 0) keylen = 0;
    int g = group_id_or_add(c, tid, ix, keylen);
    if (c->host_staged) {
        c->h_gid.push_back((uint32_t)g);
        c->h_keyoff.push_back(c->h_keys.size());
        c->h_keys.insert(c->h_keys.end(), key, key + keylen);
        c->h_lsn.push_back(lsn);
    }
    if (c->live) {  // a built window: the row goes to the device delta run
        c->app_gid.push_back((uint32_t)g);
        c->app_koff.push_back(c->app_keys.size());
        c->app_keys.insert(c->app_keys.end(), key, key + keylen);
        c->app_lsn.push_back(lsn);
    }
}

// ---------------------------------------------------------------------------
// device window build
// ---------------------------------------------------------------------------
// Row capacity: a whole number of the largest tiles (the joins stage full
// tiles without bounds checks).
static size_t window_cap(size_t n)
{
    const size_t T = kMaxTileRows;
    return std::max<size_t>(T, (n + T - 1) & ~(T - 1));
}

static int window_words(hsc_ctx *c)
{
    int W = 1;
    for (auto &g : c->groups) W = std::max(W, (g.klen + 7) / 8);
    return W;
}

// Sort + dedupe rows staged in d_gid/d_words/d_lsn (n_in rows, stride cap),
// then build group spans, tile maxima and table maxima.
#define HIPCHK_RC(c, call)                  \
    do {                                    \
        const int rc_ = (call);             \
        if (rc_ != HSC_OK) return rc_;      \
    } while (0)

// The window's distinct commit LSNs, sorted (commit ranks of the narrow
// tiles), from the staged rows' LSNs before the key sort moves them: a log
// stream arrives in LSN order (unique = flag + scan + compact); otherwise
// the LSNs are radix-sorted first.
static int build_commits(hsc_ctx *c, size_t n_in)
{
    hipStream_t s = c->stream;
    const size_t cap = c->cap;
    HIPCHK(c, c->d_nzero.ensure(4 * cap));
    HIPCHK(c, hipMemsetAsync(c->d_nzero.p, 0, 4 * cap, s));
    HIPCHK(c, c->d_commits.ensure(8 * n_in));
    uint32_t *flag = c->d_count.as<uint32_t>() + 8;
    HIPCHK(c, check_sorted_u64(c->d_lsn.as<uint64_t>(), n_in, flag, s));
    uint32_t unsorted = 0;
    HIPCHK(c, hipMemcpyAsync(&unsorted, flag, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint64_t *src = c->d_lsn.as<uint64_t>();
    size_t stride = cap;
    if (unsorted) {
        for (auto &b : c->d_ctmp) HIPCHK(c, b.ensure(8 * n_in));
        HIPCHK(c, hipMemcpyAsync(c->d_ctmp[0].p, c->d_lsn.p, 8 * n_in, hipMemcpyDeviceToDevice, s));
        bool alt = false;
        HIPCHK(c, radix_sort_rows(1, n_in, c->d_nzero.as<uint32_t>(), c->d_ctmp[0].as<uint64_t>(),
                                  c->d_ctmp[1].as<uint64_t>(), n_in, c->d_gid2.as<uint32_t>(),
                                  c->d_ctmp[2].as<uint64_t>(), c->d_ctmp[3].as<uint64_t>(),
                                  c->d_scratch.p, c->d_scratch.bytes, &alt, nullptr, s));
        src = (alt ? c->d_ctmp[2] : c->d_ctmp[0]).as<uint64_t>();
        stride = n_in;
        HIPCHK(c, hipMemsetAsync(c->d_nzero.p, 0, 4 * cap, s));
    }
    HIPCHK(c, dedupe_rows(1, n_in, c->d_nzero.as<uint32_t>(), src, src, stride,
                          c->d_gid2.as<uint32_t>(), c->d_commits.as<uint64_t>(),
                          c->d_commits.as<uint64_t>(), n_in, c->d_flags.as<uint32_t>(),
                          c->d_scratch.p, c->d_scratch.bytes, c->d_count.as<uint32_t>() + 12, s));
    // the count (d_count[12]) comes back with the window's own sizes, in
    // device_build's one readback
    return HSC_OK;
}

// Compact codes of the (wide) window w: per-group varying masks, code width
// WC; if WC < W the codes and their tile summaries become the probe view.
static int build_compact(hsc_ctx *c, const WinView &w)
{
    hipStream_t s = c->stream;
    const int W = c->W, ng = (int)c->groups.size();
    const size_t gw = (size_t)ng * W;
    HIPCHK(c, c->d_cmask.ensure(8 * gw));
    HIPCHK(c, c->d_cpat.ensure(8 * gw));
    std::vector<uint64_t> mask(gw);
    std::vector<uint32_t> gs(ng), ge(ng);
    if (c->code_sorted) {
        // the code sort's tables of the same rows (its pattern rows differ,
        // any row of a group serves): copied, not recomputed
        HIPCHK(c, hipMemcpyAsync(c->d_cmask.p, c->d_csmask.p, 8 * gw, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->d_cpat.p, c->d_cspat.p, 8 * gw, hipMemcpyDeviceToDevice, s));
        mask = c->cs_mask;
        for (int g = 0; g < ng; ++g) ge[g] = c->cs_has_rows[g] ? 1 : 0;
    } else {
        HIPCHK(c, compact_masks(w.words, w.stride, w.gid, w.n, W, ng, c->d_gstart.as<uint32_t>(),
                                c->d_gend.as<uint32_t>(), c->d_cmask.as<uint64_t>(),
                                c->d_cpat.as<uint64_t>(), s));
        HIPCHK(c, hipMemcpyAsync(mask.data(), c->d_cmask.p, 8 * gw, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(gs.data(), c->d_gstart.p, 4 * (size_t)ng, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(ge.data(), c->d_gend.p, 4 * (size_t)ng, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    std::vector<uint32_t> bits(ng);
    std::vector<uint64_t> mv(gw * 6);
    int maxbits = 0;
    for (int g = 0; g < ng; ++g) {
        if (ge[g] <= gs[g]) {
            bits[g] = 0xFFFFFFFFu;
            continue;
        }
        int b = 0;
        for (int j = 0; j < W; ++j) {
            b += __builtin_popcountll(mask[(size_t)g * W + j]);
            compress_moves(mask[(size_t)g * W + j], &mv[((size_t)g * W + j) * 6]);
        }
        bits[g] = (uint32_t)b;
        maxbits = std::max(maxbits, b);
    }
    const int WC = maxbits / 64 + 1;  // >= 1 spare bit: all-ones is above every code
    c->ct_maxbits = maxbits;
    if (WC >= W || WC > kMaxCompactWords) return HSC_OK;
    HIPCHK(c, c->d_cmv.ensure(8 * gw * 6));
    // bits[g] then wlen[g] (words inside the group's key length) in one upload
    bits.resize(2 * (size_t)ng);
    for (int g = 0; g < ng; ++g) bits[ng + g] = (uint32_t)std::min(W, (c->groups[g].klen + 7) / 8);
    HIPCHK(c, c->d_cbits.ensure(8 * (size_t)ng));
    HIPCHK(c, hipMemcpyAsync(c->d_cmv.p, mv.data(), 8 * gw * 6, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_cbits.p, bits.data(), 8 * (size_t)ng, hipMemcpyHostToDevice, s));
    c->ct = CompactTables{};
    c->ct.mask = c->d_cmask.as<uint64_t>();
    c->ct.pat = c->d_cpat.as<uint64_t>();
    c->ct.mv = c->d_cmv.as<uint64_t>();
    c->ct.bits = c->d_cbits.as<uint32_t>();
    c->ct.wlen = c->d_cbits.as<uint32_t>() + ng;
    c->ct.W = W;
    c->ct.WC = WC;
    c->ct.ng = ng;
    HIPCHK(c, c->d_cwords.ensure(8 * (size_t)WC * c->cap));
    if (!(c->code_sorted && c->cs_codes_wc == WC))  // (the code sort's unpack wrote them)
        HIPCHK(c, compact_rows(w.words, w.stride, w.gid, w.n, c->ct, c->d_cwords.as<uint64_t>(), s));
    WinView &v = c->wc;
    v = w;
    v.words = c->d_cwords.as<uint64_t>();
    v.W = WC;
    v.compact = 1;
    v.log2T = std::min(tile_log2(WC), kCTLog2);  // the compact tiles share these tiles' maxima
    v.ntiles = (uint32_t)((c->n + ((size_t)1 << v.log2T) - 1) >> v.log2T);
    v.levels = 0;
    while (((size_t)1 << v.levels) <= v.ntiles) v.levels++;
    HIPCHK(c, c->d_ctmax.ensure(8 * (size_t)std::max(1, v.levels) * std::max<uint32_t>(1, v.ntiles)));
    HIPCHK(c, c->d_csp_g.ensure(4 * (size_t)std::max<uint32_t>(1, v.ntiles)));
    HIPCHK(c, c->d_csp_w.ensure(8 * (size_t)WC * std::max<uint32_t>(1, v.ntiles)));
    v.tmax = c->d_ctmax.as<uint64_t>();
    v.sp_g = c->d_csp_g.as<uint32_t>();
    v.sp_w = c->d_csp_w.as<uint64_t>();
    HIPCHK(c, build_summaries(v, c->d_gstart.as<uint32_t>(), c->d_gend.as<uint32_t>(), ng,
                              c->d_ctmax.as<uint64_t>(), nullptr, nullptr, c->d_csp_g.as<uint32_t>(),
                              c->d_csp_w.as<uint64_t>(), s));
    v.gstart = c->d_gstart.as<uint32_t>();
    v.gend = c->d_gend.as<uint32_t>();
    c->compact = true;
    return HSC_OK;
}

// Compact tiles over the compact view c->wc (hsc_ctiles.hip): keys gid ||
// code of WG <= 3 words, 32-bit commit times.  Needs the view's 2048-row
// tiles, commits spanning < 2^32 of log, a tile count the locate's bucket
// table and LDS take; otherwise dense batches stay on the wide pipeline.
static int build_ctiles(hsc_ctx *c)
{
    c->cph_nb = 0;
    const WinView &v = c->wc;
    const int ng = (int)c->groups.size();
    int gb = 0;
    while (gb < 32 && ((size_t)1 << gb) < (size_t)ng) gb++;
    const int WG = (c->ct_maxbits + gb + 1 + 63) / 64;  // a spare bit: ~0 is above every key
    if (v.log2T != kCTLog2 || WG > 3 || WG < c->ct.WC || !c->has_commits ||
        c->commit_span[1] - c->commit_span[0] > kLsn32MaxSpan)
        return HSC_OK;
    CTiles &ct = c->ctv;
    ct = CTiles{};
    ct.n = (uint32_t)c->n;
    ct.ntiles = v.ntiles;
    ct.len = (size_t)v.ntiles << kCTLog2;
    ct.WG = WG;
    ct.WC = c->ct.WC;
    ct.gb = gb;
    ct.rank_base = c->commit_span[0];
    ct.trad_m = narrow_trad_buckets(ct.ntiles, c->paths & HSC_PATH_TILE_DIR);
    if (ct.trad_m == 0 || ct.ntiles > (uint32_t)kHistCap || ctiles_locate_lds(ct) > 65536)
        return HSC_OK;
    hipStream_t s = c->stream;
    HIPCHK(c, c->d_ckey.ensure(8 * (size_t)WG * ct.len));
    HIPCHK(c, c->d_crank.ensure(4 * ct.len));
    HIPCHK(c, c->d_cfirst.ensure(8 * (size_t)WG * ct.ntiles));
    HIPCHK(c, c->d_crel.ensure(8 * (size_t)ct.ntiles));
    HIPCHK(c, c->d_ctrad.ensure(4 * ((size_t)ct.trad_m + 2)));
    HIPCHK(c, c->d_ctb.ensure(4 * (size_t)kTBS * ct.ntiles));
    ct.tb = c->d_ctb.as<uint32_t>();
    ct.key = c->d_ckey.as<uint64_t>();
    ct.rank = c->d_crank.as<uint32_t>();
    ct.first = c->d_cfirst.as<uint64_t>();
    ct.trad = c->d_ctrad.as<uint32_t>();
    HIPCHK(c, ctiles_build(v.words, v.stride, ct.WC, v.gid, v.lsn, ct, c->d_ckey.as<uint64_t>(),
                           c->d_crank.as<uint32_t>(), c->d_cfirst.as<uint64_t>(),
                           c->d_crel.as<uint64_t>(), c->d_ctrad.as<uint32_t>(),
                           c->d_ctb.as<uint32_t>(), s));
    // the point index (hsc_compact.hip PointHash): points are answered by the
    // bound kernel (HSC_PATH_NO_CT_POINTS: they take join records, the r05 path)
    if (!(c->paths & HSC_PATH_NO_CT_POINTS) && ct.n) {
        const uint64_t nb = point_hash_buckets(ct.n);
        void *old = c->d_cph.p;
        HIPCHK(c, c->d_cph.ensure(128 * nb));
        // a rebuild over the same buffer only bumps the epoch (its entries
        // read as empty); a new buffer -- or 2^24 builds -- is cleared once
        const bool clear = c->d_cph.p != old || c->cph_ep == 0 || c->cph_ep >= (1u << 24) - 1;
        c->cph_ep = clear ? 1 : c->cph_ep + 1;
        HIPCHK(c, point_hash_build(ct, c->d_cph.as<uint64_t>(), nb, c->cph_ep, clear, s));
        c->cph_nb = nb;
    }
    HIPCHK(c, hipMemcpyAsync(&ct.base0, c->d_cfirst.p, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (getenv("HSC_CT_STATS")) {  // diagnostics: fullest buckets of the locate's and the join's tables
        std::vector<uint32_t> t(ct.trad_m + 2);
        std::vector<uint32_t> tb((size_t)kTBS * ct.ntiles);
        HIPCHK(c, hipMemcpy(t.data(), c->d_ctrad.p, 4 * t.size(), hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(tb.data(), c->d_ctb.p, 4 * tb.size(), hipMemcpyDeviceToHost));
        uint32_t w = 0;
        for (uint32_t k = 0; k < ct.trad_m; ++k) w = std::max(w, t[k + 1] - t[k]);
        std::vector<uint32_t> fb;
        for (uint32_t x = 0; x < ct.ntiles; ++x) {
            uint32_t f = 0;
            for (int k = 0; k < kTB; ++k)
                f = std::max<uint32_t>(f, (tb[(size_t)x * kTBS + k] >> 16) - (tb[(size_t)x * kTBS + k] & 0xFFFF));
            fb.push_back(f);
        }
        std::sort(fb.begin(), fb.end());
        fprintf(stderr, "[ct] tiles %u, locate buckets %u fullest %u; join fullest bucket per tile p50 %u p90 %u max %u\n",
                ct.ntiles, ct.trad_m, w, fb[fb.size() / 2], fb[fb.size() * 9 / 10], fb.back());
    }
    c->ctiles = true;
    return HSC_OK;
}

// Narrow tiles' bucket table: linear buckets (uniform keys) or log buckets
// (keys dense near the window's first, e.g. Zipf hot keys) -- whichever mode's
// fullest bucket holds fewer tiles (the locate's in-bucket search is
// log2 of it).
static int narrow_trad_pick(hsc_ctx *c)
{
    const uint32_t m = c->trad_m;
    std::vector<uint32_t> a(m + 2), b(m + 2);
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (the tables come from c->stream, a non-blocking stream)
    HIPCHK(c, hipMemcpy(a.data(), c->d_trad.p, 4 * a.size(), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(b.data(), c->d_trad2.p, 4 * b.size(), hipMemcpyDeviceToHost));
    auto fullest = [m](const std::vector<uint32_t> &t) {
        uint32_t w = 0;
        for (uint32_t k = 0; k < m; ++k) w = std::max(w, t[k + 1] - t[k]);
        return w;
    };
    const bool log = fullest(b) < fullest(a);
    if (log) std::swap(c->d_trad, c->d_trad2);
    c->trad_log = log;
    return HSC_OK;
}

// HSC_BUILD_TRACE=1: wall time of each stage of a window build on stderr
// (every stamp synchronises the stream first; diagnostics only).
struct BuildTrace {
    bool on;
    hipStream_t s;
    std::chrono::steady_clock::time_point t;
    std::string out;
    explicit BuildTrace(hipStream_t s_) : on(getenv("HSC_BUILD_TRACE") != nullptr), s(s_)
    {
        if (on) (void)hipStreamSynchronize(s);
        t = std::chrono::steady_clock::now();
    }
    void stamp(const char *what)
    {
        if (!on) return;
        (void)hipStreamSynchronize(s);
        const auto n = std::chrono::steady_clock::now();
        char b[64];
        snprintf(b, sizeof b, " %s=%.0f", what, std::chrono::duration<double, std::micro>(n - t).count());
        out += b;
        t = n;
    }
    ~BuildTrace()
    {
        if (on && !out.empty()) fprintf(stderr, "[build us]%s\n", out.c_str());
    }
};

// Sort the n_in input rows (d_gid / d_words / d_lsn) by their compact codes
// into d_gid2 / d_words2 / d_lsn2 (hsc_csort.hip), when the keys do not fit
// the packed sort but every group's varying bits fit 3 code words.  *done =
// false: not applicable (the caller takes the whole-row radix sort).
static int code_sort(hsc_ctx *c, size_t n_in, bool *done)
{
    *done = false;
    const int W = c->W, ng = (int)c->groups.size();
    const size_t gw = (size_t)ng * W;
    if (W < 2 || ng == 0 || n_in == 0 || n_in >= 0xFFFFFFFFull || 16 * gw > kCsVaryLds) return HSC_OK;
    hipStream_t s = c->stream;
    HIPCHK(c, c->d_csrep.ensure(4 * (size_t)ng));
    HIPCHK(c, c->d_csmask.ensure(8 * gw));
    HIPCHK(c, c->d_cspat.ensure(8 * gw));
    HIPCHK(c, compact_masks_unsorted(c->d_words.as<uint64_t>(), c->cap, c->d_gid.as<uint32_t>(),
                                     (uint32_t)n_in, W, ng, c->d_csrep.as<uint32_t>(),
                                     c->d_csmask.as<uint64_t>(), c->d_cspat.as<uint64_t>(), s));
    std::vector<uint64_t> mask(gw);
    std::vector<uint32_t> rep(ng);
    HIPCHK(c, hipMemcpyAsync(mask.data(), c->d_csmask.p, 8 * gw, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(rep.data(), c->d_csrep.p, 4 * (size_t)ng, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    // (host sources of the uploads below: the context's, alive past the
    // asynchronous copies)
    std::vector<uint32_t> &bits = c->cs_bits_h;
    std::vector<uint64_t> &mv = c->cs_mv_h;
    bits.assign(2 * (size_t)ng, 0);
    mv.assign(gw * 6, 0);
    int maxbits = 0;
    c->cs_mask = mask;  // build_compact takes these tables over
    c->cs_has_rows.assign(ng, 0);
    for (int g = 0; g < ng; ++g) c->cs_has_rows[g] = rep[g] != 0xFFFFFFFFu;
    for (int g = 0; g < ng; ++g) {
        int b = 0;
        for (int j = 0; j < W; ++j) {
            b += __builtin_popcountll(mask[(size_t)g * W + j]);
            compress_moves(mask[(size_t)g * W + j], &mv[((size_t)g * W + j) * 6]);
        }
        bits[g] = rep[g] == 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)b;
        bits[ng + g] = (uint32_t)std::min(W, (c->groups[g].klen + 7) / 8);
        maxbits = std::max(maxbits, b);
    }
    const int WC = maxbits / 64 + 1;
    if (WC > 3) return HSC_OK;
    HIPCHK(c, c->d_csmv.ensure(8 * gw * 6));
    HIPCHK(c, c->d_csbits.ensure(8 * (size_t)ng));
    HIPCHK(c, hipMemcpyAsync(c->d_csmv.p, mv.data(), 8 * gw * 6, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_csbits.p, bits.data(), 8 * (size_t)ng, hipMemcpyHostToDevice, s));
    CompactTables t{};
    t.mask = c->d_csmask.as<uint64_t>();
    t.pat = c->d_cspat.as<uint64_t>();
    t.mv = c->d_csmv.as<uint64_t>();
    t.bits = c->d_csbits.as<uint32_t>();
    t.wlen = c->d_csbits.as<uint32_t>() + ng;
    t.W = W;
    t.WC = WC;
    t.ng = ng;
    const int KW = WC + 1;
    // (the free key buffer becomes d_lsn below: at least the window's capacity)
    for (auto &b : c->d_cskeys) HIPCHK(c, b.ensure(8 * std::max((size_t)KW * n_in, c->cap)));
    HIPCHK(c, compact_sort_keys(c->d_words.as<uint64_t>(), c->cap, c->d_gid.as<uint32_t>(), (uint32_t)n_in,
                                t, c->d_cskeys[0].as<uint64_t>(), s));
    uint64_t *sorted = nullptr;
    HIPCHK(c, c->d_cssplit.ensure(4 * code_sort_split_words(n_in)));
    HIPCHK(c, code_keys_sort(c->d_cskeys[0].as<uint64_t>(), c->d_cskeys[1].as<uint64_t>(),
                             c->d_cssplit.as<uint32_t>(), n_in, KW, s,
                             &sorted));
    // every version, key-sorted, into d_*2; the distinct rows into d_gid /
    // d_words (the unpack reads only the input LSNs) and the free key
    // buffer, which becomes d_lsn
    DBuf &kfree = sorted == c->d_cskeys[0].as<uint64_t>() ? c->d_cskeys[1] : c->d_cskeys[0];
    // the distinct rows' codes are the compact tiles' row codes (build_compact
    // uses the same masks and width): written here, not recomputed from the
    // unpacked words
    uint64_t *codes = nullptr;
    if (WC < W) {
        HIPCHK(c, c->d_cwords.ensure(8 * (size_t)WC * c->cap));
        codes = c->d_cwords.as<uint64_t>();
    }
    HIPCHK(c, compact_unpack_dedupe(sorted, n_in, t, c->d_lsn.as<uint64_t>(), c->d_gid2.as<uint32_t>(),
                                    c->d_words2.as<uint64_t>(), c->d_lsn2.as<uint64_t>(), c->cap,
                                    c->d_gid.as<uint32_t>(), c->d_words.as<uint64_t>(),
                                    kfree.as<uint64_t>(), c->cap, c->d_count.as<uint32_t>(),
                                    c->d_scratch.as<uint32_t>(), codes, s));
    std::swap(c->d_lsn, kfree);
    c->cs_codes_wc = codes ? WC : 0;
    *done = true;
    return HSC_OK;
}

static int device_build(hsc_ctx *c, size_t n_in)
{
    BuildTrace bt(c->stream);
    HIPCHK(c, wait_lanes(c));
    hipStream_t s = c->stream;
    const int W = c->W;
    const size_t cap = c->cap;
    HIPCHK(c, c->d_gid2.ensure(cap * 4));
    HIPCHK(c, c->d_words2.ensure(cap * 8 * W));
    HIPCHK(c, c->d_lsn2.ensure(cap * 8));
    HIPCHK(c, c->d_flags.ensure(cap * 4 + 64));
    // packed-key sort (hsc_ingest.hip) unless turned off (HSC_PATH_NO_PACKED_SORT)
    // or the key has more words than it takes
    const bool try_packed = W <= kPackMaxWords && n_in > 0 && !(c->paths & HSC_PATH_NO_PACKED_SORT);
    size_t scratch = std::max(radix_scratch_bytes(n_in, W), scan_scratch_bytes(n_in) + 64);
    if (try_packed) {
        // (sized by the capacity, not this build's rows: the one-sweep status
        // region grows with the rows, and a scratch that grew on a merge of a
        // few more rows would reallocate -- a hipFree's sync -- inside a check)
        scratch = std::max(scratch, packed_scratch_bytes(cap));
        for (auto &b : c->d_pk) HIPCHK(c, b.ensure(8 * cap));
    }
    HIPCHK(c, c->d_scratch.ensure(scratch));
    HIPCHK(c, c->d_count.ensure(256));
    bt.stamp("alloc");

    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(c, hipEventCreate(&e0));
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventRecord(e0, s));
    // varying key bits and the LSN span in one pass; the distinct commit list
    // only when snapshot ranks need its directory (a window spanning >= 2^32
    // of log): otherwise rows carry lsn - oldest + 1
    uint64_t vary[kMaxWords + 1], span[2], lvary = 0;
    HIPCHK(c, vary_mask_rows(W, n_in, c->d_gid.as<uint32_t>(), c->d_words.as<uint64_t>(), cap,
                             c->d_scratch.p, vary, s, c->d_lsn.as<uint64_t>(), span, &lvary));
    bt.stamp("vary");
    const bool commits = c->layout != HSC_LAYOUT_WIDE && n_in > 0;
    const bool rank_dir = commits && span[1] - span[0] > kLsn32MaxSpan;
    c->has_commits = commits;
    c->ncommit = 0;
    if (commits) memcpy(c->commit_span, span, 16);
    if (rank_dir) HIPCHK_RC(c, build_commits(c, n_in));
    bt.stamp("commits");
    PackPlan plan;
    // (the LSNs' varying bits beside the key's: the min LSN is a row's, so its
    // bits outside them are every row's)
    const uint64_t lbits[2] = {lvary, span[0]};
    c->packed_sort = try_packed && packed_plan(W, n_in, vary, &plan, true, lbits);
    // too many varying bits for the packed sort: by compact codes if they fit
    bool code_sorted = false;
    c->cs_codes_wc = 0;
    if (!c->packed_sort && try_packed) HIPCHK_RC(c, code_sort(c, n_in, &code_sorted));
    c->code_sorted = code_sorted;
    if (c->packed_sort) {
        // every version, key-sorted, into d_*2; the distinct rows straight from
        // the unpack into d_gid / d_words (in place) and a free key buffer,
        // which becomes d_lsn (the input LSNs are gathered while it is written)
        uint64_t *dl = nullptr;
        HIPCHK(c, packed_sort_dedupe(plan, n_in, c->d_gid.as<uint32_t>(), c->d_words.as<uint64_t>(),
                                     c->d_lsn.as<uint64_t>(), cap, c->d_pk[0].as<uint64_t>(),
                                     c->d_pk[1].as<uint64_t>(), c->d_gid2.as<uint32_t>(),
                                     c->d_words2.as<uint64_t>(), c->d_lsn2.as<uint64_t>(), cap,
                                     c->d_gid.as<uint32_t>(), c->d_words.as<uint64_t>(), cap, &dl,
                                     c->d_count.as<uint32_t>(), c->d_scratch.p, c->d_scratch.bytes, s,
                                     c->d_count.as<uint32_t>() + 20));
        if (dl == c->d_pk[0].p)
            std::swap(c->d_lsn, c->d_pk[0]);
        else if (dl == c->d_pk[1].p)
            std::swap(c->d_lsn, c->d_pk[1]);
        bt.stamp("sort");
    } else if (code_sorted) {
        bt.stamp("sort");  // every version in d_*2, the distinct rows in d_* (code_sort)
    } else {
        bool in_alt = false;
        HIPCHK(c, radix_sort_known(W, n_in, c->d_gid.as<uint32_t>(), c->d_words.as<uint64_t>(),
                                   c->d_lsn.as<uint64_t>(), cap, c->d_gid2.as<uint32_t>(),
                                   c->d_words2.as<uint64_t>(), c->d_lsn2.as<uint64_t>(),
                                   c->d_scratch.p, c->d_scratch.bytes, &in_alt, vary, s));
        bt.stamp("sort");
        // dedupe from wherever the sort left the rows into the other buffer set
        DBuf *sg = in_alt ? &c->d_gid2 : &c->d_gid, *sw = in_alt ? &c->d_words2 : &c->d_words,
             *sl = in_alt ? &c->d_lsn2 : &c->d_lsn;
        DBuf *dg = in_alt ? &c->d_gid : &c->d_gid2, *dw = in_alt ? &c->d_words : &c->d_words2,
             *dl = in_alt ? &c->d_lsn : &c->d_lsn2;
        HIPCHK(c, dedupe_rows(W, n_in, sg->as<uint32_t>(), sw->as<uint64_t>(), sl->as<uint64_t>(), cap,
                              dg->as<uint32_t>(), dw->as<uint64_t>(), dl->as<uint64_t>(), cap,
                              c->d_flags.as<uint32_t>(), c->d_scratch.p, c->d_scratch.bytes,
                              c->d_count.as<uint32_t>(), s));
        if (!in_alt) {  // final rows must live in d_gid/d_words/d_lsn
            std::swap(c->d_gid, c->d_gid2);
            std::swap(c->d_words, c->d_words2);
            std::swap(c->d_lsn, c->d_lsn2);
        }
    }
    // one readback for the sizes the host plans with: distinct rows, commits,
    // the commit span and the window's end rows (all computed on the device)
    HIPCHK(c, c->d_nbase.ensure(16 * ((size_t)W + 1)));
    std::vector<uint64_t> ends(2 * ((size_t)W + 1), 0);
    uint32_t hc[24] = {0};
    if (commits) {
        WinView wc{};
        wc.words = c->d_words.as<uint64_t>();
        wc.stride = cap;
        wc.gid = c->d_gid.as<uint32_t>();
        wc.W = W;
        HIPCHK(c, narrow_end_rows(wc, c->d_count.as<uint32_t>(), c->d_nbase.as<uint64_t>(), s));
        HIPCHK(c, hipMemcpyAsync(ends.data(), c->d_nbase.p, 8 * ends.size(), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, hipMemcpyAsync(hc, c->d_count.p, sizeof hc, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    bt.stamp("dedupe");
    // (hc[20]: the packed sort's one-sweep stall flag -- never expected)
    if (c->packed_sort && hc[20]) return fail(c, HSC_EDEVICE, "window sort: a tile's look-back stalled");
    const uint32_t nu = hc[0];
    if (rank_dir) c->ncommit = hc[12];
    c->n = n_in ? nu : 0;
    c->n_all = n_in;  // every version, key-sorted, stays in d_gid2 / d_words2 / d_lsn2
    // narrow layout if the whole window fits 62-bit codes (hsc_narrow.hip)
    c->narrow = false;
    c->ncomp = false;
    c->lw = W;
    c->tz = 63;
    if (c->layout != HSC_LAYOUT_WIDE && c->n > 0) {
        // vary[j]: bits of word j (j < W) / of gid (j == W) that differ
        // between rows; limb 0 = gid, limb j + 1 = word j
        for (int l = W; l >= 0; --l) {
            const uint64_t m = l ? vary[l - 1] : vary[W];
            if (m) {
                c->lw = l;
                c->tz = __builtin_ctzll(m);
                break;
            }
        }
        c->narrow = narrow_span_fits(W, c->lw, c->tz, ends.data(), ends.data() + W + 1);
        // composite keys whose varying bits sit far apart but total <= 62:
        // the narrow index over compressed codes (hsc_narrow.hip cnarrow_bound)
        int vb = 0;
        for (int l = 0; l <= W; ++l) vb += __builtin_popcountll(l ? vary[l - 1] : vary[W]);
        c->ncomp = !c->narrow && vb <= 62 && !(c->paths & HSC_PATH_NO_COMP_NARROW);
        if (c->ncomp) {
            std::vector<uint64_t> cm(8 * (size_t)(W + 1), 0);
            uint64_t c0 = 0;
            for (int l = 0; l <= W; ++l) {
                const uint64_t m = l ? vary[l - 1] : vary[W], r0 = ends[l];  // ends[0] = gid, ends[1 + j] = word j
                cm[8 * l] = m;
                cm[8 * l + 1] = r0;
                compress_moves(m, &cm[8 * l + 2]);
                const int cnt = __builtin_popcountll(m);
                if (cnt) c0 = (cnt >= 64 ? 0 : c0 << cnt) | host_compress(r0, m);
            }
            c->nc0 = c0;
            HIPCHK(c, c->d_ncmeta.ensure(8 * cm.size()));
            HIPCHK(c, hipMemcpyAsync(c->d_ncmeta.p, cm.data(), 8 * cm.size(), hipMemcpyHostToDevice, s));
            c->narrow = true;
        }
    }
    c->log2T = tile_log2(W);
    c->ntiles = (uint32_t)((c->n + ((size_t)1 << c->log2T) - 1) >> c->log2T);
    c->levels = 0;
    while (((size_t)1 << c->levels) <= c->ntiles) c->levels++;
    const int ng = (int)c->groups.size();
    const int nt = (int)c->table_names.size();
    c->ng_built = (size_t)ng;
    HIPCHK(c, c->d_gstart.ensure(4 * (size_t)std::max(ng, 1)));
    HIPCHK(c, c->d_gend.ensure(4 * (size_t)std::max(ng, 1)));
    HIPCHK(c, c->d_tmax.ensure(8 * (size_t)std::max(1, c->levels) * std::max<uint32_t>(1, c->ntiles)));
    HIPCHK(c, c->d_table_max.ensure(8 * (size_t)std::max(nt, 1)));
    HIPCHK(c, c->d_group_table.ensure(4 * (size_t)std::max(ng, 1)));
    HIPCHK(c, c->d_sp_g.ensure(4 * (size_t)std::max<uint32_t>(1, c->ntiles)));
    HIPCHK(c, c->d_sp_w.ensure(8 * (size_t)W * std::max<uint32_t>(1, c->ntiles)));
    std::vector<uint32_t> gt(std::max(ng, 1), 0);
    for (int g = 0; g < ng; ++g) gt[g] = (uint32_t)c->groups[g].tid;
    HIPCHK(c, hipMemcpyAsync(c->d_group_table.p, gt.data(), 4 * gt.size(), hipMemcpyHostToDevice, s));
    std::vector<uint64_t> tm(std::max(nt, 1), 0);
    for (int t = 0; t < nt; ++t) tm[t] = c->h_table_max[t];
    HIPCHK(c, hipMemcpyAsync(c->d_table_max.p, tm.data(), 8 * tm.size(), hipMemcpyHostToDevice, s));
    c->nt_dev = (uint32_t)nt;
    WinView w{};
    w.words = c->d_words.as<uint64_t>();
    w.stride = cap;
    w.lsn = c->d_lsn.as<uint64_t>();
    w.gid = c->d_gid.as<uint32_t>();
    w.tmax = c->d_tmax.as<uint64_t>();
    w.n = (uint32_t)c->n;
    w.ntiles = c->ntiles;
    w.W = W;
    w.log2T = c->log2T;
    w.levels = c->levels;
    // the narrow index before the summaries: its level-1 LSN maxima (one per
    // 16 rows) give the window's tile maxima, read instead of every row's LSN
    // (HSC_NTMAX_REBUILD=1: from the LSNs, an A/B)
    bool tiles_on = false, tiles_fused = false;
    uint32_t *tiles_flag = c->d_count.as<uint32_t>() + 4;
    if (c->narrow) {
        // level sizes: level 0 = n + 1 rounded up to whole tiles (at least one
        // pad; the tile pipeline stages whole tiles), then roundup16(len / 16)
        // until one 16-entry block
        NarrowView &nv = c->nv;
        nv = NarrowView{};
        uint32_t len = (uint32_t)((c->n + 1 + kMaxTileRows - 1) & ~(size_t)(kMaxTileRows - 1));
        uint64_t off = 0;
        int L = 0;
        for (;;) {
            if (L == kMaxLevels) return fail(c, HSC_EINVAL, "window too large for the narrow index");
            nv.off[L] = off;
            nv.len[L] = len;
            off += len;
            ++L;
            if (len <= 16) break;
            len = ((len / 16) + 15) & ~15u;
        }
        nv.levels = L;
        nv.lds_from = L - 1;
        nv.lds_entries = nv.len[L - 1];
        while (nv.lds_from > 0 && nv.lds_entries + nv.len[nv.lds_from - 1] <= 4096)
            nv.lds_entries += nv.len[--nv.lds_from];
        HIPCHK(c, c->d_nkeys.ensure(8 * (size_t)off));
        HIPCHK(c, c->d_nmaxs.ensure(8 * (size_t)off));
        nv.keys = c->d_nkeys.as<uint64_t>();
        nv.maxs = c->d_nmaxs.as<uint64_t>();
        nv.base = c->d_nbase.as<uint64_t>();  // row 0 limbs (narrow_end_rows)
        nv.W = W;
        nv.lw = c->lw;
        nv.tz = c->tz;
        nv.comp = c->ncomp ? 1 : 0;
        nv.cmeta = c->d_ncmeta.as<uint64_t>();
        nv.c0 = c->nc0;
        nv.n = (uint32_t)c->n;
        // the narrow tiles (below) when their 4096-row tiles fit the locate's
        // histogram: key32 -- and rank32 in lsn32 mode -- from the level pass
        const int wn_log2T = tile_log2(1);
        const uint32_t wn_ntiles = (uint32_t)((c->n + ((size_t)1 << wn_log2T) - 1) >> wn_log2T);
        tiles_on = wn_log2T == 12 && wn_ntiles <= (uint32_t)kHistCap && c->has_commits;
        const bool tiles_lsn32 = c->commit_span[1] - c->commit_span[0] <= kLsn32MaxSpan;
        tiles_fused = tiles_on && narrow_level01_tiles(nv);
        if (tiles_fused) {
            HIPCHK(c, c->d_key32.ensure(4 * (size_t)nv.len[0]));
            HIPCHK(c, c->d_rank32.ensure(4 * (size_t)nv.len[0]));
            HIPCHK(c, narrow_build(w, nv, s, c->d_key32.as<uint32_t>(),
                                   tiles_lsn32 ? c->d_rank32.as<uint32_t>() : nullptr, c->commit_span[0],
                                   tiles_flag));
        } else {
            HIPCHK(c, narrow_build(w, nv, s));
        }
        bt.stamp("narrow");
    }
    static const bool tmax_rows = getenv("HSC_NTMAX_REBUILD") != nullptr;
    TmaxFrom wfrom;
    if (c->narrow && !tmax_rows && c->nv.levels >= 2 && c->log2T >= 4) wfrom.lsn16 = c->nv.maxs + c->nv.off[1];
    HIPCHK(c, build_summaries(w, c->d_gstart.as<uint32_t>(), c->d_gend.as<uint32_t>(), ng,
                              c->d_tmax.as<uint64_t>(), c->d_group_table.as<uint32_t>(),
                              c->d_table_max.as<uint64_t>(), c->d_sp_g.as<uint32_t>(),
                              c->d_sp_w.as<uint64_t>(), s, wfrom));
    bt.stamp("summaries");
    c->compact = false;
    uint32_t wide32 = 1;   // narrow tiles: a tile spans >= 2^32 codes (device flag)
    bool tiles32 = false;
    c->ctiles = false;
    if (!c->narrow && (c->layout == HSC_LAYOUT_AUTO || c->layout == HSC_LAYOUT_COMPACT_WIDE) &&
        c->n > 0 && W > 1 && ng > 0) {
        HIPCHK_RC(c, build_compact(c, w));
        if (c->compact) HIPCHK_RC(c, build_ctiles(c));
        bt.stamp("compact");
    }
    if (c->narrow) {
        NarrowView &nv = c->nv;
        // one-word tile view of the codes: rows (gid 0, key64), lsn
        WinView &wn = c->wn;
        wn = WinView{};
        wn.words = nv.keys;
        wn.stride = nv.len[0];
        wn.lsn = nv.maxs;
        wn.n = (uint32_t)c->n;
        wn.W = 1;
        wn.log2T = tile_log2(1);
        wn.ntiles = (uint32_t)((c->n + ((size_t)1 << wn.log2T) - 1) >> wn.log2T);
        wn.levels = 0;
        while (((size_t)1 << wn.levels) <= wn.ntiles) wn.levels++;
        HIPCHK(c, c->d_nzero.ensure(4 * (size_t)nv.len[0]));
        HIPCHK(c, hipMemsetAsync(c->d_nzero.p, 0, 4 * (size_t)nv.len[0], s));
        HIPCHK(c, c->d_ntmax.ensure(8 * (size_t)wn.levels * wn.ntiles));
        HIPCHK(c, c->d_nsp_g.ensure(4 * (size_t)wn.ntiles));
        HIPCHK(c, c->d_nsp_w.ensure(8 * (size_t)wn.ntiles));
        HIPCHK(c, c->d_ngs.ensure(16));
        wn.gid = c->d_nzero.as<uint32_t>();
        wn.tmax = c->d_ntmax.as<uint64_t>();
        // (the window's LSNs over tiles as long or twice as long as the
        // window's: its sparse table folded, HSC_NTMAX_REBUILD=1 rebuilds it
        // from the LSNs, an A/B)
        static const bool ntmax_rebuild = getenv("HSC_NTMAX_REBUILD") != nullptr;
        TmaxFrom from;
        const int tsh = wn.log2T - c->log2T;
        if (!ntmax_rebuild && (tsh == 0 || tsh == 1) && wn.ntiles > 0 && c->ntiles > 0 && c->levels >= wn.levels)
            from = TmaxFrom{c->d_tmax.as<uint64_t>(), c->ntiles, tsh};
        HIPCHK(c, build_summaries(wn, c->d_ngs.as<uint32_t>(), c->d_ngs.as<uint32_t>() + 1, 1,
                                  c->d_ntmax.as<uint64_t>(), nullptr, nullptr,
                                  c->d_nsp_g.as<uint32_t>(), c->d_nsp_w.as<uint64_t>(), s, from));
        wn.gstart = c->d_ngs.as<uint32_t>();
        wn.gend = c->d_ngs.as<uint32_t>() + 1;
        wn.sp_g = c->d_nsp_g.as<uint32_t>();
        wn.sp_w = c->d_nsp_w.as<uint64_t>();
        // 8-byte tile rows when every 4096-row tile spans < 2^32 codes
        c->ntiles32 = false;
        c->trad_m = 0;
        bt.stamp("codes");
        if (tiles_on) {
            // commit span: rank-free rows (lsn - oldest commit + 1) when it fits 32 bits
            const uint64_t *span = c->commit_span;
            c->rank_lsn32 = span[1] - span[0] <= kLsn32MaxSpan;
            c->rank_base = span[0];
            c->cdir = Dir16{};
            if (!c->rank_lsn32)
                HIPCHK(c, dir16_build(c->d_commits.as<uint64_t>(), c->ncommit, c->d_cdir, c->cdir,
                                      narrow_tiles_dir_lds(), s));
            HIPCHK(c, dir16_build(wn.sp_w, wn.ntiles, c->d_tdir, c->tdir, narrow_tiles_dir_lds(), s));
            c->trad_m = narrow_trad_buckets(wn.ntiles, c->paths & HSC_PATH_TILE_DIR);
            if (c->trad_m) {
                HIPCHK(c, c->d_trad.ensure(4 * ((size_t)c->trad_m + 2)));
                HIPCHK(c, narrow_trad_build(wn.sp_w, wn.ntiles, c->trad_m, c->d_trad.as<uint32_t>(), s));
                if (c->trad_m >= 64) {  // the log-mode table too; picked after the build's sync
                    HIPCHK(c, c->d_trad2.ensure(4 * ((size_t)c->trad_m + 2)));
                    HIPCHK(c, narrow_trad_build(wn.sp_w, wn.ntiles, c->trad_m,
                                                c->d_trad2.as<uint32_t>(), s, 1));
                }
            }
            HIPCHK(c, c->d_key32.ensure(4 * (size_t)nv.len[0]));
            HIPCHK(c, c->d_rank32.ensure(4 * (size_t)nv.len[0]));
            // (fused: key32 and the flag are written, the ranks too in lsn32 mode)
            HIPCHK(c, narrow_tiles_build(nv.keys, c->d_lsn.as<uint64_t>(), (uint32_t)c->n, nv.len[0],
                                         c->cdir, c->rank_lsn32, c->rank_base,
                                         c->d_key32.as<uint32_t>(), c->d_rank32.as<uint32_t>(),
                                         tiles_fused ? nullptr : tiles_flag, s));
            HIPCHK(c, hipMemcpyAsync(&wide32, tiles_flag, 4, hipMemcpyDeviceToHost, s));  // read below
            tiles32 = true;
        }
    }
    HIPCHK(c, hipEventRecord(e1, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (tiles32) c->ntiles32 = wide32 == 0;
    bt.stamp("tiles");
    if (c->narrow && c->trad_m >= 64) HIPCHK_RC(c, narrow_trad_pick(c));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    c->last.ingest_ms = ms;
    c->last.tiles = c->ntiles;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // table maxima back to the host (device ingest computes them on the GPU)
    if (nt > 0) {
        HIPCHK(c, hipMemcpy(tm.data(), c->d_table_max.p, 8 * (size_t)nt, hipMemcpyDeviceToHost));
        for (int t = 0; t < nt; ++t) c->h_table_max[t] = std::max(c->h_table_max[t], tm[t]);
    }
    bt.stamp("finish");
    c->dirty = false;
    c->live = true;
    c->merge_pending = false;
    c->dn = 0;  // every appended row is in the rebuilt window
    c->app_gid.clear(), c->app_keys.clear(), c->app_koff.clear(), c->app_lsn.clear();
    c->app_tmax = false;
    pend_retire(c);
    return HSC_OK;
}

static int build_from_host(hsc_ctx *c)
{
    const size_t n_in = c->h_gid.size();
    set_words(c, window_words(c));
    const int W = c->W;
    c->cap = window_cap(n_in);
    const size_t cap = c->cap;
    std::vector<uint64_t> words((size_t)W * cap, 0);
    std::vector<uint8_t> buf((size_t)W * 8);
    for (size_t i = 0; i < n_in; ++i) {
        const int klen = c->groups[c->h_gid[i]].klen;
        std::fill(buf.begin(), buf.end(), 0);
        if (klen) memcpy(buf.data(), c->h_keys.data() + c->h_keyoff[i], (size_t)klen);
        for (int j = 0; j < W; ++j) words[(size_t)j * cap + i] = load_be64(buf.data() + 8 * j);
    }
    HIPCHK(c, c->d_gid.ensure(cap * 4));
    HIPCHK(c, c->d_words.ensure(cap * 8 * W));
    HIPCHK(c, c->d_lsn.ensure(cap * 8));
    hipStream_t s = c->stream;
    if (n_in) {
        HIPCHK(c, hipMemcpyAsync(c->d_gid.p, c->h_gid.data(), 4 * n_in, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->d_words.p, words.data(), 8 * (size_t)W * cap, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->d_lsn.p, c->h_lsn.data(), 8 * n_in, hipMemcpyHostToDevice, s));
    }
    return device_build(c, n_in);
}

// Appended rows (app_*) as a sorted SoA (gid, W words, lsn) in pinned
// staging: returns the row count.
// Staged rows: [gid: 4k, padded to 16][words: 8Wk][lsn: 8k] then, nt > 0,
// [table maxima: 8nt] -- one upload for an append.
static size_t stage_bytes(size_t k, int W, int nt)
{
    return ((4 * k + 15) & ~(size_t)15) + 8 * (size_t)W * k + 8 * k + 8 * (size_t)nt;
}

static int stage_appends(hsc_ctx *c, int W, size_t *k_out, int nt = 0)
{
    const size_t k = c->app_gid.size();
    *k_out = k;
    if (!k) return HSC_OK;
    std::vector<uint64_t> rw(k * (size_t)W);
    std::vector<uint32_t> ord(k);
    uint8_t buf[kMaxWords * 8];
    for (size_t i = 0; i < k; ++i) {
        const int klen = c->groups[c->app_gid[i]].klen;
        memset(buf, 0, (size_t)W * 8);
        if (klen) memcpy(buf, c->app_keys.data() + c->app_koff[i], (size_t)klen);
        for (int j = 0; j < W; ++j) rw[i * W + j] = load_be64(buf + 8 * j);
        ord[i] = (uint32_t)i;
    }
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
        if (c->app_gid[a] != c->app_gid[b]) return c->app_gid[a] < c->app_gid[b];
        for (int j = 0; j < W; ++j)
            if (rw[a * W + j] != rw[b * W + j]) return rw[a * W + j] < rw[b * W + j];
        return false;
    });
    HIPCHK_RC(c, app_stage(c, stage_bytes(k, W, nt) + 16));
    uint32_t *g = c->h_app->as<uint32_t>();
    uint64_t *wd = (uint64_t *)(c->h_app->as<uint8_t>() + ((4 * k + 15) & ~(size_t)15));
    uint64_t *ls = wd + (size_t)W * k;
    for (size_t i = 0; i < k; ++i) {
        const uint32_t r = ord[i];
        g[i] = c->app_gid[r];
        for (int j = 0; j < W; ++j) wd[(size_t)j * k + i] = rw[(size_t)r * W + j];
        ls[i] = c->app_lsn[r];
    }
    if (nt) memcpy(ls + k, c->h_table_max.data(), 8 * (size_t)nt);
    return HSC_OK;
}

static DeltaView delta_view(const hsc_ctx *c)
{
    DeltaView d{};
    d.gid = c->d_dgid[c->dcur].as<uint32_t>();
    d.words = c->d_dwords[c->dcur].as<uint64_t>();
    d.lsn = c->d_dlsn[c->dcur].as<uint64_t>();
    d.bmax = c->d_dbmax.as<uint64_t>();
    d.stride = c->dcap;
    d.n = (uint32_t)c->dn;
    d.W = c->W;
    return d;
}

// Appends since the last call into the device delta run (one merge launch,
// asynchronous on c->stream) and the table maxima into d_table_max.  A delta
// past kDeltaCap, or a key longer than the window's words, schedules a merge
// into the main window instead (at the next check).
static int fold_start(hsc_ctx *c);
static int fold_finish(hsc_ctx *c, bool wait);
static bool small_path(hsc_ctx *c, int T);

// An append that can stay in the pending tail: k = every unmerged row
// (mirrored ones included).  The next small check scans them; the merge waits
// for kPendRows of them or a batch that is not small (probe -> settle).
static bool pend_fits(hsc_ctx *c, size_t k, bool sync_only)
{
    return !sync_only && small_path(c, 1) && c->W <= kPendMaxWords && k <= kPendRows &&
           c->dn + k <= kDeltaCap && c->pend_t + c->app_tchg.size() <= kPendRows;
}

// Mirror rows [pend_n, k) of app_* and the raised table maxima into the
// current pending buffer (rows below pend_n are never rewritten while a
// launch may read them).
static int pend_mirror(hsc_ctx *c)
{
    const int i = c->pend_i;
    HBuf &b = c->h_pend[i];
    if (!c->pend_n && !c->pend_t) {  // a buffer being refilled: its last readers ran
        if (c->pend_ev[i] && hipEventSynchronize(c->pend_ev[i]) != hipSuccess)
            return fail(c, HSC_EDEVICE, "pending tail event");
        if (b.ensure(kPendBytes, true, true)) return fail(c, HSC_ENOMEM, "pending tail");
    }
    uint8_t *p = b.as<uint8_t>();
    const size_t k = c->app_gid.size();
    const int W = c->W;
    uint8_t buf[kPendMaxWords * 8];
    for (size_t r = c->pend_n; r < k; ++r) {
        const int klen = c->groups[c->app_gid[r]].klen;
        memset(buf, 0, sizeof buf);
        if (klen) memcpy(buf, c->app_keys.data() + c->app_koff[r], (size_t)std::min(klen, 8 * W));
        ((uint32_t *)p)[r] = c->app_gid[r];
        ((uint64_t *)(p + kPendLsn))[r] = c->app_lsn[r];
        for (int j = 0; j < W; ++j) ((uint64_t *)(p + kPendWords))[(size_t)j * kPendRows + r] = load_be64(buf + 8 * j);
    }
    uint32_t *tt = (uint32_t *)(p + kPendTtid);
    uint64_t *tl = (uint64_t *)(p + kPendTlsn);
    for (uint32_t t : c->app_tchg) {
        bool seen = false;  // one entry per table and append, its latest maximum
        for (uint32_t e = c->pend_t; e-- > 0 && !seen;) seen = tt[e] == t && tl[e] == c->h_table_max[t];
        if (seen) continue;
        tt[c->pend_t] = t;
        tl[c->pend_t] = c->h_table_max[t];
        ++c->pend_t;
    }
    c->app_tchg.clear();
    std::atomic_thread_fence(std::memory_order_release);
    c->pend_n = (uint32_t)k;
    c->pend_appends++;
    return HSC_OK;
}

// Both delta-run buffers at full size for the window's words: merges never
// reallocate a run holding rows (a wider key schedules a rebuild).  Called by
// the first merge, or ahead of it by append_prepare.
static int delta_alloc(hsc_ctx *c, int W)
{
    const size_t wbytes = 8 * (size_t)W * kDeltaCap;
    if (c->dcap >= kDeltaCap && c->d_dwords[0].bytes >= wbytes && c->d_dwords[1].bytes >= wbytes) return HSC_OK;
    if (c->dn) return fail(c, HSC_EINVAL, "delta run resized while holding rows");
    c->dcap = kDeltaCap;
    for (int b = 0; b < 2; ++b) {
        HIPCHK(c, c->d_dgid[b].ensure(4 * (size_t)kDeltaCap));
        HIPCHK(c, c->d_dwords[b].ensure(wbytes));
        HIPCHK(c, c->d_dlsn[b].ensure(8 * (size_t)kDeltaCap));
    }
    HIPCHK(c, c->d_dbmax.ensure(8 * (size_t)(kDeltaCap / 64 + 1)));
    return HSC_OK;
}

static void fold_worker(hsc_ctx *c);
static hipError_t create_stream(hipStream_t *st, bool high);

// What the append path would otherwise set up on a commit's clock the first
// time it needs it: the delta-run buffers (hipMallocs, at the first merge of
// the pending tail) and, with background folds, the fold's shadow context
// with its stream, the worker thread and its event.  Run after every window
// build, so a commit stream pays them at its first check, which builds the
// window anyway.  (A stream created by the worker at the first fold stalled
// the checks running meanwhile by 1.6 ms: r06e, scripts/fold_diag.py.)
static int append_prepare(hsc_ctx *c)
{
    if (c->multi || c->host_only || !c->live || c->W <= 0) return HSC_OK;
    HIPCHK_RC(c, delta_alloc(c, c->W));
    if (!c->fold_bg) return HSC_OK;
    if (!c->fold_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fold_ev, hipEventDisableTiming));
    if (!c->shadow && c->fold_state.load(std::memory_order_acquire) == kFoldIdle) {
        hsc_ctx *s = new (std::nothrow) hsc_ctx();
        if (!s) return fail(c, HSC_ENOMEM, "fold context");
        s->device = c->device;
        if (create_stream(&s->own_stream, false) != hipSuccess) {
            delete s;
            return fail(c, HSC_EDEVICE, "fold stream");
        }
        s->stream = s->own_stream;
        c->shadow = s;
    }
    if (!c->fold_thread.joinable()) {
        try {
            c->fold_thread = std::thread(fold_worker, c);
        } catch (...) {
            // fold_start tries again (and folds inline when it cannot)
        }
    }
    return HSC_OK;
}

// lazy (the append entries): an append that fits stays in the pending tail.
// Otherwise -- and for every caller that probes outside k_small_narrow --
// the unmerged rows go to the delta run now.
static int flush_appends(hsc_ctx *c, bool lazy = false)
{
    if (c->multi) return multi_flush_appends(c, lazy);
    if (!c->live || c->host_only) return HSC_OK;
    hipStream_t s = c->stream;
    HIPCHK_RC(c, fold_finish(c, false));
    const size_t k = c->app_gid.size();
    const bool sync_only = window_words(c) > c->W || c->merge_pending || c->groups.size() > c->ng_built;
    if (lazy && (k || c->app_tmax) && pend_fits(c, k, sync_only)) return pend_mirror(c);
    if (getenv("HSC_FOLD_TRACE"))
        fprintf(stderr, "[fold] k %zu dn %zu fn %zu ww %d W %d mp %d groups %zu/%zu state %d\n", k, c->dn, c->fn,
                window_words(c), c->W, (int)c->merge_pending, c->groups.size(), c->ng_built,
                c->fold_state.load());
    if (k && !sync_only && c->fold_bg && c->dn + k > kDeltaCap && k <= kDeltaCap) {
        // the live run is full: wait for a running fold, then fold the run
        HIPCHK_RC(c, fold_finish(c, true));
        if (c->dn + k > kDeltaCap && c->dn && !c->merge_pending) HIPCHK_RC(c, fold_start(c));
    }
    if (k && (sync_only || c->merge_pending || c->dn + k > kDeltaCap)) {
        if (!sync_only && c->dn + k > kDeltaCap) c->merge_is_fold = true;  // the run is full
        c->merge_pending = true;
        c->dirty = true;  // rows stay in app_* for merge_delta (or in h_* for a host rebuild)
        return HSC_OK;
    }
    if (!k && !c->app_tmax) return HSC_OK;
    const double tf0 = fold_trace() ? trace_us() : 0;
    HIPCHK(c, wait_lanes(c));  // probes in flight on other streams keep reading the old run
    const double tf1 = fold_trace() ? trace_us() : 0;
    const int nt = c->app_tmax ? (int)c->table_names.size() : 0;
    if (c->app_tmax) HIPCHK(c, c->d_table_max.ensure(8 * (size_t)std::max(nt, 1)));
    if (!k) {  // table maxima only
        HIPCHK_RC(c, app_stage(c, 8 * (size_t)std::max(nt, 1)));
        memcpy(c->h_app->p, c->h_table_max.data(), 8 * (size_t)nt);
        if (nt) HIPCHK(c, hipMemcpyAsync(c->d_table_max.p, c->h_app->p, 8 * (size_t)nt, hipMemcpyHostToDevice, s));
        HIPCHK_RC(c, app_staged(c, s));  // the ring keeps the buffer until the copy ran
        c->app_tmax = false;
        c->nt_dev = (uint32_t)nt;
        pend_retire(c);
        return HSC_OK;
    }
    const int W = c->W;
    size_t kk = 0;
    HIPCHK_RC(c, stage_appends(c, W, &kk, nt));
    const double tf2 = fold_trace() ? trace_us() : 0;
    // one upload: rows, then the table maxima the merge kernel copies out
    const size_t woff = (4 * k + 15) & ~(size_t)15;
    const size_t sb = stage_bytes(k, W, nt);
    // a commit's rows (at most kDeltaStageRows) stay in the mapped staging,
    // the merge reads them there; more are uploaded first
    // (in place: every merge block stages the k rows from host memory into
    // LDS -- (8W + 12) k + 16 bytes of LDS and that many bytes over PCIe per
    // block; wide keys or a long run upload the rows once instead)
    const size_t merge_blocks = (c->dn + k + 255) / 256;
    const bool in_place = k <= kDeltaStageRows && c->h_app->coherent && W <= 8 &&
                          (size_t)k * (8 * (size_t)W + 12) * merge_blocks <= ((size_t)1 << 20);
    uint8_t *db = (uint8_t *)c->h_app->dp;
    if (!in_place) {
        HIPCHK(c, c->d_agid.ensure(sb));
        HIPCHK(c, hipMemcpyAsync(c->d_agid.p, c->h_app->p, sb, hipMemcpyHostToDevice, s));
        db = c->d_agid.as<uint8_t>();
    }
    HIPCHK_RC(c, delta_alloc(c, W));
    DeltaView a{};
    a.gid = (const uint32_t *)db;
    a.words = (const uint64_t *)(db + woff);
    a.lsn = (const uint64_t *)(db + woff + 8 * (size_t)W * k);
    a.stride = k;
    a.n = (uint32_t)k;
    a.W = W;
    const DeltaView d = delta_view(c);
    const int o = c->dcur ^ 1;
    HIPCHK(c, delta_merge(d, a, c->d_dgid[o].as<uint32_t>(), c->d_dwords[o].as<uint64_t>(),
                          c->d_dlsn[o].as<uint64_t>(), c->dcap, c->d_dbmax.as<uint64_t>(), s,
                          nt ? a.lsn + k : nullptr, nt ? c->d_table_max.as<uint64_t>() : nullptr,
                          (uint32_t)nt, in_place));
    if (nt) c->app_tmax = false, c->nt_dev = (uint32_t)nt;
    const double tf3 = fold_trace() ? trace_us() : 0;
    // no wait: the ring keeps h_app until its copies ran, and every later use
    // of the run is on this stream (hsc_set_stream orders a new stream after it)
    HIPCHK_RC(c, app_staged(c, s));
    if (fold_trace() && trace_us() - tf0 > 120)
        fprintf(stderr, "[merge] %.0f lanes %.0f stage %.0f merge %.0f staged %.0f us (k %zu dn %zu in_place %d)\n", tf0,
                tf1 - tf0, tf2 - tf1, tf3 - tf2, trace_us() - tf3, k, c->dn, (int)in_place);
    c->dcur = o;
    c->dn += k;
    c->app_gid.clear(), c->app_keys.clear(), c->app_koff.clear(), c->app_lsn.clear();
    if (c->pend_n || c->pend_t) c->pend_merges++;
    pend_retire(c);
    if (c->dn >= c->fold_rows) {
        if (!c->fold_bg) {  // inline: the next check folds
            c->merge_pending = true;
            c->merge_is_fold = true;
            c->dirty = true;
        } else if (c->fold_state.load(std::memory_order_acquire) == kFoldIdle) {
            HIPCHK_RC(c, fold_start(c));
        }
    }
    return HSC_OK;
}

// Fold the delta run (and rows appended since) into the main window of a
// device-ingested window: every version of the last build (key-sorted, in
// d_*2), the delta rows and the pending rows, widened to the current key
// words, become the input of one device rebuild.
static int merge_delta(hsc_ctx *c)
{
    hipStream_t s = c->stream;
    (void)fold_finish(c, true);  // a failed fold leaves its rows in the frozen run, merged below
    HIPCHK(c, wait_lanes(c));
    const int W0 = c->W, W = std::max(c->W, window_words(c));
    size_t k = 0;
    HIPCHK_RC(c, stage_appends(c, W, &k));
    const size_t nf = c->fn;
    const size_t na = c->n_all + nf, nd = c->dn, n_in = na + nd + k;
    if (n_in >= 0xFFFFFFFFull) return fail(c, HSC_EINVAL, "window too large");
    const size_t cap = window_cap(n_in);
    DBuf g, wd, l;
    HIPCHK(c, g.ensure(4 * cap));
    HIPCHK(c, wd.ensure(8 * (size_t)W * cap));
    HIPCHK(c, l.ensure(8 * cap));
    if (W > W0) HIPCHK(c, hipMemsetAsync(wd.p, 0, 8 * (size_t)W * cap, s));
    const size_t nm = c->n_all;  // the main window's versions, then the frozen run's rows
    if (nm) {
        HIPCHK(c, hipMemcpyAsync(g.p, c->d_gid2.p, 4 * nm, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(l.p, c->d_lsn2.p, 8 * nm, hipMemcpyDeviceToDevice, s));
        for (int j = 0; j < W0; ++j)
            HIPCHK(c, hipMemcpyAsync(wd.as<uint64_t>() + (size_t)j * cap,
                                     c->d_words2.as<uint64_t>() + (size_t)j * c->cap, 8 * nm,
                                     hipMemcpyDeviceToDevice, s));
    }
    if (nf) {
        HIPCHK(c, hipMemcpyAsync(g.as<uint32_t>() + nm, c->f_dgid.p, 4 * nf, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(l.as<uint64_t>() + nm, c->f_dlsn.p, 8 * nf, hipMemcpyDeviceToDevice, s));
        for (int j = 0; j < W0; ++j)
            HIPCHK(c, hipMemcpyAsync(wd.as<uint64_t>() + (size_t)j * cap + nm,
                                     c->f_dwords.as<uint64_t>() + (size_t)j * c->dcap, 8 * nf,
                                     hipMemcpyDeviceToDevice, s));
    }
    if (nd) {
        const DeltaView d = delta_view(c);
        HIPCHK(c, hipMemcpyAsync(g.as<uint32_t>() + na, d.gid, 4 * nd, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(l.as<uint64_t>() + na, d.lsn, 8 * nd, hipMemcpyDeviceToDevice, s));
        for (int j = 0; j < W0; ++j)
            HIPCHK(c, hipMemcpyAsync(wd.as<uint64_t>() + (size_t)j * cap + na, d.words + (size_t)j * d.stride,
                                     8 * nd, hipMemcpyDeviceToDevice, s));
    }
    if (k) {
        const uint8_t *hb = c->h_app->as<uint8_t>();
        const size_t woff = (4 * k + 15) & ~(size_t)15;
        HIPCHK(c, hipMemcpyAsync(g.as<uint32_t>() + na + nd, hb, 4 * k, hipMemcpyHostToDevice, s));
        for (int j = 0; j < W; ++j)
            HIPCHK(c, hipMemcpyAsync(wd.as<uint64_t>() + (size_t)j * cap + na + nd,
                                     hb + woff + 8 * (size_t)j * k, 8 * k, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(l.as<uint64_t>() + na + nd, hb + woff + 8 * (size_t)W * k, 8 * k,
                                 hipMemcpyHostToDevice, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));  // the staging and the old rows are consumed
    c->fn = 0;
    std::swap(c->d_gid, g);
    std::swap(c->d_words, wd);
    std::swap(c->d_lsn, l);
    g.release(), wd.release(), l.release();
    set_words(c, W);
    c->cap = cap;
    return device_build(c, n_in);
}

// ---- background fold -------------------------------------------------------
// The device window: every field a build sets and a probe reads (swapped
// whole between a context and its shadow when a background fold finishes).
static void swap_window(hsc_ctx *a, hsc_ctx *b)
{
    using std::swap;
    if (a->W != b->W) a->dict_epoch++, b->dict_epoch++;
    swap(a->W, b->W), swap(a->n, b->n), swap(a->cap, b->cap), swap(a->n_all, b->n_all);
    swap(a->ng_built, b->ng_built);
    swap(a->ntiles, b->ntiles), swap(a->log2T, b->log2T), swap(a->levels, b->levels);
    swap(a->narrow, b->narrow), swap(a->lw, b->lw), swap(a->tz, b->tz);
    swap(a->ncomp, b->ncomp), swap(a->nc0, b->nc0), swap(a->d_ncmeta, b->d_ncmeta);
    swap(a->d_nkeys, b->d_nkeys), swap(a->d_nmaxs, b->d_nmaxs), swap(a->d_nbase, b->d_nbase);
    swap(a->nv, b->nv), swap(a->wn, b->wn);
    swap(a->d_nzero, b->d_nzero), swap(a->d_ntmax, b->d_ntmax), swap(a->d_nsp_g, b->d_nsp_g);
    swap(a->d_nsp_w, b->d_nsp_w), swap(a->d_ngs, b->d_ngs), swap(a->d_nscratch, b->d_nscratch);
    swap(a->ntiles32, b->ntiles32), swap(a->d_trad2, b->d_trad2), swap(a->d_commits, b->d_commits);
    swap(a->d_cdir, b->d_cdir), swap(a->d_tdir, b->d_tdir), swap(a->d_trad, b->d_trad);
    swap(a->d_key32, b->d_key32), swap(a->d_rank32, b->d_rank32);
    for (int i = 0; i < 4; ++i) swap(a->d_ctmp[i], b->d_ctmp[i]);
    swap(a->cdir, b->cdir), swap(a->tdir, b->tdir), swap(a->trad_m, b->trad_m);
    swap(a->trad_log, b->trad_log), swap(a->ncommit, b->ncommit), swap(a->has_commits, b->has_commits);
    swap(a->commit_span[0], b->commit_span[0]), swap(a->commit_span[1], b->commit_span[1]);
    swap(a->rank_lsn32, b->rank_lsn32), swap(a->rank_base, b->rank_base);
    swap(a->d_gid, b->d_gid), swap(a->d_words, b->d_words), swap(a->d_lsn, b->d_lsn);
    swap(a->d_gid2, b->d_gid2), swap(a->d_words2, b->d_words2), swap(a->d_lsn2, b->d_lsn2);
    swap(a->d_flags, b->d_flags), swap(a->d_scratch, b->d_scratch);
    swap(a->d_pk[0], b->d_pk[0]), swap(a->d_pk[1], b->d_pk[1]), swap(a->packed_sort, b->packed_sort);
    swap(a->d_gstart, b->d_gstart), swap(a->d_gend, b->d_gend), swap(a->d_tmax, b->d_tmax);
    swap(a->d_table_max, b->d_table_max), swap(a->d_group_table, b->d_group_table);
    swap(a->nt_dev, b->nt_dev);
    swap(a->d_count, b->d_count), swap(a->d_sp_g, b->d_sp_g), swap(a->d_sp_w, b->d_sp_w);
    swap(a->compact, b->compact), swap(a->ct, b->ct), swap(a->wc, b->wc);
    swap(a->d_cmask, b->d_cmask), swap(a->d_cpat, b->d_cpat), swap(a->d_cmv, b->d_cmv);
    swap(a->d_cbits, b->d_cbits), swap(a->d_cwords, b->d_cwords), swap(a->d_ctmax, b->d_ctmax);
    swap(a->d_csp_g, b->d_csp_g), swap(a->d_csp_w, b->d_csp_w), swap(a->ct_maxbits, b->ct_maxbits);
    swap(a->ctiles, b->ctiles), swap(a->ctv, b->ctv);
    swap(a->d_ckey, b->d_ckey), swap(a->d_crank, b->d_crank), swap(a->d_cfirst, b->d_cfirst);
    swap(a->d_crel, b->d_crel), swap(a->d_ctrad, b->d_ctrad), swap(a->d_ctb, b->d_ctb);
    swap(a->d_cph, b->d_cph), swap(a->cph_nb, b->cph_nb), swap(a->cph_ep, b->cph_ep);
}

static DeltaView frozen_view(const hsc_ctx *c)
{
    DeltaView d{};
    d.gid = c->f_dgid.as<uint32_t>();
    d.words = c->f_dwords.as<uint64_t>();
    d.lsn = c->f_dlsn.as<uint64_t>();
    d.bmax = c->f_dbmax.as<uint64_t>();
    d.stride = c->dcap;
    d.n = (uint32_t)c->fn;
    d.W = c->W;
    return d;
}

// Stream priorities: the small-batch streams (a lone check's latency) get
// the device's highest, a background fold's build the lowest, so a fold's
// kernels never sit in front of a check's in a hardware queue.
static hipError_t create_stream(hipStream_t *st, bool high)
{
    static const bool prio = getenv("HSC_NO_STREAM_PRIO") == nullptr;  // (A/B diagnostics)
    int least = 0, greatest = 0;
    if (!prio || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest)
        return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    return hipStreamCreateWithPriority(st, hipStreamNonBlocking, high ? greatest : least);
}

// The fold worker (one host thread per context, started by its first fold):
// it creates the shadow context and its low-priority stream itself, then
// for every job copies the main window's versions and the frozen run into
// the shadow's buffers on the shadow's stream -- after the event fold_start
// recorded behind everything queued on the context's stream -- and rebuilds
// there.  An append that triggers a fold only captures the job and records
// that event (no stream creation, allocation or copy on the commit path).
static void fold_worker(hsc_ctx *c)
{
    for (;;) {
        hsc_ctx::FoldJob j;
        {
            std::unique_lock<std::mutex> g(c->fold_mu);
            c->fold_cv.wait(g, [c] { return c->fold_job || c->fold_quit; });
            if (c->fold_quit) return;
            c->fold_job = false;
            j = std::move(c->fold_jobv);
        }
        (void)hipSetDevice(c->device);
        int rc = HSC_OK;
        std::string why;
        hsc_ctx *s = c->shadow;  // (made by append_prepare when the window was built)
        if (!s) rc = HSC_EDEVICE, why = "fold context";
        if (rc == HSC_OK) {
            s->groups = std::move(j.groups);  // what device_build reads of the dictionaries
            s->table_names = std::move(j.table_names);
            s->h_table_max = std::move(j.table_max);
            s->layout = j.layout;
            s->paths = j.paths;
            s->W = j.W;
            const double tw0 = fold_trace() ? trace_us() : 0;
            const size_t nm = j.nm, nf = j.nf, n_in = nm + nf;
            const int W = j.W;
            // the shadow's buffers (its own, or the main window's after a
            // swap) are kept while they fit, and grow with room for later folds
            if (s->cap < n_in) s->cap = window_cap(n_in + n_in / 2 + c->fold_rows);
            hipStream_t ss = s->stream;
            hipError_t e = s->d_gid.ensure(4 * s->cap);
            if (e == hipSuccess) e = s->d_words.ensure(8 * (size_t)W * s->cap);
            if (e == hipSuccess) e = s->d_lsn.ensure(8 * s->cap);
            if (e == hipSuccess) e = hipStreamWaitEvent(ss, c->fold_ev, 0);
            auto cp = [&](void *dst, const void *src, size_t b) {
                if (e == hipSuccess && b) e = hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, ss);
            };
            cp(s->d_gid.p, j.gid2, 4 * nm);
            cp(s->d_lsn.p, j.lsn2, 8 * nm);
            cp(s->d_gid.as<uint32_t>() + nm, j.fgid, 4 * nf);
            cp(s->d_lsn.as<uint64_t>() + nm, j.flsn, 8 * nf);
            for (int w = 0; w < W; ++w) {
                uint64_t *dst = s->d_words.as<uint64_t>() + (size_t)w * s->cap;
                cp(dst, (const uint64_t *)j.words2 + (size_t)w * j.cap, 8 * nm);
                cp(dst + nm, (const uint64_t *)j.fwords + (size_t)w * j.dcap, 8 * nf);
            }
            const double tb0 = fold_trace() ? trace_us() : 0;
            if (e != hipSuccess) {
                rc = HSC_EDEVICE, why = std::string("fold copies: ") + hipGetErrorString(e);
            } else {
                rc = device_build(s, n_in);
                if (rc) why = s->err;
            }
            if (fold_trace())
                fprintf(stderr, "[fold] %.0f worker: n_in %zu cap %zu copies+allocs %.0f us build %.0f us\n", trace_us(),
                        n_in, s->cap, tb0 - tw0, trace_us() - tb0);
        }
        {
            std::lock_guard<std::mutex> g(c->fold_mu);
            c->fold_rc = rc;
            c->fold_err = why;
            c->fold_state.store(kFoldDone, std::memory_order_release);
        }
        c->fold_cv.notify_all();
    }
}

// Until a running fold's job is done.
static void fold_wait(hsc_ctx *c)
{
    std::unique_lock<std::mutex> g(c->fold_mu);
    c->fold_cv.wait(g, [c] { return c->fold_state.load(std::memory_order_acquire) != kFoldRunning; });
}

static void fold_stop(hsc_ctx *c)
{
    if (!c->fold_thread.joinable()) return;
    fold_wait(c);
    {
        std::lock_guard<std::mutex> g(c->fold_mu);
        c->fold_quit = true;
    }
    c->fold_cv.notify_all();
    c->fold_thread.join();
}

// Freeze the live run and hand the rebuild of the main window with it to the
// fold worker: the run's buffers become the frozen run (probed beside the
// main window and a fresh live run until the swap), the job captures what
// the build reads, and an event behind everything queued on the context's
// stream so far (the run's last merge, and the readers of the shadow's
// buffers -- the window before the last swap) orders the worker's copies.
static int fold_start(hsc_ctx *c)
{
    if (!c->shadow) HIPCHK_RC(c, append_prepare(c));  // (normally made at the build)
    if (!c->fold_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fold_ev, hipEventDisableTiming));
    if (!c->fold_thread.joinable()) {
        try {
            c->fold_thread = std::thread(fold_worker, c);
        } catch (...) {
            c->merge_pending = c->dirty = true;  // no worker: the run is merged inline
            c->merge_is_fold = true;
            return HSC_OK;
        }
    }
    std::swap(c->d_dgid[c->dcur], c->f_dgid);
    std::swap(c->d_dwords[c->dcur], c->f_dwords);
    std::swap(c->d_dlsn[c->dcur], c->f_dlsn);
    std::swap(c->d_dbmax, c->f_dbmax);
    c->fn = c->dn;
    c->dn = 0;
    HIPCHK(c, hipEventRecord(c->fold_ev, c->stream));
    {
        std::lock_guard<std::mutex> g(c->fold_mu);
        hsc_ctx::FoldJob &j = c->fold_jobv;
        j.nm = c->n_all, j.nf = c->fn, j.cap = c->cap, j.dcap = c->dcap;
        j.W = c->W, j.layout = c->layout, j.paths = c->paths;
        j.gid2 = c->d_gid2.p, j.lsn2 = c->d_lsn2.p, j.words2 = c->d_words2.p;
        j.fgid = c->f_dgid.p, j.flsn = c->f_dlsn.p, j.fwords = c->f_dwords.p;
        j.groups = c->groups;
        j.table_names = c->table_names;
        j.table_max = c->h_table_max;
        c->fold_rc = HSC_OK;
        c->fold_state.store(kFoldRunning, std::memory_order_release);
        c->fold_job = true;
    }
    c->fold_cv.notify_all();
    c->folds_started++;
    if (fold_trace()) fprintf(stderr, "[fold] %.0f start: main %zu frozen %zu\n", trace_us(), c->n_all, c->fn);
    return HSC_OK;
}

// A finished background fold (or, wait = true, a running one once done):
// swap the shadow's window in.  On failure the frozen run stays probed and
// the next check merges it inline.
static int fold_finish(hsc_ctx *c, bool wait)
{
    const int st = c->fold_state.load(std::memory_order_acquire);
    if (st == kFoldIdle || (st == kFoldRunning && !wait)) return HSC_OK;
    fold_wait(c);
    c->fold_state.store(kFoldIdle, std::memory_order_relaxed);
    hsc_ctx *s = c->shadow;
    if (c->fold_rc != HSC_OK || !s) {
        c->merge_pending = c->dirty = true;
        c->merge_is_fold = true;
        (void)fail(c, c->fold_rc ? c->fold_rc : HSC_EDEVICE, ("background fold: " + c->fold_err).c_str());
        return HSC_OK;
    }
    const double ts0 = fold_trace() ? trace_us() : 0;
    HIPCHK(c, wait_lanes(c));  // batches of other streams finish on the old window
    swap_window(c, s);
    // table maxima raised while the fold ran (the shadow's are as of its start)
    const int nt = (int)c->table_names.size();
    for (int t = 0; t < nt && t < (int)s->h_table_max.size(); ++t)
        c->h_table_max[t] = std::max(c->h_table_max[t], s->h_table_max[t]);
    HIPCHK(c, c->d_table_max.ensure(8 * (size_t)std::max(nt, 1)));
    // (on c->stream: the probes that read the maxima are queued there)
    if (nt)
        HIPCHK(c, hipMemcpyAsync(c->d_table_max.p, c->h_table_max.data(), 8 * (size_t)nt, hipMemcpyHostToDevice,
                                 c->stream));
    c->nt_dev = (uint32_t)nt;
    c->app_tmax = false;
    c->fn = 0;
    HIPCHK(c, hipEventRecord(c->fold_ev, c->stream));  // the old window's last readers
    c->folds_swapped++;
    c->fold_ms = s->last.ingest_ms;
    if (fold_trace()) fprintf(stderr, "[fold] %.0f swap %.0f us (n %zu)\n", trace_us(), trace_us() - ts0, c->n);
    return HSC_OK;
}

static void fold_discard(hsc_ctx *c)
{
    if (c->fold_state.load(std::memory_order_acquire) != kFoldIdle) {
        fold_wait(c);
        c->fold_state.store(kFoldIdle, std::memory_order_relaxed);
    }
    c->fn = 0;
}

static int ensure_built(hsc_ctx *c)
{
    if (c->multi) {  // the window lives on the member contexts (hsc_multi.cpp)
        if (!c->dirty && c->groups.size() <= c->ng_built) return HSC_OK;
        return multi_build(c);
    }
    if (c->host_only) {  // dictionaries + marshalling only
        set_words(c, window_words(c));
        return HSC_OK;
    }
    HIPCHK_RC(c, fold_finish(c, false));
    // A group first seen after the build (the first write to an index, or
    // hsc_register_group) has no entry in the per-group tables, which are
    // sized at the build: the marshal would emit probes with its gid, so the
    // window is rebuilt before any probe runs.
    if (!c->dirty && c->groups.size() > c->ng_built) {
        c->dirty = true;
        if (!c->host_staged) c->merge_pending = true;
    }
    if (!c->dirty) return HSC_OK;
    if (c->merge_pending && c->merge_is_fold) c->folds_inline++;  // (a new group / wider key: a rebuild)
    c->merge_is_fold = false;
    int rc;
    if (c->host_staged) {  // staged rows include the appended ones (and a frozen run's)
        fold_discard(c);
        rc = build_from_host(c);
    } else if (c->merge_pending) {
        rc = merge_delta(c);
    } else {
        return fail(c, HSC_ESTATE, "device window must be re-ingested");
    }
    return rc ? rc : append_prepare(c);
}

// ---------------------------------------------------------------------------
// log decode (what osql_serial_check + serial_check_this_txn visit)
// ---------------------------------------------------------------------------
static bool is_regop(uint32_t t)
{
    return t == HSC_REC_TXN_REGOP || t == HSC_REC_TXN_REGOP_GEN || t == HSC_REC_TXN_REGOP_ROWLOCKS;
}

// Index of the stored record at lsn, or -1.
static long lg_find(const hsc_ctx *c, uint64_t lsn)
{
    const auto &v = c->lg.lsn;
    auto p = std::lower_bound(v.begin(), v.end(), lsn);
    return (p != v.end() && *p == lsn) ? (long)(p - v.begin()) : -1;
}

// Append log records (the continuation of the window's log: LSNs above every
// stored one) and take in the writes of every txn they commit -- what
// osql_serial_check / serial_check_this_txn visit (bdb/serializable.c:426-534,
// 60-332): a regop whose prev record is an ltran_commit with isabort == 0 and
// prevllsn.file != 0 commits the logical chain walked back from prevllsn to
// ltran_start.  Chains may reach into records of earlier appends.  On an
// unreadable record the reference's scan errors out (nonzero): poison LSNs.
static int append_log(hsc_ctx *c, const hsc_llog *log)
{
    const uint64_t last = c->lg.lsn.empty() ? 0 : c->lg.lsn.back();
    for (size_t i = 0; i < log->nrec; ++i)
        if ((i ? log->lsn[i] <= log->lsn[i - 1] : (!c->lg.lsn.empty() && log->lsn[0] <= last)))
            return fail(c, HSC_EINVAL, "log LSNs not increasing");
    if (log->end_lsn < (log->nrec ? log->lsn[log->nrec - 1] : last))
        return fail(c, HSC_EINVAL, "end LSN before the last record");
    std::vector<int> tmap(std::max(log->ntbnames, 0), -1);
    auto tid_of = [&](int32_t t) -> int {
        if (t < 0 || t >= log->ntbnames) return -1;
        if (tmap[t] < 0) tmap[t] = table_id_or_add(c, log->tbnames[t]);
        return tmap[t];
    };
    // store the new records
    auto &L = c->lg;
    const size_t r0 = L.lsn.size();
    for (size_t i = 0; i < log->nrec; ++i) {
        const uint32_t t = log->rectype[i];
        L.lsn.push_back(log->lsn[i]);
        L.rectype.push_back(t);
        L.prev.push_back(log->prev[i]);
        L.isabort.push_back(log->isabort[i]);
        const bool undo = t >= HSC_REC_UNDO_ADD_DTA && t != HSC_REC_LTRAN_COMMIT &&
                          t != HSC_REC_LTRAN_START && t != HSC_REC_LTRAN_COMPREC;
        L.table.push_back(undo ? tid_of(log->table[i]) : -1);
        L.ix.push_back(log->ix[i]);
        const int32_t kl = log->keylen[i];
        const bool has_key = t == HSC_REC_UNDO_ADD_IX || t == HSC_REC_UNDO_DEL_IX ||
                             t == HSC_REC_UNDO_DEL_IX_LK || t == HSC_REC_UNDO_UPD_IX ||
                             t == HSC_REC_UNDO_ADD_IX_LK || t == HSC_REC_UNDO_UPD_IX_LK;
        L.key_off.push_back(L.keys.size());
        L.keylen.push_back(has_key ? kl : 0);
        if (has_key && kl > 0) L.keys.insert(L.keys.end(), log->keys + log->key_off[i],
                                             log->keys + log->key_off[i] + kl);
    }
    c->end_lsn = log->end_lsn;
    // take in the txns the new regops commit
    for (size_t i = r0; i < L.lsn.size(); ++i) {
        if (!is_regop(L.rectype[i])) continue;
        const uint64_t c_lsn = L.lsn[i];
        long p = lg_find(c, L.prev[i]);
        if (p < 0) {  // prevcur->get fails -> the scan errors out (nonzero)
            c->poison_regop = std::max(c->poison_regop, c_lsn);
            continue;
        }
        if (L.rectype[p] != HSC_REC_LTRAN_COMMIT) continue;
        if ((uint32_t)(L.prev[p] >> 32) == 0) continue;  // not a write txn
        if (L.isabort[p]) continue;
        // committed write txn: walk prevllsn back to ltran_start
        if (c_lsn > c->max_commit) c->max_commit = c_lsn;
        long r = lg_find(c, L.prev[p]);
        if (r < 0) {
            c->poison_chain = std::max(c->poison_chain, c_lsn);
            continue;
        }
        for (;;) {
            const uint32_t t = L.rectype[r];
            if (t == HSC_REC_LTRAN_START) break;
            switch (t) {
            case HSC_REC_UNDO_ADD_DTA:
            case HSC_REC_UNDO_DEL_DTA:
            case HSC_REC_UNDO_UPD_DTA:
            case HSC_REC_UNDO_ADD_DTA_LK:
            case HSC_REC_UNDO_DEL_DTA_LK:
            case HSC_REC_UNDO_UPD_DTA_LK:
                if (L.table[r] < 0) return fail(c, HSC_ELOG, "bad table index in log");
                add_write(c, L.table[r], -2, nullptr, 0, false, c_lsn);
                break;
            case HSC_REC_UNDO_ADD_IX:
            case HSC_REC_UNDO_DEL_IX:
            case HSC_REC_UNDO_DEL_IX_LK:
            case HSC_REC_UNDO_UPD_IX:
            case HSC_REC_UNDO_ADD_IX_LK:
            case HSC_REC_UNDO_UPD_IX_LK:
                if (L.table[r] < 0) return fail(c, HSC_ELOG, "bad table index in log");
                add_write(c, L.table[r], (int)L.ix[r], L.keys.data() + L.key_off[r], L.keylen[r],
                          true, c_lsn);
                break;
            case HSC_REC_LTRAN_COMMIT:
            case HSC_REC_LTRAN_COMPREC:
                break;
            default:  // the reference abort()s (bdb/serializable.c:283-286)
                return fail(c, HSC_ELOG, "unknown record type in logical chain");
            }
            const uint64_t lsn = L.prev[r];
            if ((uint32_t)(lsn >> 32) == 0) break;
            r = lg_find(c, lsn);
            if (r < 0) {
                c->poison_chain = std::max(c->poison_chain, c_lsn);
                break;
            }
        }
    }
    if (!c->live) c->dirty = true;
    return HSC_OK;
}

static int ingest_log(hsc_ctx *c, const hsc_llog *log)
{
    clear_window(c);
    c->lg_rule = true;  // every record of the window is in the store
    return append_log(c, log);
}

// ---------------------------------------------------------------------------
// marshalling
// ---------------------------------------------------------------------------
// Bound normalised to the group's key length klen (padding lemma, SURVEY
// §8(a) A0): lower = lkey[0..min) ++ 0x00.., upper = rkey[0..min) ++ 0xFF..;
// open bounds become 0x00^klen / 0xFF^klen.  Then zero padded to W words.
// The first nk (0..8) bytes at p as the high bytes of a big-endian word
// (reads exactly nk bytes: fixed-size loads, no variable-length copy).
static inline uint64_t be_head(const uint8_t *p, int nk)
{
    if (nk >= 8) {
        uint64_t x;
        memcpy(&x, p, 8);
        return __builtin_bswap64(x);
    }
    uint64_t v = 0;
    int sh = 56;
    if (nk & 4) {
        uint32_t x;
        memcpy(&x, p, 4);
        v = (uint64_t)__builtin_bswap32(x) << 32;
        p += 4, sh = 24;
    }
    if (nk & 2) {
        uint16_t x;
        memcpy(&x, p, 2);
        v |= (uint64_t)__builtin_bswap16(x) << (sh - 8);
        p += 2, sh -= 16;
    }
    if (nk & 1) v |= (uint64_t)*p << sh;
    return v;
}

// Word q of a bound key that holds the group's whole key length: its nk
// (0..8) key bytes, big-endian.  One 8-byte load when the 8 bytes from p stay
// inside p's page (bytes past the key are masked off, the page is mapped);
// at a page end the exact-length form.
__attribute__((no_sanitize("address"))) static inline uint64_t key_word(const uint8_t *p, int nk)
{
    if (nk <= 0) return 0;
    if (nk >= 8 || ((uintptr_t)p & 4095) <= 4096 - 8) {
        uint64_t x;
        memcpy(&x, p, 8);
        x = __builtin_bswap64(x);
        return nk >= 8 ? x : x & ~(~0ull >> (8 * nk));
    }
    return be_head(p, nk);
}

static inline void norm_bound(const uint8_t *key, int keylen, int flag, int klen, bool upper, int W,
                              uint64_t *out)
{
    // bytes [0, m) from the key, [m, klen) padding (0xFF for an upper bound),
    // [klen, 8W) zero -- built word by word (a key word is one big-endian
    // load when all its 8 bytes are key bytes)
    const int m = flag ? 0 : ((key && keylen > 0) ? std::min(keylen, klen) : 0);
    for (int j = 0; j < W; ++j) {
        const int lo = 8 * j;
        const int nk = std::min(std::max(m - lo, 0), 8);
        uint64_t v = nk ? be_head(key + lo, nk) : 0;
        if (upper) {  // 0xFF over bytes [max(lo, m), min(lo + 8, klen)) of this word
            const int p0 = std::max(lo, m) - lo, p1 = std::min(lo + 8, klen) - lo;
            if (p1 > p0) {
                const uint64_t a = p0 >= 8 ? 0 : ~0ull >> (8 * p0);
                const uint64_t b = p1 >= 8 ? 0 : ~0ull >> (8 * p1);
                v |= a & ~b;
            }
        }
        out[j] = v;
    }
}

// Forced verdicts of a full check that do not depend on the ranges.
// Returns -1 if the device decides, else the rc.  Read-only on c.
static int full_forced(const hsc_ctx *c, uint64_t S)
{
    if (S >= c->end_lsn) return 0;  // DB_SET at/after the end -> DB_NOTFOUND -> 0
    if (c->lg_rule && !std::binary_search(c->lg.lsn.begin(), c->lg.lsn.end(), S))
        return 1;                    // DB_SET inside the log on a non-record -> error
    if (c->poison_regop > S || c->poison_chain > S) return 1;
    return -1;
}

static int regop_rc(hsc_ctx *c, uint64_t S)
{
    if (S >= c->end_lsn) return 0;
    if (c->lg_rule && !std::binary_search(c->lg.lsn.begin(), c->lg.lsn.end(), S)) return 1;
    return (c->max_commit > S || c->poison_regop > S) ? 1 : 0;
}

template <class D, class Get>  // D: hsc_ctx or a MarshalDict snapshot
static void marshal_txn(const D *c, MarshalPart &mp, uint32_t txn, uint64_t S, int nr, Get get)
{
    const int W = c->W;
    auto &tabs = mp.tabs;
    auto &spans = mp.spans;
    auto &refs = mp.refs;
    tabs.clear();
    spans.clear();
    if ((int)refs.size() < nr) refs.resize(nr);
    // pass 1: tables (first range fixes islocked) and per-index [begin, end]
    // spans in array order (currangearr_build_hash, db/sqlglue.c:312-351);
    // spans of one table are kept contiguous by moving later tables' spans.
    // Every range is read once (refs) for both passes.
    size_t slots = 0;
    for (int k = 0; k < nr; ++k) {
        const RangeRef r = refs[k] = get(k);
        if (r.tid < 0) continue;  // table never written: nothing can conflict
        int ti = 0;
        while (ti < (int)tabs.size() && tabs[ti].tid != r.tid) ++ti;
        if (ti == (int)tabs.size()) tabs.push_back(TxnTable{r.tid, r.islocked, (int)spans.size(), 0});
        TxnTable &tt = tabs[ti];
        int j = 0;
        while (j < tt.ns && spans[tt.s0 + j].idx != r.idxnum) ++j;
        if (j < tt.ns) {
            spans[tt.s0 + j].e = k;
            continue;
        }
        // new index of table ti: insert at tt.s0 + tt.ns (shifts later tables);
        // its key groups are looked up once here (one-entry cache across sets)
        const uint64_t ik = ixkey(r.tid, r.idxnum);
        if (ik != mp.ix_last) {
            auto it = c->ix_groups.find(ik);
            mp.ix_last = ik;
            mp.ix_groups = it == c->ix_groups.end() ? nullptr : &it->second;
        }
        spans.insert(spans.begin() + tt.s0 + tt.ns, IdxSpan{r.idxnum, k, k, mp.ix_groups});
        tt.ns++;
        for (int q = ti + 1; q < (int)tabs.size(); ++q) tabs[q].s0++;
    }
    // pass 2: the probes, written in place (room for every span slot x group;
    // empty ranges are dropped by not advancing)
    size_t n = mp.gid.size();
    for (const TxnTable &t : tabs) {
        if (t.islocked) {
            mp.lock_table.push_back((uint32_t)t.tid);
            mp.lock_snap.push_back(S);
            mp.lock_txn.push_back(txn);
            continue;
        }
        for (int j = 0; j < t.ns; ++j) {
            const IdxSpan &sp = spans[t.s0 + j];
            if (sp.groups) slots += sp.groups->size() * (size_t)(sp.e - sp.b + 1);
        }
    }
    if (!slots) return;
    mp.lohi.resize((n + slots) * 2 * (size_t)W);
    mp.gid.resize(n + slots);
    mp.snap.resize(n + slots);
    mp.txn.resize(n + slots);
    uint64_t *lohi = mp.lohi.data();
    for (const TxnTable &t : tabs) {
        if (t.islocked) continue;
        for (int j = 0; j < t.ns; ++j) {
            const IdxSpan &sp = spans[t.s0 + j];
            if (!sp.groups) continue;
            for (int g : *sp.groups) {
                const int klen = c->groups[g].klen;
                // key bytes per word of a bound that holds the whole key length
                // (a bound key at least klen long: the common case, no padding)
                int nkw[kMaxWords];
                for (int q = 0; q < W; ++q) nkw[q] = std::min(std::max(klen - 8 * q, 0), 8);
                // WT: W as a compile-time constant (unrolled word loops) up to 4
                auto fill = [&](auto wt) {
                    constexpr int WT = decltype(wt)::value;
                    const int Wn = WT ? WT : W;
                    for (int k = sp.b; k <= sp.e; ++k) {  // span quirk: every array slot
                        const RangeRef &r = refs[k];
                        uint64_t *w2 = lohi + n * 2 * (size_t)Wn;
                        if (!r.lflag && r.lkey && r.lkeylen >= klen) {
                            for (int q = 0; q < Wn; ++q) w2[q] = key_word(r.lkey + 8 * q, nkw[q]);
                        } else {
                            norm_bound(r.lkey, r.lkeylen, r.lflag, klen, false, Wn, w2);
                        }
                        if (!r.rflag && r.rkey && r.rkeylen >= klen) {
                            for (int q = 0; q < Wn; ++q) w2[Wn + q] = key_word(r.rkey + 8 * q, nkw[q]);
                        } else {
                            norm_bound(r.rkey, r.rkeylen, r.rflag, klen, true, Wn, w2 + Wn);
                        }
                        int cmp = 0;
                        for (int q = 0; q < Wn && !cmp; ++q)
                            if (w2[q] != w2[Wn + q]) cmp = w2[q] < w2[Wn + q] ? -1 : 1;
                        if (cmp > 0) continue;  // empty range never matches
                        mp.gid[n] = (uint32_t)g;
                        mp.snap[n] = S;
                        mp.txn[n] = txn;
                        ++n;
                    }
                };
                switch (W) {
                case 1: fill(std::integral_constant<int, 1>{}); break;
                case 2: fill(std::integral_constant<int, 2>{}); break;
                case 3: fill(std::integral_constant<int, 3>{}); break;
                case 4: fill(std::integral_constant<int, 4>{}); break;
                default: fill(std::integral_constant<int, 0>{});
                }
            }
        }
    }
    mp.lohi.resize(n * 2 * (size_t)W);
    mp.gid.resize(n);
    mp.snap.resize(n);
    mp.txn.resize(n);
}

// Table name -> window table id, with a one-entry cache (a read set names a
// few tables; comdb2 strdup's every CurRange's name, so pointers differ).
template <class D>
struct TableLookupT {
    const D *c;
    const char *last = nullptr;
    int last_tid = -1;
    int operator()(const char *name)
    {
        if (!name) return -1;
        if (last) {  // names are short: an inline compare, no strcmp call
            const char *a = name, *b = last;
            while (*a && *a == *b) ++a, ++b;
            if (*a == *b) return last_tid;
        }
        auto it = c->table_ids.find(name);
        last = name;
        last_tid = it == c->table_ids.end() ? -1 : it->second;
        return last_tid;
    }
};
using TableLookup = TableLookupT<hsc_ctx>;

// A caller's own read set marshalled ahead of its batch (hsc_collect.cpp):
// the rows of marshal_txn (txn 0) against the snapshot of epoch `epoch`.
struct hsc::PreMarshal {
    uint64_t epoch = 0;
    MarshalPart mp;
};

// Source of read sets: flat arrays (hsc_readsets) ...
struct FlatSrc {
    const hsc_readsets *rs;
    const int *tmap;  // rs table -> window table id
    int ntxn() const { return rs->ntxn; }
    uint64_t snap(int t) const { return rs->snap[t]; }
    template <class F>
    void each(int t, TableLookup &, F f) const
    {
        const int64_t r0 = rs->txn_off[t];
        const int nr = (int)(rs->txn_off[t + 1] - r0);
        f(nr, [&](int k) {
            const int64_t r = r0 + k;
            RangeRef x;
            const int32_t tb = rs->table[r];
            x.tid = (tb >= 0 && tb < rs->ntbnames) ? tmap[tb] : -1;
            x.idxnum = rs->idxnum[r];
            x.lkey = rs->lkey_off[r] == HSC_KEY_NULL ? nullptr : rs->keys + rs->lkey_off[r];
            x.rkey = rs->rkey_off[r] == HSC_KEY_NULL ? nullptr : rs->keys + rs->rkey_off[r];
            x.lkeylen = rs->lkeylen[r];
            x.rkeylen = rs->rkeylen[r];
            x.lflag = rs->lflag[r];
            x.rflag = rs->rflag[r];
            x.islocked = rs->islocked[r];
            return x;
        });
    }
    void prefetch(int, int) const {}
    void ahead(int, int) const {}
    bool premarshalled(const hsc_ctx *, int, MarshalPart &, uint32_t) const { return false; }
};

// append a premarshalled read set's rows as read set `txn` of the batch
static void append_pre(const PreMarshal &pm, MarshalPart &mp, uint32_t txn)
{
    const MarshalPart &q = pm.mp;
    mp.lohi.append(q.lohi.data(), q.lohi.size());
    mp.gid.append(q.gid.data(), q.gid.size());
    mp.snap.append(q.snap.data(), q.snap.size());
    mp.txn.append_fill(q.txn.size(), txn);
    mp.lock_table.append(q.lock_table.data(), q.lock_table.size());
    mp.lock_snap.append(q.lock_snap.data(), q.lock_snap.size());
    mp.lock_txn.append_fill(q.lock_txn.size(), txn);
}

// ... or CurRangeArr pointers (the drop-in entry; db/comdb2.h:1105-1124)
struct ArrSrc {
    hsc_currangearr *const *arr;
    const uint64_t *snaps;
    int n;
    PreMarshal *const *pre = nullptr;  // per read set, may be null: marshalled by its caller
    uint64_t epoch = 0;                // the context's dictionary epoch now
    bool pre_ok(int t) const { return pre && pre[t] && pre[t]->epoch == epoch; }
    bool premarshalled(const hsc_ctx *, int t, MarshalPart &mp, uint32_t txn) const
    {
        if (!pre_ok(t)) return false;
        append_pre(*pre[t], mp, txn);
        return true;
    }
    int ntxn() const { return n; }
    uint64_t snap(int t) const { return snaps[t]; }
    template <class F>
    void each(int t, TableLookup &tl, F f) const
    {
        const hsc_currangearr *a = arr[t];
        // table ids once per range (the span builder and the probe pass both
        // read them)
        f(a->size, [&, a](int k) {
            const hsc_currange *r = a->ranges[k];
            RangeRef x;
            x.tid = tl(r->tbname);
            x.idxnum = r->idxnum;
            x.lkey = (const uint8_t *)r->lkey;
            x.rkey = (const uint8_t *)r->rkey;
            x.lkeylen = r->lkeylen;
            x.rkeylen = r->rkeylen;
            x.lflag = r->lflag;
            x.rflag = r->rflag;
            x.islocked = r->islocked;
            return x;
        });
    }
    // A large batch's worker walks its read sets in order: touch the ones a
    // few sets ahead level by level (each level's pointer was prefetched at a
    // larger distance), so a set's cache misses are in flight before its turn.
    void ahead(int t, int t1) const
    {
        if (t + 12 < t1 && !pre_ok(t + 12)) __builtin_prefetch(arr[t + 12]);
        if (t + 8 < t1 && !pre_ok(t + 8)) __builtin_prefetch(arr[t + 8]->ranges);
        if (t + 4 < t1 && !pre_ok(t + 4))
            for (int k = 0; k < arr[t + 4]->size; ++k) __builtin_prefetch(arr[t + 4]->ranges[k]);
        if (t + 2 < t1 && !pre_ok(t + 2))
            for (int k = 0; k < arr[t + 2]->size; ++k) {
                const hsc_currange *r = arr[t + 2]->ranges[k];
                __builtin_prefetch(r->tbname);
                if (r->lkey) __builtin_prefetch(r->lkey);
                if (r->rkey) __builtin_prefetch(r->rkey);
            }
    }
    // A small batch's CurRangeArrs come from other threads' heaps (a
    // collector's callers): touch them level by level -- arrays, range
    // pointers, ranges, keys and names -- so each level's cache misses are
    // in flight together instead of one after another in the marshal.
    void prefetch(int t0, int t1) const
    {
        // callers' premarshalled rows (written on other cores): the objects,
        // then every line of their rows, all in flight before the copies
        if (pre) {
            for (int t = t0; t < t1; ++t)
                if (pre[t]) __builtin_prefetch(pre[t]);
            auto lines = [](const void *p, size_t bytes) {
                for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch((const char *)p + o);
            };
            for (int t = t0; t < t1; ++t)
                if (pre_ok(t)) {
                    const MarshalPart &q = pre[t]->mp;
                    lines(q.lohi.data(), 8 * q.lohi.size());
                    lines(q.gid.data(), 4 * q.gid.size());
                    lines(q.snap.data(), 8 * q.snap.size());
                    if (q.lock_table.size()) {
                        lines(q.lock_table.data(), 4 * q.lock_table.size());
                        lines(q.lock_snap.data(), 8 * q.lock_snap.size());
                    }
                }
        }
        for (int t = t0; t < t1; ++t)
            if (!pre_ok(t)) __builtin_prefetch(arr[t]);
        for (int t = t0; t < t1; ++t)
            if (!pre_ok(t)) __builtin_prefetch(arr[t]->ranges);
        for (int t = t0; t < t1; ++t)
            for (int k = 0; !pre_ok(t) && k < arr[t]->size; ++k) __builtin_prefetch(arr[t]->ranges[k]);
        for (int t = t0; t < t1; ++t)
            for (int k = 0; !pre_ok(t) && k < arr[t]->size; ++k) {
                const hsc_currange *r = arr[t]->ranges[k];
                __builtin_prefetch(r->tbname);
                if (r->lkey) __builtin_prefetch(r->lkey);
                if (r->rkey) __builtin_prefetch(r->rkey);
            }
    }
};

// Host worker threads for the marshal: the box's CPUs (affinity mask, cgroup
// quota), HSC_THREADS or hsc_set_threads.
static int default_threads()
{
    if (const char *e = getenv("HSC_THREADS")) {
        const int n = atoi(e);
        if (n > 0) return std::min(n, 256);
    }
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long per = 0;
        if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
            n = std::min<long>(n, std::max<long>(1, atol(q) / per));
        fclose(f);
    }
    return std::max(1, std::min(n, 64));
}

// Runs f(i) for i in [0, nwork) on the context's worker pool (parallel) or
// on the caller's thread.
template <class F>
static void par_for(hsc_ctx *c, bool parallel, int nwork, F f, bool stat = false)
{
    if (!parallel || c->threads <= 1 || nwork <= 1) {
        for (int i = 0; i < nwork; ++i) f(i);
        return;
    }
    if (!c->pool || c->pool->size() != c->threads) c->pool.reset(new WorkPool(c->threads));
    if (stat)
        c->pool->run_static(nwork, std::function<void(int)>(f));
    else
        c->pool->run(nwork, std::function<void(int)>(f));
}

// Marshal read sets [t0, t1) of src into the staging set st: parts in
// parallel (chunks of read sets), then the SoA assembly ([W][n] words),
// in parallel too.  Sets c->m to point at st.
template <class Src>
static int marshal_into(hsc_ctx *c, const Src &src, int t0, int t1, Stage &st)
{
    const int W = c->W;
    const int nt = t1 - t0;
    // work items of ~kMarshalTxns read sets (one part each)
    const int per = std::max(1, std::min(kMarshalTxns, (nt + c->threads - 1) / std::max(1, c->threads)));
    const int nwork = std::max(1, (nt + per - 1) / per);
    if ((int)c->parts.size() < nwork) c->parts.resize(nwork);
    if (c->parts_cls.size() < c->parts.size()) c->parts_cls.resize(c->parts.size());
    const bool pin = !c->host_only || c->multi;  // a multi context uploads from it
    if (st.forced.ensure((size_t)std::max(nt, 1), pin)) return fail(c, HSC_ENOMEM, "staging");
    uint8_t *forced = st.forced.as<uint8_t>();
    const auto tp0 = std::chrono::steady_clock::now();
    if (nt < kMarshalParallelMin) src.prefetch(t0, t1);
    par_for(c, nt >= kMarshalParallelMin, nwork, [&](int w) {
        MarshalPart &mp = c->parts[w];
        mp.clear();
        TableLookup tl{c};
        const int a = t0 + w * per, e = std::min(t1, a + per);
        for (int t = a; t < e; ++t) {
            src.ahead(t, e);
            const uint64_t S = src.snap(t);
            const int f = full_forced(c, S);
            forced[t - t0] = f > 0;
            if (f >= 0) continue;
            if (src.premarshalled(c, t, mp, (uint32_t)(t - t0))) continue;
            src.each(t, tl, [&](int nr, auto get) { marshal_txn(c, mp, (uint32_t)(t - t0), S, nr, get); });
        }
    }, true);  // static: part w marshalled and assembled on one core
    size_t n = 0, nl = 0;
    for (int w = 0; w < nwork; ++w) {
        c->parts[w].out0 = n;
        c->parts[w].lock0 = nl;
        n += c->parts[w].gid.size();
        nl += c->parts[w].lock_table.size();
    }
    const auto tp1 = std::chrono::steady_clock::now();
    st.L = stage_layout(W, n, nl);
    if (st.arena.ensure(std::max<size_t>(st.L.total + (st.coh ? small_tail((size_t)nt) : 0), 256), pin,
                        st.coh && pin))
        return fail(c, HSC_ENOMEM, "staging buffers");
    uint64_t *lo = st.col<uint64_t>(st.L.lo), *hi = st.col<uint64_t>(st.L.hi);
    uint64_t *sn = st.col<uint64_t>(st.L.snap);
    uint32_t *gid = st.col<uint32_t>(st.L.gid), *txn = st.col<uint32_t>(st.L.txn);
    uint32_t *ltab = st.col<uint32_t>(st.L.lock_table), *ltxn = st.col<uint32_t>(st.L.lock_txn);
    uint64_t *lsnap = st.col<uint64_t>(st.L.lock_snap);
    // Groups of different key lengths (in words): each part's probes are laid
    // out grouped by that length (stable), so the compact bound kernel's waves
    // skip the zero words past it together, and inside a length the points (lo
    // == hi) after the ranges, so its waves of points map one bound for both.
    // One length: read-set order.
    std::vector<uint8_t> &gcls = c->gcls;  // per dictionary epoch (groups and W fixed by it)
    if (c->gcls_epoch != c->dict_epoch || gcls.size() != c->groups.size()) {
        gcls.resize(c->groups.size());
        for (size_t g = 0; g < c->groups.size(); ++g) gcls[g] = (uint8_t)std::min(W, (c->groups[g].klen + 7) / 8);
        c->gcls_epoch = c->dict_epoch;
    }
    int ncls = 0, cls0 = -1;
    for (size_t g = 0; g < gcls.size(); ++g) {
        if (cls0 < 0) cls0 = gcls[g];
        ncls = std::max(ncls, (int)gcls[g] + 1);
        if (gcls[g] != cls0) cls0 = kMaxWords + 1;
    }
    const bool by_len = cls0 == kMaxWords + 1;
    const auto tp2 = std::chrono::steady_clock::now();
    par_for(c, n >= (size_t)kMarshalParallelMin, nwork, [&](int w) {
        const MarshalPart &mp = c->parts[w];
        const size_t o = mp.out0, k = mp.gid.size();
        if (by_len) {
            size_t cnt[2 * kMaxWords + 4] = {0};
            std::vector<uint8_t> &cls = c->parts_cls[w];
            cls.resize(k);
            for (size_t i = 0; i < k; ++i) {
                const uint64_t *r = &mp.lohi[i * 2 * W];
                const int kc = gcls[mp.gid[i]];
                cls[i] = (uint8_t)(2 * kc + (memcmp(r, r + W, 8 * (size_t)kc) == 0));
                cnt[cls[i] + 1]++;
            }
            for (int q = 1; q <= 2 * ncls; ++q) cnt[q] += cnt[q - 1];
            for (size_t i = 0; i < k; ++i) {
                const size_t d = o + cnt[cls[i]]++;
                for (int j = 0; j < W; ++j) {
                    lo[(size_t)j * n + d] = mp.lohi[i * 2 * W + j];
                    hi[(size_t)j * n + d] = mp.lohi[i * 2 * W + W + j];
                }
                gid[d] = mp.gid[i];
                sn[d] = mp.snap[i];
                txn[d] = mp.txn[i];
            }
        } else {
            // AoS rows -> SoA columns, W unrolled up to 4
            auto cols = [&](auto wt) {
                constexpr int WT = decltype(wt)::value;
                const int Wn = WT ? WT : W;
                const uint64_t *src = mp.lohi.data();
                for (size_t i = 0; i < k; ++i, src += 2 * (size_t)Wn)
                    for (int j = 0; j < Wn; ++j) {
                        lo[(size_t)j * n + o + i] = src[j];
                        hi[(size_t)j * n + o + i] = src[Wn + j];
                    }
            };
            switch (W) {
            case 1: cols(std::integral_constant<int, 1>{}); break;
            case 2: cols(std::integral_constant<int, 2>{}); break;
            case 3: cols(std::integral_constant<int, 3>{}); break;
            case 4: cols(std::integral_constant<int, 4>{}); break;
            default: cols(std::integral_constant<int, 0>{});
            }
            if (k) {
                memcpy(gid + o, mp.gid.data(), 4 * k);
                memcpy(sn + o, mp.snap.data(), 8 * k);
                memcpy(txn + o, mp.txn.data(), 4 * k);
            }
        }
        const size_t lo0 = mp.lock0, kl = mp.lock_table.size();
        if (kl) {
            memcpy(ltab + lo0, mp.lock_table.data(), 4 * kl);
            memcpy(lsnap + lo0, mp.lock_snap.data(), 8 * kl);
            memcpy(ltxn + lo0, mp.lock_txn.data(), 4 * kl);
        }
    }, true);  // static: part w marshalled and assembled on one core
    const auto tp3 = std::chrono::steady_clock::now();
    auto ns = [](auto a, auto b) {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    };
    c->mb_marshals.fetch_add(1, std::memory_order_relaxed);
    c->mb_txns.fetch_add((uint64_t)nt, std::memory_order_relaxed);
    c->mb_ranges.fetch_add(n, std::memory_order_relaxed);
    c->mb_parts_ns.fetch_add(ns(tp0, tp1), std::memory_order_relaxed);
    c->mb_alloc_ns.fetch_add(ns(tp1, tp2), std::memory_order_relaxed);
    c->mb_assemble_ns.fetch_add(ns(tp2, tp3), std::memory_order_relaxed);
    st.n = n;
    st.n_lock = nl;
    st.n_txn = (size_t)nt;
    hsc_marshalled &m = c->m;
    m.n = n;
    m.n_lock = nl;
    m.n_txn = (size_t)nt;
    m.words = W;
    m.lo = lo;
    m.hi = hi;
    m.gid = gid;
    m.snap = sn;
    m.txn = txn;
    m.lock_table = ltab;
    m.lock_snap = lsnap;
    m.lock_txn = ltxn;
    m.forced = forced;
    return HSC_OK;
}

static FlatSrc flat_src(hsc_ctx *c, const hsc_readsets *rs, std::vector<int> &tmap)
{
    tmap.assign(std::max(rs->ntbnames, 0), -1);
    for (int t = 0; t < rs->ntbnames; ++t) {
        auto it = rs->tbnames[t] ? c->table_ids.find(rs->tbnames[t]) : c->table_ids.end();
        if (it != c->table_ids.end()) tmap[t] = it->second;
    }
    return FlatSrc{rs, tmap.data()};
}

static int marshal_readsets(hsc_ctx *c, const hsc_readsets *rs)
{
    std::vector<int> tmap;
    return marshal_into(c, flat_src(c, rs, tmap), 0, rs->ntxn, c->stage[0]);
}

// ---------------------------------------------------------------------------
// device probe
// ---------------------------------------------------------------------------
static WinView win_view(hsc_ctx *c)
{
    WinView w{};
    w.words = c->d_words.as<uint64_t>();
    w.stride = c->cap;
    w.lsn = c->d_lsn.as<uint64_t>();
    w.gid = c->d_gid.as<uint32_t>();
    w.gstart = c->d_gstart.as<uint32_t>();
    w.gend = c->d_gend.as<uint32_t>();
    w.tmax = c->d_tmax.as<uint64_t>();
    w.table_max = c->d_table_max.as<uint64_t>();
    w.sp_g = c->d_sp_g.as<uint32_t>();
    w.sp_w = c->d_sp_w.as<uint64_t>();
    w.n = (uint32_t)c->n;
    w.ntiles = c->ntiles;
    w.ntables = (uint32_t)c->table_names.size();
    w.W = c->W;
    w.log2T = c->log2T;
    w.levels = c->levels;
    w.gbits = 0;
    while (w.gbits < 32 && ((size_t)1 << w.gbits) < c->groups.size()) w.gbits++;
    return w;
}

static int probe_delta(hsc_ctx *c, uint8_t *target);
// the batch's delta probe will mark verdict bytes (then a pack pass builds the bitmap)
static bool pack_after_delta(const hsc_ctx *c) { return c->raw_probe.n && (c->fn || c->dn); }

// Narrow layout: one kernel answers every range and table lock.
static int probe_narrow(hsc_ctx *c, const hsc_probe_batch *b, const WinView &w,
                        const ProbeView &p)
{
    hipStream_t s = c->stream;
    NarrowView nv = c->nv;
    nv.table_max = w.table_max;
    nv.ntables = w.ntables;
    const bool tm = c->timing;
    if (tm)
        for (int i = 0; i < 6; ++i)
            if (!c->ev[i]) HIPCHK(c, hipEventCreate(&c->ev[i]));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[0], s));
    if (b->n_txn) HIPCHK(c, hipMemsetAsync(b->verdict, 0, b->n_txn, s));
    // timing slots: locate = verdict clear, plan = scatter = 0, join = the probe
    if (tm)
        for (int i = 1; i <= 3; ++i) HIPCHK(c, hipEventRecord(c->ev[i], s));
    HIPCHK(c, launch_probe_narrow(nv, p, b->verdict, s));
    HIPCHK_RC(c, probe_delta(c, b->verdict));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[4], s));
    HIPCHK(c, launch_pack(b->verdict, (uint32_t)b->n_txn, b->bitmap, s));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[5], s));
    return HSC_OK;
}

static int probe_tiles(hsc_ctx *c, const hsc_probe_batch *b, const WinView &w, const ProbeView &p,
                       bool started = false);

#ifdef HSC_STAMPS
// Diagnostic builds: phase durations of the locate (np0 stamps) and the join
// (np1 stamps), median over blocks, in shader cycles; clears the stamps.
static int stamp_report(hsc_ctx *c, const ProbeWork &work, uint32_t max_items, int np0, int np1)
{
    hipStream_t s = c->stream;
    if (!work.stamps) return HSC_OK;
    std::vector<uint64_t> h(2 * 8192 * 8);
    HIPCHK(c, hipMemcpyAsync(h.data(), work.stamps, 8 * h.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint32_t nb[2] = {8 * ((work.G + 7) / 8), max_items};
    const int np[2] = {np0, np1};
    for (int k = 0; k < 2; ++k) {
        fprintf(stderr, "[stamps] %s blocks %u:", k ? "join" : "locate", nb[k]);
        uint64_t t0 = ~0ull, t1 = 0;
        for (uint32_t b = 0; b < nb[k] && b < 8192; ++b) {
            const uint64_t *r = &h[((size_t)k * 8192 + b) * 8];
            if (!r[0]) continue;
            t0 = std::min(t0, r[0]);
            t1 = std::max(t1, r[np[k] - 1]);
        }
        for (int q = 1; q < np[k]; ++q) {
            std::vector<uint64_t> d;
            for (uint32_t b = 0; b < nb[k] && b < 8192; ++b) {
                const uint64_t *r = &h[((size_t)k * 8192 + b) * 8];
                if (r[q] && r[q - 1]) d.push_back(r[q] - r[q - 1]);
            }
            std::sort(d.begin(), d.end());
            fprintf(stderr, " p%d %llu", q, d.empty() ? 0ull : (unsigned long long)d[d.size() / 2]);
        }
        std::vector<uint64_t> st;
        for (uint32_t b = 0; b < nb[k] && b < 8192; ++b) {
            const uint64_t *r = &h[((size_t)k * 8192 + b) * 8];
            if (r[0]) st.push_back(r[0] - t0);
        }
        std::sort(st.begin(), st.end());
        fprintf(stderr, " | span %llu, start p50 %llu p90 %llu\n", (unsigned long long)(t1 - t0),
                st.empty() ? 0ull : (unsigned long long)st[st.size() / 2],
                st.empty() ? 0ull : (unsigned long long)st[st.size() * 9 / 10]);
    }
    HIPCHK(c, hipMemsetAsync(work.stamps, 0, 8 * h.size(), s));
    return HSC_OK;
}

static DBuf &stamp_buffer()
{
    static DBuf b;
    return b;
}
#endif

// Narrow tiles (dense batch): locate (codes, snapshot ranks, per-chunk tile
// histograms) -> column scan + plan -> scatter (16-byte records) -> join
// (8-byte rows) -> pack.
static int probe_ntiles(hsc_ctx *c, const hsc_probe_batch *b, const WinView &wn,
                        const ProbeView &p)
{
    hipStream_t s = c->stream;
    c->probe_ntiles = wn.ntiles;
    c->probe_buckets = true;
    const uint32_t nt = std::max<uint32_t>(wn.ntiles, 1);
    ProbeWork work{};
    work.lds_mode = 1;
    const size_t nwork = std::max<size_t>(p.n, p.n_lock);
    // chunks of narrow_tiles_chunk() probes (at most kMaxChunks: the caller
    // sends larger batches down the code-tile path)
    work.chunk = narrow_tiles_chunk();
    work.G = (uint32_t)std::max<size_t>(1, (nwork + work.chunk - 1) / work.chunk);
    const size_t n1 = std::max<uint32_t>(p.n, 1);
    HIPCHK(c, c->w_hist.ensure(4 * (size_t)hist_stride(work.G) * nt));
    // tile buckets of kTileCap records, then the overflow area (at most 2n
    // records spill); join items: one per tile + the overflow chunks (each hot
    // tile rounds its own run up: at most 2 ceil(2n / kJoinChunk) of them)
    HIPCHK(c, c->w_counts.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_bucket.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_items.ensure(4 * std::max<size_t>((size_t)nt + 1, 4)));
    const uint32_t extra_items = 2 * (uint32_t)((2 * n1 + kJoinChunk - 1) / kJoinChunk);
    const uint32_t max_items = nt + extra_items;
    HIPCHK(c, c->w_item_desc.ensure(16 * (size_t)extra_items + 16));
    // chunk-sorted records: each chunk's records in an area of its own, tile
    // runs found by the join through the plan's scan (no scatter pass)
    HIPCHK(c, c->w_tcode2.ensure(2 * (size_t)hist_stride(work.G) * nt));  // cst
    HIPCHK(c, c->w_tcode.ensure(4 * (size_t)work.G * ((nt + 3) & ~3u)));  // chunk-major rows
    HIPCHK(c, c->w_trecs.ensure(16 * 2 * (size_t)work.chunk * work.G));
    work.cst = c->w_tcode2.as<uint16_t>();
    work.cm = c->w_tcode.as<uint32_t>();
    work.hist = c->w_hist.as<uint32_t>();
    work.counts = c->w_counts.as<uint32_t>();
    work.bucket_off = c->w_bucket.as<uint32_t>();
    work.cursor = c->w_cursor.as<uint32_t>();
    work.item_off = c->w_items.as<uint32_t>();
    work.item_tile = c->w_item_tile.as<uint32_t>();
    work.item_desc = c->w_item_desc.as<uint4>();
#ifdef HSC_STAMPS
    DBuf &stamp_buf = stamp_buffer();
    if (getenv("HSC_STAMPS")) {
        if (!stamp_buf.p) {
            HIPCHK(c, stamp_buf.ensure(8 * 2 * 8192 * 8));
            HIPCHK(c, hipMemsetAsync(stamp_buf.p, 0, 8 * 2 * 8192 * 8, s));
        }
        work.stamps = stamp_buf.as<uint64_t>();
    }
#endif
    NarrowTiles ntl{};
    ntl.key32 = c->d_key32.as<uint32_t>();
    ntl.rank32 = c->d_rank32.as<uint32_t>();
    ntl.rank_lsn32 = c->rank_lsn32;
    ntl.rank_base = c->rank_base;
    ntl.cdir = c->cdir;
    ntl.tdir = c->tdir;
    ntl.trad = c->trad_m ? c->d_trad.as<uint32_t>() : nullptr;
    ntl.trad_m = c->trad_m;
    ntl.recs = c->w_trecs.as<uint4>();
    // conflict flags: internal, all zero between batches (the pack clears them)
    const size_t had = c->w_vflags.bytes;
    HIPCHK(c, c->w_vflags.ensure((std::max<size_t>(b->n_txn, 1) + 15) & ~(size_t)15));
    if (c->w_vflags.bytes != had) HIPCHK(c, hipMemsetAsync(c->w_vflags.p, 0, c->w_vflags.bytes, s));
    uint8_t *flags = c->w_vflags.as<uint8_t>();
    const bool tm = c->timing;
    if (tm)
        for (int i = 0; i < 6; ++i)
            if (!c->ev[i]) HIPCHK(c, hipEventCreate(&c->ev[i]));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[0], s));
    HIPCHK(c, launch_locate_t(c->nv, wn, p, work, ntl, flags, s));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[1], s));
    if (p.n && wn.ntiles) {
        // the plan writes the verdict bytes (and bitmap words) from the
        // locate's flags; the join and the delta probe then mark the verdict
        // itself, the join its bitmap bits too (no pack pass unless the delta
        // probe ran: it marks bytes only)
        const bool delta = pack_after_delta(c);
        work.bitmap = delta ? nullptr : b->bitmap;
        HIPCHK(c, launch_plan_s(work, wn.ntiles, c->w_items.as<uint32_t>(), s, flags,
                                (uint32_t)b->n_txn, b->verdict));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[2], s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[3], s));
        // blocks past the tiles for the hot tiles' overflow items: 512, or 2048
        // on a skewed window (the bucket table took log mode: Zipf keys crowd
        // a few tiles -- r03: config 5 one stream 83 -> 80 us with 2048, while
        // config 2's idle extra blocks cost its overlapped batch); diagnostics:
        // HSC_JOIN_EXTRA
        static const int extra_env = getenv("HSC_JOIN_EXTRA") ? atoi(getenv("HSC_JOIN_EXTRA")) : 0;
        const uint32_t extra = extra_env > 0 ? (uint32_t)extra_env : c->trad_log ? 2048u : 512u;
        HIPCHK(c, launch_join_t(work, ntl, wn.n, wn.ntiles, max_items, b->verdict, s, extra));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[4], s));
        HIPCHK_RC(c, probe_delta(c, b->verdict));
        if (delta) HIPCHK(c, launch_pack(b->verdict, (uint32_t)b->n_txn, b->bitmap, s));
    } else {
        if (tm)
            for (int i = 2; i <= 4; ++i) HIPCHK(c, hipEventRecord(c->ev[i], s));
        HIPCHK_RC(c, probe_delta(c, flags));
        HIPCHK(c, launch_pack_flags(flags, (uint32_t)b->n_txn, b->verdict, b->bitmap, s));
    }
    if (tm) HIPCHK(c, hipEventRecord(c->ev[5], s));
#ifdef HSC_STAMPS
    HIPCHK_RC(c, stamp_report(c, work, max_items, 6, 4));
#endif
    return HSC_OK;
}

// Compact tiles (dense or sparse batch over a compact window): code bounds
// (compact_probes) -> locate (gid || code keys, end tiles, 64-byte probe
// entries) -> plan -> scatter (4-byte bucket entries) -> join -> pack.
static int probe_ctiles(hsc_ctx *c, const hsc_probe_batch *b, const ProbeView &p)
{
    hipStream_t s = c->stream;
    const WinView w = win_view(c);
    CTiles ct = c->ctv;
    c->probe_ntiles = ct.ntiles;
    c->probe_buckets = true;
    const uint32_t nt = std::max<uint32_t>(ct.ntiles, 1);
    ProbeWork work{};
    work.lds_mode = 1;
    work.chunk = ctiles_chunk();
    work.G = (uint32_t)std::max<size_t>(1, (std::max<size_t>(p.n, p.n_lock) + work.chunk - 1) / work.chunk);
    const size_t n1 = std::max<uint32_t>(p.n, 1);
    const int WC = c->ct.WC;
    HIPCHK(c, c->p_code_lo.ensure(8 * (size_t)WC * n1));
    HIPCHK(c, c->p_code_hi.ensure(8 * (size_t)WC * n1));
    HIPCHK(c, c->w_hist.ensure(4 * (size_t)hist_stride(work.G) * nt));
    HIPCHK(c, c->w_counts.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_bucket.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_items.ensure(4 * std::max<size_t>((size_t)nt + 1, 4)));
    const uint32_t extra_items = 2 * (uint32_t)((2 * n1 + kJoinChunk - 1) / kJoinChunk);
    const uint32_t max_items = nt + extra_items;
    HIPCHK(c, c->w_item_desc.ensure(16 * (size_t)extra_items + 16));
    // chunk-sorted 64-byte records (the read set number shares its word with
    // the record kind: the caller sends batches of >= 2^30 read sets down the
    // wide pipeline)
    HIPCHK(c, c->w_tcode.ensure(4 * (size_t)work.G * ((nt + 3) & ~3u)));  // chunk-major rows
    HIPCHK(c, c->w_tcode2.ensure(2 * (size_t)hist_stride(work.G) * nt));  // run starts
    HIPCHK(c, c->w_trecs.ensure(64 * 2 * (size_t)work.chunk * work.G));
    work.cm = c->w_tcode.as<uint32_t>();
    work.cst = c->w_tcode2.as<uint16_t>();
    work.hist = c->w_hist.as<uint32_t>();
    work.counts = c->w_counts.as<uint32_t>();
    work.bucket_off = c->w_bucket.as<uint32_t>();
    work.item_off = c->w_items.as<uint32_t>();
    work.item_desc = c->w_item_desc.as<uint4>();
    ct.recs = c->w_trecs.as<uint32_t>();
    ct.np = p.n;
#ifdef HSC_STAMPS
    DBuf &stamp_buf = stamp_buffer();
    if (getenv("HSC_STAMPS")) {
        if (!stamp_buf.p) {
            HIPCHK(c, stamp_buf.ensure(8 * 2 * 8192 * 8));
            HIPCHK(c, hipMemsetAsync(stamp_buf.p, 0, 8 * 2 * 8192 * 8, s));
        }
        work.stamps = stamp_buf.as<uint64_t>();
    }
#endif
    static const int dbg = getenv("HSC_CT_DBG") ? atoi(getenv("HSC_CT_DBG")) : 0;
    ct.dbg = dbg;
    const size_t had = c->w_vflags.bytes;
    HIPCHK(c, c->w_vflags.ensure((std::max<size_t>(b->n_txn, 1) + 15) & ~(size_t)15));
    if (c->w_vflags.bytes != had) HIPCHK(c, hipMemsetAsync(c->w_vflags.p, 0, c->w_vflags.bytes, s));
    uint8_t *flags = c->w_vflags.as<uint8_t>();
    WinView wt = c->wc;  // tile maxima of the same 2048-row tiles
    wt.table_max = w.table_max;
    wt.ntables = w.ntables;
    const bool tm = c->timing;
    if (tm)
        for (int i = 0; i < 6; ++i)
            if (!c->ev[i]) HIPCHK(c, hipEventCreate(&c->ev[i]));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[0], s));
    // (measured: the bound mapping fused into the locate -- code bounds kept in
    // registers -- ran 83 us against 67 us for the two kernels on config 3)
    PointHash ph{};
    if (c->cph_nb) {
        ph.e = c->d_cph.as<uint64_t>();
        ph.nb = c->cph_nb;
        ph.WG = ct.WG;
        ph.gb = ct.gb;
        ph.rank_base = ct.rank_base;
        ph.flags = flags;
        ph.ep = c->cph_ep;
    }
    if (p.n)
        HIPCHK(c, compact_probes(p, c->ct, c->p_code_lo.as<uint64_t>(), c->p_code_hi.as<uint64_t>(), s, &ph));
    HIPCHK(c, launch_locate_c(ct, wt, p, c->p_code_lo.as<uint64_t>(), c->p_code_hi.as<uint64_t>(),
                              work, flags, s));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[1], s));
    if (p.n && ct.ntiles) {
        // verdict bytes and bitmap from the plan and the join, as probe_ntiles
        const bool delta = pack_after_delta(c);
        work.bitmap = delta ? nullptr : b->bitmap;
        HIPCHK(c, launch_plan_s(work, ct.ntiles, c->w_items.as<uint32_t>(), s, flags,
                                (uint32_t)b->n_txn, b->verdict));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[2], s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[3], s));
        HIPCHK(c, launch_join_c(ct, work, max_items, b->verdict, s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[4], s));
        HIPCHK_RC(c, probe_delta(c, b->verdict));
        if (delta) HIPCHK(c, launch_pack(b->verdict, (uint32_t)b->n_txn, b->bitmap, s));
    } else {
        if (tm)
            for (int i = 2; i <= 4; ++i) HIPCHK(c, hipEventRecord(c->ev[i], s));
        HIPCHK_RC(c, probe_delta(c, flags));
        HIPCHK(c, launch_pack_flags(flags, (uint32_t)b->n_txn, b->verdict, b->bitmap, s));
    }
    if (tm) HIPCHK(c, hipEventRecord(c->ev[5], s));
#ifdef HSC_STAMPS
    HIPCHK_RC(c, stamp_report(c, work, max_items, 2, 7));
#endif
    return HSC_OK;
}

static int probe_lane(hsc_ctx *c, const hsc_probe_batch *b);
static int probe(hsc_ctx *c, const hsc_probe_batch *b)
{
    if (c->host_only) return fail(c, HSC_EDEVICE, "host-only context");
    if (c->pend_n || c->pend_t) HIPCHK_RC(c, flush_appends(c));  // the pending tail is k_small_narrow's only
    HIPCHK(c, select_lane(c));
    const int rc = probe_lane(c, b);
    // the lane's done event fences whatever probe_lane launched, also when it
    // failed part way: a later take-over of the lane or a window rebuild from
    // another stream waits on it before touching the lane's scratch; it is
    // recorded when the context leaves this stream (ctx_switch_stream)
    lane_mark(c);
    return rc;
}

// Range probes of the batch against the delta run (appends since the last
// build) into the path's verdict target, before its pack.
static int probe_delta(hsc_ctx *c, uint8_t *target)
{
    if (!c->raw_probe.n) return HSC_OK;
    if (c->fn) HIPCHK(c, launch_probe_delta(frozen_view(c), c->raw_probe, target, c->stream));
    if (c->dn) HIPCHK(c, launch_probe_delta(delta_view(c), c->raw_probe, target, c->stream));
    return HSC_OK;
}

static int probe_lane(hsc_ctx *c, const hsc_probe_batch *b)
{
    const WinView w = win_view(c);
    if (b->n > 0xFFFFFFFFull / 2 || b->n_lock > 0xFFFFFFFFull || b->n_txn > 0xFFFFFFFFull)
        return fail(c, HSC_EINVAL, "batch too large");
    ProbeView p{};
    p.lo = b->lo;
    p.hi = b->hi;
    p.gid = b->gid;
    p.snap = b->snap;
    p.txn = b->txn;
    p.lock_table = b->lock_table;
    p.lock_snap = b->lock_snap;
    p.lock_txn = b->lock_txn;
    p.n = w.n ? (uint32_t)b->n : 0;  // empty key window: no range can match
    p.n_lock = (uint32_t)b->n_lock;
    c->raw_probe = p;
    c->raw_probe.n = (uint32_t)b->n;  // the delta may hold keys of an empty main window
    // compact tiles for dense batches; a sparse one (fewer than kDirectPerTile
    // ranges per tile) takes the wide pipeline, which stages only the tiles
    // its ranges reach (the compact-tile join stages every tile)
    if (!c->narrow && c->compact && c->ctiles && c->layout != HSC_LAYOUT_COMPACT_WIDE &&
        p.n < (1u << 30) && b->n_txn < (1u << 30) && (size_t)p.n >= kDirectPerTile * (size_t)c->ctv.ntiles &&
        (std::max<size_t>(p.n, p.n_lock) + ctiles_chunk() - 1) / ctiles_chunk() <= (size_t)kMaxChunks)
        return probe_ctiles(c, b, p);
    if (!c->narrow && c->compact) {
        // wide keys as compact codes: map the bounds, then the tile pipeline
        const int WC = c->ct.WC;
        const size_t n = std::max<uint32_t>(p.n, 1);
        HIPCHK(c, c->p_code_lo.ensure(8 * (size_t)WC * n));
        HIPCHK(c, c->p_code_hi.ensure(8 * (size_t)WC * n));
        if (c->timing) {
            if (!c->ev[0]) HIPCHK(c, hipEventCreate(&c->ev[0]));
            HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
        }
        HIPCHK(c, compact_probes(p, c->ct, c->p_code_lo.as<uint64_t>(), c->p_code_hi.as<uint64_t>(),
                                 c->stream));
        ProbeView pc = p;
        pc.lo = c->p_code_lo.as<uint64_t>();
        pc.hi = c->p_code_hi.as<uint64_t>();
        WinView wc = c->wc;
        wc.table_max = w.table_max;
        wc.ntables = w.ntables;
        wc.gbits = w.gbits;
        return probe_tiles(c, b, wc, pc, c->timing);
    }
    if (!c->narrow) return probe_tiles(c, b, w, p);
    // narrow window: a sparse batch is answered by the direct probe; a dense
    // one maps its bounds to codes and runs the tile pipeline on the codes
    const bool direct = c->layout == HSC_LAYOUT_NARROW_DIRECT ||
                        (c->layout != HSC_LAYOUT_NARROW_TILES &&
                         (size_t)p.n < kDirectPerTile * (size_t)c->wn.ntiles);
    if (direct) {
        c->probe_ntiles = 0;
        return probe_narrow(c, b, w, p);
    }
    WinView wn = c->wn;
    wn.table_max = w.table_max;
    wn.ntables = w.ntables;
    // 8-byte tile rows when they fit and the batch fits one column scan
    const size_t nchunks = (std::max<size_t>(p.n, p.n_lock) + narrow_tiles_chunk() - 1) /
                           narrow_tiles_chunk();
    if (c->ntiles32 && c->layout != HSC_LAYOUT_NARROW_CODES && nchunks <= (size_t)kMaxChunks)
        return probe_ntiles(c, b, wn, p);
    const size_t n = std::max<uint32_t>(p.n, 1);
    HIPCHK(c, c->p_code_lo.ensure(8 * n));
    HIPCHK(c, c->p_code_hi.ensure(8 * n));
    const size_t zb = c->p_zero.bytes;
    HIPCHK(c, c->p_zero.ensure(4 * n));
    if (c->p_zero.bytes != zb) HIPCHK(c, hipMemsetAsync(c->p_zero.p, 0, c->p_zero.bytes, c->stream));
    NarrowView nv = c->nv;
    HIPCHK(c, narrow_codes(nv, p, c->p_code_lo.as<uint64_t>(), c->p_code_hi.as<uint64_t>(),
                           c->stream));
    ProbeView pn = p;
    pn.lo = c->p_code_lo.as<uint64_t>();
    pn.hi = c->p_code_hi.as<uint64_t>();
    pn.gid = c->p_zero.as<uint32_t>();
    return probe_tiles(c, b, wn, pn);
}

// The tile pipeline: locate -> plan -> scatter -> join -> pack.
// started: ev[0] was recorded by the caller (a bound transform before locate
// counts as locate time).
static int probe_tiles(hsc_ctx *c, const hsc_probe_batch *b, const WinView &w, const ProbeView &p,
                       bool started)
{
    hipStream_t s = c->stream;
    c->probe_ntiles = w.ntiles;
    c->probe_buckets = false;
    const uint32_t nt = std::max<uint32_t>(w.ntiles, 1);
    ProbeWork work{};
    work.lds_mode = w.ntiles <= (uint32_t)kHistCap;
    const size_t nwork = std::max<size_t>(p.n, p.n_lock);
    work.G = (uint32_t)std::min<size_t>(kMaxChunks, std::max<size_t>(1, (nwork + 2047) / 2048));
    work.chunk = (uint32_t)((p.n + work.G - 1) / work.G);
    HIPCHK(c, c->w_code.ensure(8 * (size_t)std::max<uint32_t>(p.n, 1)));
    HIPCHK(c, c->w_hist.ensure(4 * (size_t)work.G * nt));
    HIPCHK(c, c->w_counts.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_bucket.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_cursor.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_items.ensure(4 * ((size_t)nt + 1)));
    HIPCHK(c, c->w_recs.ensure(8 * (size_t)rec_stride(w.W) * 2 * std::max<uint32_t>(p.n, 1)));
    const uint32_t max_items = nt + (uint32_t)((2 * (size_t)p.n + kJoinChunk - 1) / kJoinChunk);
    HIPCHK(c, c->w_item_tile.ensure(4 * (size_t)max_items + 16));
    HIPCHK(c, c->w_item_desc.ensure(16 * (size_t)max_items + 16));
    work.item_desc = c->w_item_desc.as<uint4>();
    work.code = c->w_code.as<uint64_t>();
    work.hist = c->w_hist.as<uint32_t>();
    work.counts = c->w_counts.as<uint32_t>();
    work.bucket_off = c->w_bucket.as<uint32_t>();
    work.cursor = c->w_cursor.as<uint32_t>();
    work.item_off = c->w_items.as<uint32_t>();
    work.item_tile = c->w_item_tile.as<uint32_t>();
    work.recs = c->w_recs.as<uint64_t>();
    const bool tm = c->timing;
    if (tm)
        for (int i = 0; i < 6; ++i)
            if (!c->ev[i]) HIPCHK(c, hipEventCreate(&c->ev[i]));
    if (tm && !started) HIPCHK(c, hipEventRecord(c->ev[0], s));
    if (b->n_txn) HIPCHK(c, hipMemsetAsync(b->verdict, 0, b->n_txn, s));
    if (!work.lds_mode) HIPCHK(c, hipMemsetAsync(c->w_counts.p, 0, 4 * ((size_t)nt + 1), s));
    HIPCHK(c, launch_locate(w, p, work, b->verdict, s));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[1], s));
    if (p.n && w.ntiles) {
        HIPCHK(c, launch_plan(w, work, s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[2], s));
        HIPCHK(c, launch_scatter(w, p, work, s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[3], s));
        HIPCHK(c, launch_join(w, work, max_items, b->verdict, s));
        if (tm) HIPCHK(c, hipEventRecord(c->ev[4], s));
    } else if (tm) {
        HIPCHK(c, hipEventRecord(c->ev[2], s));
        HIPCHK(c, hipEventRecord(c->ev[3], s));
        HIPCHK(c, hipEventRecord(c->ev[4], s));
    }
    HIPCHK_RC(c, probe_delta(c, b->verdict));
    HIPCHK(c, launch_pack(b->verdict, (uint32_t)b->n_txn, b->bitmap, s));
    if (tm) HIPCHK(c, hipEventRecord(c->ev[5], s));
    return HSC_OK;
}

static int collect_timing(hsc_ctx *c)
{
    if (!c->timing || !c->ev[5]) return HSC_OK;
    HIPCHK(c, hipEventSynchronize(c->ev[5]));
    float t[5];
    for (int i = 0; i < 5; ++i) (void)hipEventElapsedTime(&t[i], c->ev[i], c->ev[i + 1]);
    c->last.locate_ms = t[0];
    c->last.plan_ms = t[1];
    c->last.scatter_ms = t[2];
    c->last.join_ms = t[3];
    c->last.pack_ms = t[4];
    (void)hipEventElapsedTime(&c->last.probe_total_ms, c->ev[0], c->ev[5]);
    uint64_t nrec = 0;
    if (c->probe_ntiles && c->w_counts.p && c->probe_buckets) {  // per-tile record counts
        std::vector<uint32_t> cnt(c->probe_ntiles);
        HIPCHK(c, hipMemcpy(cnt.data(), c->w_counts.p, 4 * cnt.size(), hipMemcpyDeviceToHost));
        for (uint32_t v : cnt) nrec += v;
    } else if (c->probe_ntiles && c->w_bucket.p) {
        uint32_t r = 0;
        HIPCHK(c, hipMemcpy(&r, c->w_bucket.as<uint32_t>() + c->probe_ntiles, 4, hipMemcpyDeviceToHost));
        nrec = r;
    }
    c->last.records = nrec;
    c->last.tiles = c->probe_ntiles;  // tiles of the view the last probe joined over
    return HSC_OK;
}

// Upload staging set st (pinned), run the join, download the verdict bytes
// into st.verdict -- all asynchronous on c->stream; st.done marks the end.
static int launch_stage(hsc_ctx *c, Stage &st)
{
    if (c->host_only) return fail(c, HSC_EDEVICE, "host-only context");
    hipStream_t s = c->stream;
    HIPCHK(c, c->p_arena.ensure(std::max<size_t>(st.L.total, 256)));
    HIPCHK(c, c->p_verdict.ensure(std::max<size_t>(st.n_txn, 1)));
    if (st.verdict.ensure(std::max<size_t>(st.n_txn, 1), true)) return fail(c, HSC_ENOMEM, "staging");
    if (st.n || st.n_lock)  // every column in one transfer
        HIPCHK(c, hipMemcpyAsync(c->p_arena.p, st.arena.p, st.L.total, hipMemcpyHostToDevice, s));
    auto dcol = [&](size_t off) { return (void *)((uint8_t *)c->p_arena.p + off); };
    hsc_probe_batch b{};
    b.n = st.n;
    b.lo = (const uint64_t *)dcol(st.L.lo);
    b.hi = (const uint64_t *)dcol(st.L.hi);
    b.gid = (const uint32_t *)dcol(st.L.gid);
    b.snap = (const uint64_t *)dcol(st.L.snap);
    b.txn = (const uint32_t *)dcol(st.L.txn);
    b.n_lock = st.n_lock;
    b.lock_table = (const uint32_t *)dcol(st.L.lock_table);
    b.lock_snap = (const uint64_t *)dcol(st.L.lock_snap);
    b.lock_txn = (const uint32_t *)dcol(st.L.lock_txn);
    b.n_txn = st.n_txn;
    b.verdict = c->p_verdict.as<uint8_t>();
    b.bitmap = nullptr;
    const int rc = probe(c, &b);
    if (rc) return rc;
    if (st.n_txn)
        HIPCHK(c, hipMemcpyAsync(st.verdict.p, c->p_verdict.p, st.n_txn, hipMemcpyDeviceToHost, s));
    if (!st.done) HIPCHK(c, hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(st.done, s));
    return HSC_OK;
}

// Wait for st's download; rc_out[t] = forced | device verdict.
static int finish_stage(hsc_ctx *c, Stage &st, int *rc_out)
{
    HIPCHK(c, hipEventSynchronize(st.done));
    const uint8_t *f = st.forced.as<uint8_t>(), *v = st.verdict.as<uint8_t>();
    for (size_t t = 0; t < st.n_txn; ++t) rc_out[t] = (f[t] | v[t]) ? 1 : 0;
    return HSC_OK;
}

// Small batches (a lone bdb_osql_serial_check, a collector's batch): one
// k_small_narrow launch reads the marshalled columns from fine-grained pinned
// memory and writes the verdict bytes into it, and the host polls the
// kernel's done word -- no copies, no event (the per-call
// latency db/toblock.c:4779-4836 sees).  Narrow windows (the direct probe's
// key and max trees); hsc_set_paths(HSC_PATH_NO_SMALL) turns it off.
constexpr int kSmallMaxTxns = 1024;
constexpr size_t kSmallMaxRanges = 16384;

static bool small_path(hsc_ctx *c, int T)
{
    // a layout forced to the tile or code pipeline (tests, A/B) keeps it
    const bool direct_ok = c->layout == HSC_LAYOUT_AUTO || c->layout == HSC_LAYOUT_NARROW ||
                           c->layout == HSC_LAYOUT_NARROW_DIRECT;
    return !c->no_small && c->narrow && direct_ok && !c->timing && T <= kSmallMaxTxns && c->n > 0 &&
           c->nv.levels <= kSmallMaxLevels;
}

using SteadyClock = std::chrono::steady_clock;
static uint64_t ns_since(SteadyClock::time_point t0)
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(SteadyClock::now() - t0).count();
}

// Under c->mu: copy the marshalled batch st into a free slot and launch its
// kernel on c->stream.  With every slot taken, wait for the oldest launch's
// owner to release it (owners release without c->mu, so this cannot block
// them).  -> slot index, or < 0 (an HSC_ error code, already recorded).
static int small_launch(hsc_ctx *c, Stage &st)
{
    // the lowest free slot; with every slot taken, the oldest launch's
    int k = -1;
    for (int i = 0; i < hsc_ctx::kSmallSlots && k < 0; ++i)
        if (!c->small[i].busy.load(std::memory_order_acquire)) k = i;
    if (k < 0) {
        c->sm_slot_waits.fetch_add(1, std::memory_order_relaxed);
        k = 0;
        for (int i = 1; i < hsc_ctx::kSmallSlots; ++i)
            if ((int32_t)(c->small[i].seq - c->small[k].seq) < 0) k = i;
        const auto t0 = SteadyClock::now();
        while (c->small[k].busy.load(std::memory_order_acquire)) {
            __builtin_ia32_pause();
            if (SteadyClock::now() - t0 > std::chrono::seconds(60))
                return fail(c, HSC_EDEVICE, "small-batch slot not released within 60 s");
        }
    }
    hsc_ctx::SmallSlot &sl = c->small[k];
    sl.vo = (st.L.total + 63) & ~(size_t)63;
    sl.dn = (sl.vo + st.n_txn + 63) & ~(size_t)63;
    sl.n_txn = st.n_txn;
    // the columns stay where the marshal wrote them: the stage's arena becomes
    // the slot's, the slot's old buffer the stage's next arena
    if (!st.arena.coherent || st.arena.bytes < sl.dn + 64)
        return fail(c, HSC_EINVAL, "small batch marshalled outside the small stage");
    std::swap(sl.io, st.arena);
    HIPCHK(c, c->small_blocks.ensure(64 * hsc_ctx::kSmallSlots));
    if (!c->small_side[k]) HIPCHK(c, create_stream(&c->small_side[k], true));
    hipStream_t s = c->small_side[k];
    sl.wait_ev = nullptr;
    if (c->app_last && c->small_app_seq[k] != c->app_seq) {  // after the appends' device work
        sl.wait_ev = c->app_last;  // not re-recorded while a slot is busy (wait_small)
        c->small_app_seq[k] = c->app_seq;
    }
    sl.stream = s;
    if (!c->small_blocks_zeroed) {  // every slot's counters, before any slot's first launch
        HIPCHK(c, hipMemsetAsync(c->small_blocks.p, 0, 64 * hsc_ctx::kSmallSlots, s));
        HIPCHK(c, hipStreamSynchronize(s));
        c->small_blocks_zeroed = true;
    }
    uint8_t *io = sl.io.as<uint8_t>(), *dio = (uint8_t *)sl.io.dp;
    memset(io + sl.vo, 0, st.n_txn);
    sl.forced.assign(st.forced.as<uint8_t>(), st.forced.as<uint8_t>() + st.n_txn);
    volatile uint64_t *done = (volatile uint64_t *)(io + sl.dn);
    if (++c->small_seq == 0) c->small_seq = 1;
    sl.seq = c->small_seq;
    *done = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    ProbeView &p = sl.p;
    p = ProbeView{};
    p.lo = (const uint64_t *)(dio + st.L.lo);
    p.hi = (const uint64_t *)(dio + st.L.hi);
    p.gid = (const uint32_t *)(dio + st.L.gid);
    p.snap = (const uint64_t *)(dio + st.L.snap);
    p.txn = (const uint32_t *)(dio + st.L.txn);
    p.lock_table = (const uint32_t *)(dio + st.L.lock_table);
    p.lock_snap = (const uint64_t *)(dio + st.L.lock_snap);
    p.lock_txn = (const uint32_t *)(dio + st.L.lock_txn);
    p.n = (uint32_t)st.n;
    p.n_lock = (uint32_t)st.n_lock;
    static const bool empty = getenv("HSC_SMALL_EMPTY") != nullptr;  // diagnostics: the
    if (empty) p.n = p.n_lock = 0;  // launch + done-word floor (verdicts all 0: wrong answers)
    sl.nv = c->nv;
    sl.nv.table_max = c->d_table_max.as<uint64_t>();
    // tables past nt_dev have their maxima in the pending tail only
    sl.nv.ntables = std::min((uint32_t)c->table_names.size(), c->nt_dev);
    sl.d = c->dn ? delta_view(c) : DeltaView{};
    sl.d2 = c->fn ? frozen_view(c) : DeltaView{};
    sl.pd = PendView{};
    if (c->pend_n || c->pend_t) {
        sl.pd.base = (const uint8_t *)c->h_pend[c->pend_i].dp;
        sl.pd.n = c->pend_n;
        sl.pd.nt = c->pend_t;
    }
    // busy before the lock is dropped: a window change waits for the slot
    // (wait_small), so what the captured views point at stays as it is until
    // the kernel finished
    sl.busy.store(true, std::memory_order_release);
    return k;
}

// The launch of slot k (prepared by small_launch), without c->mu.
static hipError_t small_fire(hsc_ctx *c, int k)
{
    hsc_ctx::SmallSlot &sl = c->small[k];
    if (sl.wait_ev) {
        const hipError_t e = hipStreamWaitEvent(sl.stream, sl.wait_ev, 0);
        if (e != hipSuccess) return e;
    }
    uint8_t *dio = (uint8_t *)sl.io.dp;
    return launch_small_narrow(sl.nv, sl.d, sl.d2, sl.pd, sl.p, dio + sl.vo,
                               c->small_blocks.as<uint32_t>() + 16 * k, (uint64_t *)(dio + sl.dn), sl.seq,
                               sl.n_txn <= kSmallPackTxns, sl.stream);
}

// Without c->mu: poll slot k's done word (every few thousand spins ask the
// stream whether it failed: a fault never releases the word), read the
// verdicts, release the slot.  Errors come back as (code, message) for the
// caller to record under c->mu.
static int small_wait(hsc_ctx *c, int k, hipStream_t s, int *rc_out, const char **why,
                      hipError_t *herr)
{
    hsc_ctx::SmallSlot &sl = c->small[k];
    const uint8_t *io = sl.io.as<uint8_t>();
    volatile const uint64_t *done = (volatile const uint64_t *)(io + sl.dn);
    const uint32_t seq = sl.seq;
    const auto t0 = SteadyClock::now();
    int rc = HSC_OK;
    bool running = false;  // timed out: the kernel may still write the slot
    for (uint32_t spin = 1; (uint32_t)(*done >> 32) != seq; ++spin) {
        __builtin_ia32_pause();
        if ((spin & 4095) == 0) {
            if (SteadyClock::now() - t0 > std::chrono::seconds(30)) {
                rc = HSC_EDEVICE, *why = "small batch did not finish within 30 s";
                running = true;
                break;
            }
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) {
                if ((uint32_t)(*done >> 32) != seq)
                    rc = HSC_EDEVICE, *why = "small batch finished without its done word";
                break;
            }
            if (e != hipErrorNotReady) {
                rc = HSC_EDEVICE, *why = "small batch", *herr = e;
                break;
            }
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (rc == HSC_OK) {
        const uint32_t low = (uint32_t)*done;
        if (low & kSmallPacked) {  // one block: the verdict bits came with the done word
            for (size_t t = 0; t < sl.n_txn; ++t) rc_out[t] = (sl.forced[t] || ((low >> t) & 1)) ? 1 : 0;
        } else {
            const uint8_t *v = io + sl.vo;
            for (size_t t = 0; t < sl.n_txn; ++t) rc_out[t] = (sl.forced[t] | v[t]) ? 1 : 0;
        }
    }
    // a slot whose kernel may still write it stays taken
    if (!running) sl.busy.store(false, std::memory_order_release);
    c->sm_wait_ns.fetch_add(ns_since(t0), std::memory_order_relaxed);
    return rc;
}

// Full checks of every read set of src: marshal (host threads) -> upload ->
// join -> download.  A large batch runs as a pipeline of chunks over the two
// staging sets: chunk i + 1 is marshalled on the host while chunk i is
// uploaded, probed and read back.
// lk (the caller's hold on c->mu, may be null): a small batch releases it
// while its kernel runs and returns without it.
template <class Src>
static int check_src(hsc_ctx *c, const Src &src, int *rc_out,
                     std::unique_lock<std::mutex> *lk = nullptr)
{
    if (c->multi) {  // the members' routed pipeline (hsc_multi.cpp)
        const int rc = marshal_into(c, src, 0, src.ntxn(), c->stage[0]);
        return rc ? rc : multi_check_stage(c, c->stage[0], rc_out, lk);
    }
    if (c->host_only) return fail(c, HSC_EDEVICE, "host-only context");
    const int T = src.ntxn();
    const int nchunks = T >= 2 * kPipeTxns ? (T + kPipeTxns - 1) / kPipeTxns : 1;
    const int per = std::max(1, (T + nchunks - 1) / nchunks);
    if (nchunks == 1 && small_path(c, T)) {
        Stage &st = c->small_st;
        st.coh = true;
        const auto t0 = SteadyClock::now();
        int rc = marshal_into(c, src, 0, T, st);
        if (rc == HSC_OK && st.n <= kSmallMaxRanges && st.n_lock <= kSmallMaxRanges) {
            const auto t1 = SteadyClock::now();
            const int k = small_launch(c, st);
            if (k < 0) return k;
            c->sm_calls.fetch_add(1, std::memory_order_relaxed);
            c->sm_marshal_ns.fetch_add(
                (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                std::memory_order_relaxed);
            hipStream_t s = c->small[k].stream;
            if (lk) lk->unlock();
            if (const hipError_t e = small_fire(c, k); e != hipSuccess) {
                c->small[k].busy.store(false, std::memory_order_release);
                if (lk) lk->lock();
                return fail(c, HSC_EDEVICE, "small batch launch", e);
            }
            c->sm_launch_ns.fetch_add(ns_since(t1), std::memory_order_relaxed);  // slot + launch
            const char *why = nullptr;
            hipError_t herr = hipSuccess;
            rc = small_wait(c, k, s, rc_out, &why, &herr);
            if (rc != HSC_OK) {
                if (lk) lk->lock();
                return fail(c, rc, why, herr);
            }
            return HSC_OK;
        }
        if (rc == HSC_OK) rc = launch_stage(c, st);
        if (rc == HSC_OK) rc = finish_stage(c, st, rc_out);
        if (rc != HSC_OK) (void)hipStreamSynchronize(c->stream);
        return rc;
    }
    int pending[2] = {-1, -1};
    int rc = HSC_OK;
    auto timed = [&](std::atomic<uint64_t> &acc, auto f) {
        const auto a = SteadyClock::now();
        const int r = f();
        acc.fetch_add(ns_since(a), std::memory_order_relaxed);
        return r;
    };
    for (int i = 0; i < nchunks && rc == HSC_OK; ++i) {
        Stage &st = c->stage[i & 1];
        if (pending[i & 1] >= 0)
            rc = timed(c->mb_wait_ns, [&] { return finish_stage(c, st, rc_out + pending[i & 1]); });
        pending[i & 1] = -1;
        const int t0 = i * per, t1 = std::min(T, t0 + per);
        if (rc == HSC_OK) rc = marshal_into(c, src, t0, t1, st);
        if (rc == HSC_OK) rc = timed(c->mb_launch_ns, [&] { return launch_stage(c, st); });
        if (rc == HSC_OK) pending[i & 1] = t0;
    }
    for (int i = nchunks; i < nchunks + 2 && rc == HSC_OK; ++i)
        if (pending[i & 1] >= 0)
            rc = timed(c->mb_wait_ns, [&] { return finish_stage(c, c->stage[i & 1], rc_out + pending[i & 1]); });
    if (rc != HSC_OK) {
        (void)hipStreamSynchronize(c->stream);  // nothing in flight on the staging sets
        return rc;
    }
    collect_timing(c);
    return HSC_OK;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int hsc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// The drop-in entry's first calls without allocations: the slots' counters
// and fine-grained staging for two small batches (the marshal's stage and
// slot 0 trade arenas at every launch) on both the direct and the
// collector's premarshalled path.  Failures here only leave it to the first
// call, as before.  (Not slot 0's stream: a stream made here took a hardware
// queue from the caller's streams -- GPU_MAX_HW_QUEUES is 4 -- and config 3's
// three bench streams then shared one, 72.6 -> 99 us per batch, r05ac.)
static void warm_small(hsc_ctx *c)
{
    constexpr size_t kWarmBytes = 64 * 1024;
    if (c->small_blocks.ensure(64 * hsc_ctx::kSmallSlots) == hipSuccess &&
        hipMemsetAsync(c->small_blocks.p, 0, 64 * hsc_ctx::kSmallSlots, c->own_stream) == hipSuccess &&
        hipStreamSynchronize(c->own_stream) == hipSuccess)
        c->small_blocks_zeroed = true;
    (void)c->small[0].io.ensure(kWarmBytes, true, true);
    (void)c->small_st.arena.ensure(kWarmBytes, true, true);
    (void)c->small_st.forced.ensure(1024, true);
    Stage *ps = new (std::nothrow) Stage();
    if (!ps) return;
    (void)ps->arena.ensure(kWarmBytes, true, true);
    (void)ps->forced.ensure(1024, true);
    c->pre_stages.emplace_back(ps);
    c->pre_free.push_back(ps);
}

int hsc_ctx_create(int device, hsc_ctx **out)
{
    if (!out) return HSC_EINVAL;
    *out = nullptr;
    if (device == -1) {
        hsc_ctx *c = new (std::nothrow) hsc_ctx();
        if (!c) return HSC_ENOMEM;
        c->device = -1;
        c->host_only = true;
        c->threads = default_threads();
        *out = c;
        return HSC_OK;
    }
    int n = hsc_device_count();
    if (device < 0 || device >= n) return HSC_EDEVICE;
    if (hipSetDevice(device) != hipSuccess) return HSC_EDEVICE;
    hsc_ctx *c = new (std::nothrow) hsc_ctx();
    if (!c) return HSC_ENOMEM;
    c->device = device;
    c->threads = default_threads();
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return HSC_EDEVICE;
    }
    c->stream = c->own_stream;
    warm_small(c);
    // every file's code object now, not lazily inside the first build / probe
    static std::mutex warm_mu;
    static std::vector<bool> warmed;
    {
        std::lock_guard<std::mutex> g(warm_mu);
        if (warmed.size() < (size_t)n) warmed.resize(n, false);
        if (!warmed[device]) {
            for (auto f : {warm_kernels, warm_ingest, warm_narrow, warm_ctiles, warm_delta,
                           warm_compact, warm_csort, warm_coalesce, warm_edges, warm_graph, warm_route})
                (void)f();
            warmed[device] = true;
        }
    }
    *out = c;
    return HSC_OK;
}

void hsc_ctx_destroy(hsc_ctx *c)
{
    if (!c) return;
    if (hsc_collector *k = c->auto_col.exchange(nullptr)) hsc_collector_destroy(k);
    if (c->multi) multi_destroy(c);  // the members first; the front is host-only
    if (c->host_only) {
        for (Stage &st : c->stage) st.release();
    c->small_st.release();
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    (void)wait_small(c);
    for (hipStream_t &st : c->small_side)
        if (st) (void)hipStreamSynchronize(st), (void)hipStreamDestroy(st), st = nullptr;
    fold_discard(c);
    fold_stop(c);
    if (c->shadow) hsc_ctx_destroy(c->shadow);
    c->shadow = nullptr;
    (void)hipStreamSynchronize(c->stream);
    for (auto &L : c->lanes)
        if (L.done) (void)hipEventSynchronize(L.done);
    for (DBuf *b : {&c->f_dgid, &c->f_dwords, &c->f_dlsn, &c->f_dbmax, &c->d_pk[0], &c->d_pk[1]}) b->release();
    if (c->fold_ev) (void)hipEventDestroy(c->fold_ev);
    DBuf *bufs[] = {&c->d_gid, &c->d_words, &c->d_lsn, &c->d_gid2, &c->d_words2, &c->d_lsn2,
                    &c->d_flags, &c->d_scratch, &c->d_gstart, &c->d_gend, &c->d_tmax,
                    &c->d_table_max, &c->d_group_table, &c->d_count, &c->d_sp_g, &c->d_sp_w,
                    &c->w_item_tile, &c->w_hist, &c->p_lo, &c->p_hi,
                    &c->p_gid, &c->p_snap, &c->p_txn, &c->p_lock_table, &c->p_lock_snap,
                    &c->p_lock_txn, &c->p_arena, &c->p_verdict, &c->p_bitmap, &c->w_code, &c->w_counts,
                    &c->w_bucket, &c->w_cursor, &c->w_items, &c->w_item_desc, &c->w_recs,
                    &c->d_nkeys, &c->d_nmaxs, &c->d_nbase, &c->d_nzero, &c->d_ntmax,
                    &c->d_nsp_g, &c->d_nsp_w, &c->d_ngs, &c->d_nscratch, &c->p_code_lo,
                    &c->p_code_hi, &c->p_zero, &c->d_commits, &c->d_cdir, &c->d_tdir, &c->d_trad, &c->d_done, &c->w_vflags, &c->d_key32, &c->d_rank32,
                    &c->d_ctmp[0], &c->d_ctmp[1], &c->d_ctmp[2], &c->d_ctmp[3], &c->w_tcode,
                    &c->w_tcode2, &c->w_trecs};
    for (DBuf *b : bufs) b->release();
    for (Stage &st : c->stage) st.release();
    c->small_st.release();
    for (auto &ps : c->pre_stages) ps->release();
    for (auto &sl : c->small) sl.io.release();
    c->small_blocks.release();
    for (DBuf *b : {&c->d_csrep, &c->d_csmask, &c->d_cspat, &c->d_csmv, &c->d_csbits, &c->d_cskeys[0],
                    &c->d_cskeys[1], &c->d_cssplit, &c->d_cmask, &c->d_cpat, &c->d_cmv, &c->d_cbits,
                    &c->d_cwords})
        b->release();
    for (DBuf *b : {&c->d_dgid[0], &c->d_dgid[1], &c->d_dwords[0], &c->d_dwords[1], &c->d_dlsn[0],
                    &c->d_dlsn[1], &c->d_dbmax, &c->d_agid})
        b->release();
    for (HBuf &b : c->h_appq) b.release();
    for (hipEvent_t &e : c->app_ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    for (HBuf &b : c->h_pend) b.release();
    for (hipEvent_t &e : c->pend_ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    for (DBuf &b : c->co_dev) b.release();
    for (DBuf *b : {&c->e_span, &c->e_cnt, &c->e_txn, &c->e_lsn, &c->e_txn2, &c->e_lsn2, &c->e_gid,
                    &c->e_scratch, &c->e_flags, &c->e_after})
        b->release();
    for (auto &L : c->lanes) {
        for (DBuf &b : L.b) b.release();
        if (L.done) (void)hipEventDestroy(L.done);
    }
    c->graph.release_all();
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int hsc_set_stream(hsc_ctx *c, void *st)
{
    if (!c) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    hipStream_t ns = st ? (hipStream_t)st : c->own_stream;
    // small batches launched on the old stream may still read the delta run
    // a later append on the new stream rewrites: let them finish first
    if (ns != c->stream && wait_small(c) != hipSuccess)
        return fail(c, HSC_EDEVICE, "set_stream: a small batch did not finish");
    // appends return before their upload and merge ran: the new stream waits
    if (c->app_last && ns != c->stream && hipStreamWaitEvent(ns, c->app_last, 0) != hipSuccess)
        return fail(c, HSC_EDEVICE, "set_stream: order after the appends");
    if (ctx_switch_stream(c, ns) != hipSuccess) return fail(c, HSC_EDEVICE, "set_stream: lane fence");
    return HSC_OK;
}

const char *hsc_last_error(hsc_ctx *c) { return c ? c->err.c_str() : "null context"; }

int hsc_window_reset(hsc_ctx *c)
{
    if (!c) return HSC_EINVAL;
    MuGuard g(c);
    clear_window(c);
    c->phys.clear();
    c->end_lsn = 0;
    return HSC_OK;
}

static int ingest_log_locked(hsc_ctx *c, const hsc_llog *log)
{
    if (!c->host_only) (void)hipSetDevice(c->device);
    int rc = ingest_log(c, log);
    if (rc) return rc;
    return ensure_built(c);
}

int hsc_window_ingest_log(hsc_ctx *c, const hsc_llog *log)
{
    if (!c || !log) return HSC_EINVAL;
    MuGuard g(c);
    c->phys.clear();  // a decoded log brings no physical records for later walks
    return ingest_log_locked(c, log);
}

int hsc_window_append(hsc_ctx *c, const hsc_write *w, size_t n)
{
    if (!c || (!w && n)) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    if (c->multi && multi_adopted(c))  // the members hold the window: append to them
        return fail(c, HSC_ESTATE, "append to an adopted multi context: append to its members");
    for (size_t i = 0; i < n; ++i) {
        if (!w[i].tbname) return fail(c, HSC_EINVAL, "write without table");
        if (w[i].commit_lsn < c->last_append_lsn) return fail(c, HSC_EINVAL, "commit LSNs must not decrease");
        if (w[i].key && (w[i].keylen < 0 || w[i].keylen > kMaxWords * 8))
            return fail(c, HSC_EINVAL, "key longer than MAXKEYLEN");
    }
    // decoded writes carry no record LSNs: the window no longer knows every
    // record, so the DB_SET-on-a-non-record rule is off from here on
    c->lg_rule = false;
    for (size_t i = 0; i < n; ++i) {
        c->last_append_lsn = w[i].commit_lsn;
        // the log ends past every commit it holds: a snapshot in [old end,
        // commit] must still see this write even if the caller skips
        // hsc_window_set_end (which can only raise the end further)
        if (w[i].commit_lsn >= c->end_lsn) c->end_lsn = w[i].commit_lsn + 1;
        int tid = table_id_or_add(c, w[i].tbname);
        add_write(c, tid, w[i].idxnum, (const uint8_t *)w[i].key, w[i].keylen, w[i].key != nullptr,
                  w[i].commit_lsn);
    }
    if (!c->live) {
        c->dirty = true;
        return HSC_OK;
    }
    return flush_appends(c, true);
}

int hsc_window_append_log(hsc_ctx *c, const hsc_llog *log)
{
    if (!c || !log) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    if (c->multi && multi_adopted(c))
        return fail(c, HSC_ESTATE, "append to an adopted multi context: append to its members");
    const double t0 = fold_trace() ? trace_us() : 0;
    int rc = append_log(c, log);
    if (rc) return rc;
    const double t1 = fold_trace() ? trace_us() : 0;
    const size_t pend0 = c->pend_merges;
    rc = c->live ? flush_appends(c, true) : HSC_OK;
    if (fold_trace() && trace_us() - t0 > 150)  // (diagnostics: where a slow append went)
        fprintf(stderr, "[append] %.0f slow: decode %.0f us, flush %.0f us (merged %d)\n", t0, t1 - t0,
                trace_us() - t1, (int)(c->pend_merges - pend0));
    return rc;
}

int hsc_window_append_raw(hsc_ctx *c, const hsc_raw_log *raw)
{
    const hsc_llog *lg = nullptr;
    int rc = hsc_decode_log(c, raw, &lg);
    if (rc) return rc;
    return hsc_window_append_log(c, lg);
}

size_t hsc_window_delta_rows(hsc_ctx *c) { return c ? c->dn + c->fn + c->pend_n : 0; }

int hsc_set_fold(hsc_ctx *c, size_t rows, int background)
{
    if (!c || rows > kDeltaCap) return HSC_EINVAL;
    MuGuard g(c);
    c->fold_rows = rows ? rows : kDeltaCap / 2;
    c->fold_bg = background != 0;
    return c->dirty ? HSC_OK : append_prepare(c);  // (a built window: the worker starts now)
}

int hsc_fold_stats(hsc_ctx *c, uint64_t out[4])
{
    if (!c || !out) return HSC_EINVAL;
    MuGuard g(c);
    out[0] = c->folds_started;
    out[1] = c->folds_swapped;
    out[2] = c->folds_inline;
    out[3] = (uint64_t)(c->fold_ms * 1000.0f);
    return HSC_OK;
}

int hsc_set_paths(hsc_ctx *c, unsigned flags)
{
    if (!c || (flags & ~(unsigned)HSC_PATH_ALL)) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only && (flags & HSC_PATH_NO_SMALL) && !c->no_small && wait_small(c) != hipSuccess)
        return fail(c, HSC_EDEVICE, "set_paths: a small batch did not finish");
    if (((flags ^ c->paths) & (HSC_PATH_NO_PACKED_SORT | HSC_PATH_TILE_DIR)) && c->live) {
        c->dirty = true;  // the next check rebuilds the window the new way
        if (!c->host_staged) c->merge_pending = true;
    }
    c->paths = flags;
    c->no_small = (flags & HSC_PATH_NO_SMALL) != 0;
    if (c->no_small && (c->pend_n || c->pend_t)) return flush_appends(c);  // the tail is the small kernel's
    return HSC_OK;
}

int hsc_append_stats(hsc_ctx *c, uint64_t out[3])
{
    if (!c || !out) return HSC_EINVAL;
    MuGuard g(c);
    out[0] = c->pend_appends;
    out[1] = c->pend_merges;
    out[2] = c->pend_n;
    return HSC_OK;
}

int hsc_window_set_end(hsc_ctx *c, uint64_t end_lsn)
{
    if (!c) return HSC_EINVAL;
    MuGuard g(c);
    c->end_lsn = end_lsn;
    return HSC_OK;
}

static bool raw_args_ok(const hsc_raw_log *raw)
{
    return !((raw->nrec && (!raw->lsn || !raw->off || !raw->len || !raw->buf)) ||
             (raw->nrecon && (!raw->recon_lsn || !raw->recon_off || !raw->recon_len || !raw->recon_keys)));
}

static int decode_locked(hsc_ctx *c, const hsc_raw_log *raw, bool reset)
{
    std::string err;
    int rc = decode_raw_log(raw, c->decoded, c->phys, reset, err);
    return rc ? fail(c, rc, err.c_str()) : HSC_OK;
}

int hsc_decode_log(hsc_ctx *c, const hsc_raw_log *raw, const hsc_llog **out)
{
    if (!c || !raw || !out || !raw_args_ok(raw)) return HSC_EINVAL;
    MuGuard g(c);
    int rc = decode_locked(c, raw, false);
    if (rc) return rc;
    *out = &c->decoded.llog;
    return HSC_OK;
}

int hsc_window_ingest_raw(hsc_ctx *c, const hsc_raw_log *raw)
{
    if (!c || !raw || !raw_args_ok(raw)) return HSC_EINVAL;
    MuGuard g(c);
    int rc = decode_locked(c, raw, true);  // a new log: walks see only its records
    if (rc) return rc;
    return ingest_log_locked(c, &c->decoded.llog);
}

int hsc_decode_serial(hsc_ctx *c, const hsc_serial_msgs *m, const hsc_readsets **out)
{
    if (!c || !m || !out || (m->nmsg && (!m->buf || !m->off || !m->len)) || m->nmsg > 0x7FFFFFFF)
        return HSC_EINVAL;
    MuGuard g(c);
    std::string err;
    int rc = decode_serial_msgs(m, c->wire, err);
    if (rc) return fail(c, rc, err.c_str());
    *out = &c->wire.rs;
    return HSC_OK;
}

int hsc_check_serial(hsc_ctx *c, const hsc_serial_msgs *m, int *rc_out)
{
    if (!c || !m || (m->nmsg && !rc_out)) return HSC_EINVAL;
    const hsc_readsets *rs = nullptr;
    int rc = hsc_decode_serial(c, m, &rs);
    if (rc) {  // fail closed
        for (size_t i = 0; i < m->nmsg; ++i) rc_out[i] = 1;
        return rc;
    }
    return hsc_check_readsets(c, rs, rc_out);
}

int hsc_window_build(hsc_ctx *c)
{
    if (!c) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    return ensure_built(c);
}

int hsc_register_group(hsc_ctx *c, const char *tbname, int idxnum, int keylen)
{
    if (!c || !tbname || keylen < 0 || keylen > kMaxWords * 8) return HSC_EINVAL;
    MuGuard lk(c);
    int tid = table_id_or_add(c, tbname);
    const int g = group_id_or_add(c, tid, idxnum, keylen);
    if (c->multi) multi_sync_dict(c);  // members keep the same table ids and gids
    return g;
}

int hsc_window_ingest_device(hsc_ctx *c, size_t n, int words, const uint32_t *gid,
                             const uint64_t *key_words, const uint64_t *lsn, uint64_t end_lsn)
{
    if (c && c->host_only) return HSC_EDEVICE;
    if (!c || words < 1 || words > kMaxWords || (n && (!gid || !key_words || !lsn)))
        return HSC_EINVAL;
    if (n >= 0xFFFFFFFFull) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    clear_window(c);
    c->phys.clear();
    c->host_staged = false;
    c->end_lsn = end_lsn;
    if (words < window_words(c)) return fail(c, HSC_EINVAL, "fewer key words than a registered group needs");
    set_words(c, words);
    c->cap = window_cap(n);
    HIPCHK(c, c->d_gid.ensure(c->cap * 4));
    HIPCHK(c, c->d_words.ensure(c->cap * 8 * (size_t)words));
    HIPCHK(c, c->d_lsn.ensure(c->cap * 8));
    hipStream_t s = c->stream;
    if (n) {
        HIPCHK(c, hipMemcpyAsync(c->d_gid.p, gid, 4 * n, hipMemcpyDeviceToDevice, s));
        for (int j = 0; j < words; ++j)
            HIPCHK(c, hipMemcpyAsync(c->d_words.as<uint64_t>() + (size_t)j * c->cap, key_words + (size_t)j * n,
                                     8 * n, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->d_lsn.p, lsn, 8 * n, hipMemcpyDeviceToDevice, s));
    }
    int rc = device_build(c, n);
    if (rc) return rc;
    for (uint64_t v : c->h_table_max) c->max_commit = std::max(c->max_commit, v);
    return HSC_OK;
}

int hsc_set_layout(hsc_ctx *c, int layout)
{
    if (!c || layout < HSC_LAYOUT_AUTO || layout > HSC_LAYOUT_COMPACT_WIDE ||
        layout == HSC_LAYOUT_NARROW || layout == HSC_LAYOUT_COMPACT)
        return HSC_EINVAL;
    MuGuard g(c);
    const bool rebuild = (c->layout == HSC_LAYOUT_WIDE) != (layout == HSC_LAYOUT_WIDE);
    c->layout = layout;
    if (rebuild) {
        if (!c->host_staged) return fail(c, HSC_ESTATE, "device window must be re-ingested");
        c->dirty = true;
    }
    return HSC_OK;
}

int hsc_window_layout(hsc_ctx *c)
{
    if (!c) return HSC_LAYOUT_WIDE;
    return c->narrow ? HSC_LAYOUT_NARROW : c->compact ? HSC_LAYOUT_COMPACT : HSC_LAYOUT_WIDE;
}

int hsc_window_code_words(hsc_ctx *c) { return c && c->compact ? c->ct.WC : c ? c->W : 0; }
int hsc_window_tile_key_words(hsc_ctx *c) { return c && c->compact && c->ctiles ? c->ctv.WG : 0; }

int hsc_window_words(hsc_ctx *c) { return c ? c->W : 0; }
int hsc_window_sort_path(hsc_ctx *c) { return !c ? 0 : c->packed_sort ? 1 : c->code_sorted ? 2 : 0; }
size_t hsc_window_keys(hsc_ctx *c) { return c ? c->n : 0; }
// (the published values: callers read them without the context lock)
uint64_t hsc_window_end(hsc_ctx *c) { return c ? c->rg_end.load(std::memory_order_acquire) : 0; }
uint64_t hsc_window_max_commit(hsc_ctx *c) { return c ? c->rg_max.load(std::memory_order_acquire) : 0; }

int hsc_table_id(hsc_ctx *c, const char *tbname)
{
    if (!c || !tbname) return -1;
    auto it = c->table_ids.find(tbname);
    return it == c->table_ids.end() ? -1 : it->second;
}

const char *hsc_table_name(hsc_ctx *c, int tid)
{
    if (!c || tid < 0 || tid >= (int)c->table_names.size()) return nullptr;
    return c->table_names[tid].c_str();
}

int hsc_group_info(hsc_ctx *c, int gid, int *table_id, int *idxnum, int *keylen)
{
    if (!c || gid < 0 || gid >= (int)c->groups.size()) return HSC_EINVAL;
    if (table_id) *table_id = c->groups[gid].tid;
    if (idxnum) *idxnum = c->groups[gid].ix;
    if (keylen) *keylen = c->groups[gid].klen;
    return HSC_OK;
}

int hsc_table_max(hsc_ctx *c, uint64_t *out, int n)
{
    if (!c || n < 0 || (n && !out)) return HSC_EINVAL;
    const int nt = (int)c->table_names.size();
    for (int t = 0; t < std::min(n, nt); ++t) out[t] = c->h_table_max[t];
    return nt;
}

int hsc_merge_table_max(hsc_ctx *c, const uint64_t *in, int n)
{
    if (!c || n < 0 || (n && !in) || n > (int)c->table_names.size()) return HSC_EINVAL;
    MuGuard g(c);
    for (int t = 0; t < n; ++t) {
        c->h_table_max[t] = std::max(c->h_table_max[t], in[t]);
        c->max_commit = std::max(c->max_commit, in[t]);
    }
    if (c->multi)
        for (int m = 0; m < hsc_multi_local(c); ++m) {
            hsc_ctx *mc = hsc_multi_member(c, m);
            const int rc = hsc_merge_table_max(mc, in, std::min(n, (int)mc->table_names.size()));
            if (rc) return fail(c, rc, "merge_table_max: member");
        }
    if (!c->host_only && !c->dirty && n > 0) {
        (void)hipSetDevice(c->device);
        const size_t nt = c->table_names.size();
        HIPCHK(c, wait_small(c));  // no reader of the old buffer in flight
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, c->d_table_max.ensure(8 * nt));
        HIPCHK(c, hipMemcpyAsync(c->d_table_max.p, c->h_table_max.data(), 8 * nt,
                                 hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->nt_dev = (uint32_t)nt;
    }
    return HSC_OK;
}

int hsc_marshal_readsets(hsc_ctx *c, const hsc_readsets *rs, const hsc_marshalled **out)
{
    if (!c || !rs || !out) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    int rc = ensure_built(c);
    if (rc) return rc;
    rc = marshal_readsets(c, rs);
    *out = &c->m;
    return rc;
}

int hsc_marshal_arrs(hsc_ctx *c, void *const *ranges, const uint64_t *snaps, int n,
                     const hsc_marshalled **out)
{
    if (!c || n < 0 || (n && (!ranges || !snaps)) || !out) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    int rc = ensure_built(c);
    if (rc) return rc;
    for (int i = 0; i < n; ++i)
        if (!ranges[i]) return fail(c, HSC_EINVAL, "marshal: NULL CurRangeArr");
    ArrSrc src{(hsc_currangearr *const *)ranges, snaps, n};
    rc = marshal_into(c, src, 0, n, c->stage[0]);
    *out = &c->m;
    return rc;
}

long hsc_window_export(hsc_ctx *c, int all_versions, uint32_t *gid, uint64_t *key_words,
                       uint64_t *lsn, size_t cap)
{
    if (!c) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    const bool copy = gid || key_words || lsn;
    if (copy && !(gid && key_words && lsn)) return HSC_EINVAL;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    if (c->live && (c->dn || !c->app_gid.empty())) {  // the snapshot includes the delta run
        c->merge_pending = true;
        c->dirty = true;
    }
    int rc = ensure_built(c);
    if (rc) return rc;
    const size_t n = all_versions ? c->n_all : c->n;
    if (!copy || n == 0 || n > cap) return (long)n;
    const DBuf &dg = all_versions ? c->d_gid2 : c->d_gid;
    const DBuf &dw = all_versions ? c->d_words2 : c->d_words;
    const DBuf &dl = all_versions ? c->d_lsn2 : c->d_lsn;
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(gid, dg.p, 4 * n, hipMemcpyDeviceToHost, s));
    for (int j = 0; j < c->W; ++j)
        HIPCHK(c, hipMemcpyAsync(key_words + (size_t)j * cap, dw.as<uint64_t>() + (size_t)j * c->cap, 8 * n,
                                 hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(lsn, dl.p, 8 * n, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return (long)n;
}

int hsc_rw_edges(hsc_ctx *c, const hsc_readsets *rs, size_t *n_pairs, const uint32_t **txn,
                 const uint64_t **writer_lsn)
{
    if (!c || !rs || !n_pairs || !txn || !writer_lsn) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    if (c->dn || !c->app_gid.empty()) {  // pairs need every version: fold the delta in first
        c->merge_pending = true;
        c->dirty = true;
    }
    int rc = ensure_built(c);
    if (!rc) rc = marshal_readsets(c, rs);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const hsc_marshalled &m = c->m;
    const int W = c->W;
    const size_t n = m.n;
    c->e_out_txn.clear();
    c->e_out_lsn.clear();
    c->e_dev_n = 0;
    *n_pairs = 0;
    *txn = nullptr;
    *writer_lsn = nullptr;
    if (n == 0 || c->n_all == 0) return HSC_OK;
    HIPCHK(c, c->p_lo.ensure(8 * (size_t)W * n));
    HIPCHK(c, c->p_hi.ensure(8 * (size_t)W * n));
    HIPCHK(c, c->p_gid.ensure(4 * n));
    HIPCHK(c, c->p_snap.ensure(8 * n));
    HIPCHK(c, c->p_txn.ensure(4 * n));
    HIPCHK(c, hipMemcpyAsync(c->p_lo.p, m.lo, 8 * (size_t)W * n, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->p_hi.p, m.hi, 8 * (size_t)W * n, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->p_gid.p, m.gid, 4 * n, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->p_snap.p, m.snap, 8 * n, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->p_txn.p, m.txn, 4 * n, hipMemcpyHostToDevice, s));
    ProbeView p{};
    p.n = (uint32_t)n;
    p.lo = c->p_lo.as<uint64_t>();
    p.hi = c->p_hi.as<uint64_t>();
    p.gid = c->p_gid.as<uint32_t>();
    p.snap = c->p_snap.as<uint64_t>();
    p.txn = c->p_txn.as<uint32_t>();
    EdgeView all{};
    all.gid = c->d_gid2.as<uint32_t>();
    all.words = c->d_words2.as<uint64_t>();
    all.lsn = c->d_lsn2.as<uint64_t>();
    all.stride = c->cap;
    all.n = (uint32_t)c->n_all;
    all.W = W;
    // only versions committed after the oldest snapshot of the batch can pair
    uint64_t smin = ~0ull;
    for (size_t q = 0; q < n; ++q) smin = std::min<uint64_t>(smin, m.snap[q]);
    const size_t na = c->n_all;
    HIPCHK(c, c->e_flags.ensure(4 * (na + 1) + 64));
    HIPCHK(c, c->e_scratch.ensure(scan_scratch_bytes(na + 1) + 64));
    HIPCHK(c, c->e_after.ensure((4 + 8 + 8 * (size_t)W) * std::max<size_t>(na, 1)));
    EdgeView w{};
    w.stride = std::max<size_t>(na, 1);
    w.gid = c->e_after.as<uint32_t>();
    w.lsn = (const uint64_t *)(c->e_after.as<uint8_t>() + 4 * w.stride + 4 * (w.stride & 1));
    w.words = w.lsn + w.stride;
    w.W = W;
    uint32_t nafter = 0;
    HIPCHK(c, edge_after(all, smin, c->e_flags.as<uint32_t>(), c->e_scratch.as<uint32_t>(), w,
                         &nafter, s));
    w.n = nafter;
    if (nafter == 0) return HSC_OK;
    HIPCHK(c, c->e_span.ensure(8 * n));
    HIPCHK(c, c->e_cnt.ensure(4 * (n + 1)));
    HIPCHK(c, c->e_scratch.ensure(scan_scratch_bytes(n + 1) + 64));
    HIPCHK(c, launch_edge_count(w, p, c->e_span.as<uint2>(), c->e_cnt.as<uint32_t>(), s));
    HIPCHK(c, hipMemsetAsync(c->e_cnt.as<uint32_t>() + n, 0, 4, s));
    HIPCHK(c, scan_exclusive_u32(c->e_cnt.as<uint32_t>(), n + 1, c->e_scratch.as<uint32_t>(), s));
    uint32_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, c->e_cnt.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (total == 0) return HSC_OK;
    // pairs as rows (gid = txn, one word = commit LSN) for the window's sort + dedupe
    const size_t t1 = total;
    HIPCHK(c, c->e_txn.ensure(4 * t1));
    HIPCHK(c, c->e_lsn.ensure(8 * t1));
    HIPCHK(c, c->e_txn2.ensure(4 * t1));
    HIPCHK(c, c->e_lsn2.ensure(8 * t1));
    HIPCHK(c, c->e_gid.ensure(16 * t1));  // carried LSN (two buffers)
    HIPCHK(c, c->e_flags.ensure(4 * t1 + 64));
    HIPCHK(c, c->e_scratch.ensure(std::max(radix_scratch_bytes(t1, 1), scan_scratch_bytes(t1) + 64)));
    HIPCHK(c, launch_edge_emit(w, p, c->e_span.as<uint2>(), c->e_cnt.as<uint32_t>(),
                               c->e_txn.as<uint32_t>(), c->e_lsn.as<uint64_t>(), s));
    uint64_t *carry = c->e_gid.as<uint64_t>(), *carry2 = carry + t1;
    HIPCHK(c, hipMemcpyAsync(carry, c->e_lsn.p, 8 * t1, hipMemcpyDeviceToDevice, s));
    bool in_alt = false;
    HIPCHK(c, radix_sort_rows(1, t1, c->e_txn.as<uint32_t>(), c->e_lsn.as<uint64_t>(), carry, t1,
                              c->e_txn2.as<uint32_t>(), c->e_lsn2.as<uint64_t>(), carry2,
                              c->e_scratch.p, c->e_scratch.bytes, &in_alt, nullptr, s));
    uint32_t *st = in_alt ? c->e_txn2.as<uint32_t>() : c->e_txn.as<uint32_t>();
    uint64_t *sl = in_alt ? c->e_lsn2.as<uint64_t>() : c->e_lsn.as<uint64_t>();
    uint64_t *sc = in_alt ? carry2 : carry;
    uint32_t *dt = in_alt ? c->e_txn.as<uint32_t>() : c->e_txn2.as<uint32_t>();
    uint64_t *dl = in_alt ? c->e_lsn.as<uint64_t>() : c->e_lsn2.as<uint64_t>();
    uint64_t *dc = in_alt ? carry : carry2;
    uint32_t *dcount = c->e_cnt.as<uint32_t>();  // reuse: n + 1 >= 1 entries
    HIPCHK(c, dedupe_rows(1, t1, st, sl, sc, t1, dt, dl, dc, t1, c->e_flags.as<uint32_t>(),
                          c->e_scratch.p, c->e_scratch.bytes, dcount, s));
    uint32_t nu = 0;
    HIPCHK(c, hipMemcpyAsync(&nu, dcount, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->e_out_txn.resize(nu);
    c->e_out_lsn.resize(nu);
    if (nu) {
        HIPCHK(c, hipMemcpyAsync(c->e_out_txn.data(), dt, 4 * (size_t)nu, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->e_out_lsn.data(), dl, 8 * (size_t)nu, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    *n_pairs = nu;
    *txn = c->e_out_txn.data();
    *writer_lsn = c->e_out_lsn.data();
    c->e_dev_txn = dt;
    c->e_dev_lsn = dl;
    c->e_dev_n = nu;
    return HSC_OK;
}

int hsc_coalesce_readsets(hsc_ctx *c, const hsc_readsets *rs, hsc_coalesced *out)
{
    if (!c || !rs || !out || rs->ntxn < 0) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    const int T = rs->ntxn;
    const size_t nr = T ? (size_t)rs->txn_off[T] : 0;
    // rows are indexed as uint32 on the device (ord / tmp / big-set offsets)
    if (nr > 0xFFFFFFFFull) return fail(c, HSC_EINVAL, "coalesce: more than 2^32 - 1 ranges");
    // strcmp rank of every table name (equal names share a rank)
    std::vector<int32_t> rank(std::max(rs->ntbnames, 1), 0);
    {
        std::vector<int> order(rs->ntbnames);
        for (int i = 0; i < rs->ntbnames; ++i) order[i] = i;
        std::sort(order.begin(), order.end(),
                  [&](int a, int b) { return strcmp(rs->tbnames[a], rs->tbnames[b]) < 0; });
        for (int k = 0; k < rs->ntbnames; ++k)
            rank[order[k]] = k && strcmp(rs->tbnames[order[k]], rs->tbnames[order[k - 1]]) == 0
                                 ? rank[order[k - 1]]
                                 : k;
    }
    for (size_t r = 0; r < nr; ++r)
        if (rs->table[r] < 0 || rs->table[r] >= rs->ntbnames)
            return fail(c, HSC_EINVAL, "coalesce: a range names no table");
    uint64_t nkeys = 0;
    for (size_t r = 0; r < nr; ++r) {
        if ((rs->lkeylen[r] > 0 && rs->lkey_off[r] == HSC_KEY_NULL) ||
            (rs->rkeylen[r] > 0 && rs->rkey_off[r] == HSC_KEY_NULL))
            return fail(c, HSC_EINVAL, "coalesce: a NULL key with a nonzero length");
        if (rs->lkeylen[r] > 0) nkeys = std::max<uint64_t>(nkeys, rs->lkey_off[r] + rs->lkeylen[r]);
        if (rs->rkeylen[r] > 0) nkeys = std::max<uint64_t>(nkeys, rs->rkey_off[r] + rs->rkeylen[r]);
    }
    hipStream_t s = c->stream;
    DBuf *d = c->co_dev;
    const size_t n1 = std::max<size_t>(nr, 1);
    const size_t sz[18] = {8 * ((size_t)T + 1), 4 * n1, 4 * n1, 4 * n1, 4 * n1, 4 * n1, 4 * n1,
                           4 * n1, 8 * n1, 8 * n1, std::max<uint64_t>(nkeys, 1), 4 * rank.size(),
                           4 * n1, 4 * n1, 4 * n1, 8 * n1, 8 * n1 /* ord + tmp */,
                           4 * (size_t)std::max(T, 1)};
    for (int k = 0; k < 18; ++k) HIPCHK(c, d[k].ensure(sz[k]));
    const void *src[12] = {rs->txn_off, rs->table, rs->idxnum, rs->lflag, rs->rflag, rs->islocked,
                           rs->lkeylen, rs->rkeylen, rs->lkey_off, rs->rkey_off, rs->keys,
                           rank.data()};
    const size_t bytes[12] = {8 * ((size_t)T + 1), 4 * nr, 4 * nr, 4 * nr, 4 * nr, 4 * nr, 4 * nr,
                              4 * nr, 8 * nr, 8 * nr, nkeys, 4 * rank.size()};
    for (int k = 0; k < 12; ++k)
        if (bytes[k]) HIPCHK(c, hipMemcpyAsync(d[k].p, src[k], bytes[k], hipMemcpyHostToDevice, s));
    CoView v{};
    v.ntxn = T;
    v.off = d[0].as<int64_t>();
    v.table = d[1].as<int32_t>(), v.idxnum = d[2].as<int32_t>(), v.lflag = d[3].as<int32_t>();
    v.rflag = d[4].as<int32_t>(), v.islocked = d[5].as<int32_t>(), v.lkeylen = d[6].as<int32_t>();
    v.rkeylen = d[7].as<int32_t>();
    v.lkey_off = d[8].as<uint64_t>(), v.rkey_off = d[9].as<uint64_t>();
    v.keys = d[10].as<uint8_t>(), v.nkeys = nkeys, v.tbrank = d[11].as<int32_t>();
    v.w_rflag = d[12].as<int32_t>(), v.w_islocked = d[13].as<int32_t>();
    v.w_rkeylen = d[14].as<int32_t>(), v.w_rkey_off = d[15].as<uint64_t>();
    v.ord = d[16].as<uint32_t>(), v.tmp = d[16].as<uint32_t>() + n1;
    v.count = d[17].as<uint32_t>();
    // large sets take the level-parallel sort (see hsc_coalesce.hip); one with a
    // tie-with-everything range (NULL lower key) replays glibc's merge tree
    std::vector<uint32_t> isbig((size_t)std::max(T, 1), 0), bset, bpre(1, 0);
    uint32_t bmax = 0;
    bool ties = false;
    if (!(c->paths & HSC_PATH_CO_SERIAL)) {  // else every set on the per-thread path
        for (int t = 0; t < T; ++t) {
            const size_t b = (size_t)rs->txn_off[t], e = (size_t)rs->txn_off[t + 1];
            if (e - b < kCoBig || bpre.back() + (e - b) > 0xFFFFFFFFull) continue;
            bool ok = true, tie = false;
            for (size_t r = b; r < e && ok; ++r) {  // locked ranges open at both ends
                ok = !rs->islocked[r] || (rs->lflag[r] && rs->rflag[r]);
                tie |= !rs->islocked[r] && !rs->lflag[r] && rs->lkey_off[r] == HSC_KEY_NULL;
            }
            if (!ok) continue;
            ties |= tie;
            isbig[t] = 1;
            bset.push_back((uint32_t)t);
            bpre.push_back(bpre.back() + (uint32_t)(e - b));
            bmax = std::max(bmax, (uint32_t)(e - b));
        }
    }
    const uint32_t nbig = (uint32_t)bset.size();
    if (nbig) {
        HIPCHK(c, d[18].ensure(4 * isbig.size()));
        HIPCHK(c, d[19].ensure(4 * (size_t)nbig));
        HIPCHK(c, d[20].ensure(4 * ((size_t)nbig + 1)));
        HIPCHK(c, d[21].ensure(4 * n1));
        HIPCHK(c, d[22].ensure(8 * n1));
        HIPCHK(c, hipMemcpyAsync(d[18].p, isbig.data(), 4 * isbig.size(), hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(d[19].p, bset.data(), 4 * (size_t)nbig, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(d[20].p, bpre.data(), 4 * ((size_t)nbig + 1), hipMemcpyHostToDevice, s));
    }
    if (ties) HIPCHK(c, d[23].ensure(coalesce_tie_scratch_bytes(bpre.back())));
    // HSC_PATH_CO_RUN_THREAD: one thread per run in the merge scan (A/B, tests)
    const bool run_chunks = !(c->paths & HSC_PATH_CO_RUN_THREAD);
    if (nbig && run_chunks) HIPCHK(c, d[24].ensure(coalesce_run_scratch_bytes(bpre.back())));
    HIPCHK(c, launch_coalesce(v, d[18].as<uint32_t>(), d[19].as<uint32_t>(), d[20].as<uint32_t>(),
                              nbig, bpre.back(), bmax, d[21].as<uint32_t>(), d[22].as<uint32_t>(),
                              ties ? d[23].p : nullptr, nbig && run_chunks ? d[24].p : nullptr, s));
    std::vector<uint32_t> cnt(T), ord(nr);
    std::vector<int32_t> wrf(nr), wlk(nr), wrl(nr);
    std::vector<uint64_t> wro(nr);
    if (T) HIPCHK(c, hipMemcpyAsync(cnt.data(), v.count, 4 * (size_t)T, hipMemcpyDeviceToHost, s));
    if (nr) {
        HIPCHK(c, hipMemcpyAsync(ord.data(), v.ord, 4 * nr, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(wrf.data(), v.w_rflag, 4 * nr, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(wlk.data(), v.w_islocked, 4 * nr, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(wrl.data(), v.w_rkeylen, 4 * nr, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(wro.data(), v.w_rkey_off, 8 * nr, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));
    // compact the surviving rows of every set, in coalesced order
    c->co_off.assign((size_t)T + 1, 0);
    for (auto &a : c->co_i32) a.clear();
    for (auto &a : c->co_u64) a.clear();
    for (int t = 0; t < T; ++t) {
        const size_t b = (size_t)rs->txn_off[t];
        for (uint32_t k = 0; k < cnt[t]; ++k) {
            const uint32_t r = ord[b + k];
            c->co_i32[0].push_back(rs->table[r]);
            c->co_i32[1].push_back(rs->idxnum[r]);
            c->co_i32[2].push_back(rs->lflag[r]);
            c->co_i32[3].push_back(wrf[r]);
            c->co_i32[4].push_back(wlk[r]);
            c->co_i32[5].push_back(rs->lkeylen[r]);
            c->co_i32[6].push_back(wrl[r]);
            c->co_u64[0].push_back(rs->lkey_off[r]);
            c->co_u64[1].push_back(wro[r]);
        }
        c->co_off[t + 1] = c->co_off[t] + cnt[t];
    }
    out->ntxn = T;
    out->txn_off = c->co_off.data();
    out->table = c->co_i32[0].data(), out->idxnum = c->co_i32[1].data();
    out->lflag = c->co_i32[2].data(), out->rflag = c->co_i32[3].data();
    out->islocked = c->co_i32[4].data(), out->lkeylen = c->co_i32[5].data();
    out->rkeylen = c->co_i32[6].data();
    out->lkey_off = c->co_u64[0].data(), out->rkey_off = c->co_u64[1].data();
    return HSC_OK;
}

int hsc_check_readsets(hsc_ctx *c, const hsc_readsets *rs, int *rc_out)
{
    if (!c || !rs || (!rc_out && rs->ntxn)) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    int rc = ensure_built(c);
    if (!rc) {
        std::vector<int> tmap;
        rc = check_src(c, flat_src(c, rs, tmap), rc_out);
    }
    if (rc)
        for (int t = 0; t < rs->ntxn; ++t) rc_out[t] = 1;  // fail closed
    return rc;
}

// Publish the dictionaries as a snapshot for premarshal (under c->mu; only
// when the epoch moved).
static void publish_dict(hsc_ctx *c)
{
    const MarshalDict *cur = c->dict_cur.load(std::memory_order_acquire);
    if (cur && cur->epoch == c->dict_epoch) return;
    auto d = std::make_unique<MarshalDict>();
    d->epoch = c->dict_epoch;
    d->W = c->W;
    d->table_ids = c->table_ids;
    d->groups = c->groups;
    d->ix_groups = c->ix_groups;
    c->dict_cur.store(d.get(), std::memory_order_release);
    c->dict_all.push_back(std::move(d));
}

static int check_batch(hsc_ctx *c, void *const *ranges, PreMarshal *const *pre, unsigned int *file,
                       unsigned int *offset, int regop_only, int n, int *rc_out);

int hip_serial_check_batch(void *vctx, void *const *ranges, unsigned int *file,
                           unsigned int *offset, int regop_only, int n, int *rc_out)
{
    return check_batch((hsc_ctx *)vctx, ranges, nullptr, file, offset, regop_only, n, rc_out);
}

}  // extern "C"

namespace hsc {
PreMarshal *premarshal_new() { return new (std::nothrow) PreMarshal; }
void premarshal_free(PreMarshal *pm) { delete pm; }

// A caller's read set marshalled against the published dictionary snapshot,
// without the context lock.  false: no snapshot yet (the batch marshals it).
bool premarshal(hsc_ctx *c, const hsc_currangearr *a, uint64_t S, PreMarshal *pm)
{
    const MarshalDict *d = c->dict_cur.load(std::memory_order_acquire);
    if (!d || !a || !pm) return false;
    pm->epoch = d->epoch;
    pm->mp.clear();
    TableLookupT<MarshalDict> tl{d};
    marshal_txn(d, pm->mp, 0, S, a->size, [&, a](int k) {
        const hsc_currange *r = a->ranges[k];
        RangeRef x;
        x.tid = tl(r->tbname);
        x.idxnum = r->idxnum;
        x.lkey = (const uint8_t *)r->lkey;
        x.rkey = (const uint8_t *)r->rkey;
        x.lkeylen = r->lkeylen;
        x.rkeylen = r->rkeylen;
        x.lflag = r->lflag;
        x.rflag = r->rflag;
        x.islocked = r->islocked;
        return x;
    });
    return true;
}

int check_batch_pre(hsc_ctx *c, void *const *ranges, PreMarshal *const *pre, unsigned int *file,
                    unsigned int *offset, int n, int *rc_out)
{
    return check_batch(c, ranges, pre, file, offset, 0, n, rc_out);
}
}  // namespace hsc

extern "C" {

// A collector batch whose read sets were all premarshalled against the
// current dictionary snapshot: its columns are assembled into a stage of the
// context's pool BEFORE the context lock (the rows live in the callers'
// caches: copying them under the lock made every other leader wait), and
// the lock covers the window rules, the slot and the launch.  Rows of read
// sets the window rules decide are kept: a snapshot at or past the end of
// the log (rule 0) sees no write after it, so they cannot conflict; a forced
// conflict ORs in.  -> true when the batch was handled (rc set).
static bool check_batch_assembled(hsc_ctx *c, void *const *ranges, PreMarshal *const *pre, unsigned int *file,
                                  unsigned int *offset, int n, int *rc_out, int *rc)
{
    const MarshalDict *d = c->dict_cur.load(std::memory_order_acquire);
    if (!d || n > kSmallMaxTxns || c->multi || c->host_only) return false;
    size_t nr = 0, nl = 0;
    for (int i = 0; i < n; ++i) {
        if (!ranges[i] || !pre[i] || pre[i]->epoch != d->epoch) return false;
        nr += pre[i]->mp.gid.size();
        nl += pre[i]->mp.lock_table.size();
    }
    if (nr > kSmallMaxRanges || nl > kSmallMaxRanges) return false;
    Stage *st = nullptr;
    {
        std::lock_guard<std::mutex> g(c->pre_mu);
        if (c->pre_free.empty()) {
            c->pre_stages.emplace_back(new (std::nothrow) Stage());
            if (!c->pre_stages.back()) {
                c->pre_stages.pop_back();
                return false;
            }
            c->pre_free.push_back(c->pre_stages.back().get());
        }
        st = c->pre_free.back();
        c->pre_free.pop_back();
    }
    auto give_back = [&] {
        std::lock_guard<std::mutex> g(c->pre_mu);
        c->pre_free.push_back(st);
    };
    const int W = d->W;
    st->coh = true;
    st->L = stage_layout(W, nr, nl);
    if (st->arena.ensure(std::max<size_t>(st->L.total + small_tail((size_t)n), 256), true, true) ||
        st->forced.ensure((size_t)std::max(n, 1), true)) {
        give_back();
        return false;
    }
    uint64_t *lo = st->col<uint64_t>(st->L.lo), *hi = st->col<uint64_t>(st->L.hi);
    uint64_t *sn = st->col<uint64_t>(st->L.snap), *lsnap = st->col<uint64_t>(st->L.lock_snap);
    uint32_t *gid = st->col<uint32_t>(st->L.gid), *txn = st->col<uint32_t>(st->L.txn);
    uint32_t *ltab = st->col<uint32_t>(st->L.lock_table), *ltxn = st->col<uint32_t>(st->L.lock_txn);
    size_t o = 0, ol = 0;
    for (int i = 0; i < n; ++i) {
        const MarshalPart &q = pre[i]->mp;
        const size_t k = q.gid.size();
        for (size_t r = 0; r < k; ++r)
            for (int j = 0; j < W; ++j) {
                lo[(size_t)j * nr + o + r] = q.lohi[r * 2 * W + j];
                hi[(size_t)j * nr + o + r] = q.lohi[r * 2 * W + W + j];
            }
        if (k) {
            memcpy(gid + o, q.gid.data(), 4 * k);
            memcpy(sn + o, q.snap.data(), 8 * k);
            for (size_t r = 0; r < k; ++r) txn[o + r] = (uint32_t)i;
        }
        const size_t kl = q.lock_table.size();
        if (kl) {
            memcpy(ltab + ol, q.lock_table.data(), 4 * kl);
            memcpy(lsnap + ol, q.lock_snap.data(), 8 * kl);
            for (size_t r = 0; r < kl; ++r) ltxn[ol + r] = (uint32_t)i;
        }
        o += k, ol += kl;
    }
    st->n = nr, st->n_lock = nl, st->n_txn = (size_t)n;
    const auto tl0 = SteadyClock::now();
    std::unique_lock<std::mutex> lk(c->mu);
    c->sm_lock_ns.fetch_add(ns_since(tl0), std::memory_order_relaxed);
    (void)hipSetDevice(c->device);
    int r = ensure_built(c);
    // the snapshot the rows were marshalled against must still be the
    // dictionaries (a new group or a wider key since: the usual path)
    if (r != HSC_OK || c->dict_epoch != d->epoch || c->W != W || !small_path(c, n)) {
        lk.unlock();
        give_back();
        if (r == HSC_OK) return false;
        for (int i = 0; i < n; ++i) rc_out[i] = 1;
        *rc = r;
        return true;
    }
    publish_dict(c);
    const unsigned int ef = (unsigned int)(c->end_lsn >> 32), eo = (unsigned int)c->end_lsn;
    uint8_t *forced = st->forced.as<uint8_t>();
    for (int i = 0; i < n; ++i) {
        hsc_currangearr *a = (hsc_currangearr *)ranges[i];
        unsigned int *pf = file ? &file[i] : &a->file;
        unsigned int *po = offset ? &offset[i] : &a->offset;
        const uint64_t S = ((uint64_t)*pf << 32) | *po;
        *pf = ef, *po = eo;  // full mode: *file,*offset := curlsn
        forced[i] = full_forced(c, S) > 0;
    }
    const int k = small_launch(c, *st);
    if (k < 0) {
        lk.unlock();
        give_back();
        for (int i = 0; i < n; ++i) rc_out[i] = 1;
        *rc = k;
        return true;
    }
    c->sm_calls.fetch_add(1, std::memory_order_relaxed);
    hipStream_t s = c->small[k].stream;
    lk.unlock();
    give_back();  // the slot owns the columns now (its arena swapped in)
    if (const hipError_t e = small_fire(c, k); e != hipSuccess) {
        c->small[k].busy.store(false, std::memory_order_release);
        MuGuard g(c);
        for (int i = 0; i < n; ++i) rc_out[i] = 1;
        *rc = fail(c, HSC_EDEVICE, "small batch launch", e);
        return true;
    }
    const char *why = nullptr;
    hipError_t herr = hipSuccess;
    r = small_wait(c, k, s, rc_out, &why, &herr);
    if (r != HSC_OK) {
        MuGuard g(c);
        for (int i = 0; i < n; ++i) rc_out[i] = 1;
        *rc = fail(c, r, why, herr);
        return true;
    }
    *rc = HSC_OK;
    return true;
}

static int check_batch(hsc_ctx *c, void *const *ranges, PreMarshal *const *pre, unsigned int *file,
                       unsigned int *offset, int regop_only, int n, int *rc_out)
{
    if (!c || n < 0 || (n && (!ranges || !rc_out)) || (!file) != (!offset)) return HSC_EINVAL;
    if (regop_only && n > 0) {
        // every element from the published snapshot, without mu (the locked
        // path below only when some snapshot needs the log's record LSNs)
        bool all = true;
        for (int i = 0; i < n && all; ++i) {
            const hsc_currangearr *a = (const hsc_currangearr *)ranges[i];
            if (!a) {
                rc_out[i] = 0;
                continue;
            }
            const unsigned int f = file ? file[i] : a->file, o = offset ? offset[i] : a->offset;
            const int r = ctx_regop_fast(c, ((uint64_t)f << 32) | o);
            if (r < 0) all = false;
            rc_out[i] = r;
        }
        if (all) {
            c->rg_fast.fetch_add((uint64_t)n, std::memory_order_relaxed);
            return HSC_OK;
        }
        c->rg_slow.fetch_add((uint64_t)n, std::memory_order_relaxed);
    }
    static const bool assemble = getenv("HSC_NO_PRE_ASSEMBLE") == nullptr;  // (A/B diagnostics)
    if (assemble && pre && !regop_only && n > 0) {
        int rc = HSC_OK;
        if (check_batch_assembled(c, ranges, pre, file, offset, n, rc_out, &rc)) return rc;
    }
    const auto tl0 = SteadyClock::now();
    std::unique_lock<std::mutex> lk(c->mu);  // a small batch drops it while its kernel runs
    c->sm_lock_ns.fetch_add(ns_since(tl0), std::memory_order_relaxed);
    if (!c->host_only) (void)hipSetDevice(c->device);
    int rc = ensure_built(c);
    if (rc) {
        for (int i = 0; i < n; ++i) rc_out[i] = 1;
        return rc;
    }
    publish_dict(c);
    // per-thread scratch, reused across calls (a lone call allocates nothing)
    static thread_local std::vector<int> slot, rcs;  // slot: element -> txn index in the device batch
    static thread_local std::vector<hsc_currangearr *> full;
    static thread_local std::vector<PreMarshal *> fpre;
    static thread_local std::vector<uint64_t> snaps;
    // every element a full check (the batch entry's usual call): the caller's
    // arrays are the device batch as they are, verdicts land in rc_out
    bool dense = !regop_only;
    for (int i = 0; i < n && dense; ++i) dense = ranges[i] != nullptr;
    if (dense && n) {
        snaps.resize(n);
        const unsigned int ef = (unsigned int)(c->end_lsn >> 32), eo = (unsigned int)c->end_lsn;
        for (int i = 0; i < n; ++i) {
            hsc_currangearr *a = (hsc_currangearr *)ranges[i];
            unsigned int *pf = file ? &file[i] : &a->file;
            unsigned int *po = offset ? &offset[i] : &a->offset;
            snaps[i] = ((uint64_t)*pf << 32) | *po;
            *pf = ef, *po = eo;  // full mode: *file,*offset := curlsn
        }
        ArrSrc src{(hsc_currangearr *const *)ranges, snaps.data(), n};
        if (pre) src.pre = pre, src.epoch = c->dict_epoch;
        rc = check_src(c, src, rc_out, &lk);
        if (rc)
            for (int i = 0; i < n; ++i) rc_out[i] = 1;
        return rc;
    }
    slot.assign(n, -1);
    full.clear(), fpre.clear(), snaps.clear();
    for (int i = 0; i < n; ++i) {
        hsc_currangearr *a = (hsc_currangearr *)ranges[i];
        rc_out[i] = 0;
        if (!a) continue;  // bdb_osql_serial_check: ranges == NULL -> 0
        unsigned int *pf = file ? &file[i] : &a->file;
        unsigned int *po = offset ? &offset[i] : &a->offset;
        const uint64_t S = ((uint64_t)*pf << 32) | *po;
        if (regop_only) {
            rc_out[i] = regop_rc(c, S);
            continue;
        }
        *pf = (unsigned int)(c->end_lsn >> 32);  // full mode: *file,*offset := curlsn
        *po = (unsigned int)c->end_lsn;
        slot[i] = (int)full.size();
        full.push_back(a);
        snaps.push_back(S);
        if (pre) fpre.push_back(pre[i]);
    }
    if (full.empty()) return HSC_OK;
    rcs.assign(full.size(), 1);
    ArrSrc src{full.data(), snaps.data(), (int)full.size()};
    if (pre) src.pre = fpre.data(), src.epoch = c->dict_epoch;
    rc = check_src(c, src, rcs.data(), &lk);
    for (int i = 0; i < n; ++i)
        if (slot[i] >= 0) rc_out[i] = rc ? 1 : rcs[slot[i]];
    return rc;
}

}  // extern "C"

int hsc::ctx_regop_probe(hsc_ctx *c, void *ranges, unsigned int *file, unsigned int *offset)
{
    if (!ranges) return 0;
    hsc_currangearr *a = (hsc_currangearr *)ranges;
    const unsigned int f = file ? *file : a->file, o = offset ? *offset : a->offset;
    const int r = ctx_regop_fast(c, ((uint64_t)f << 32) | o);
    if (r >= 0) {
        c->rg_fast.fetch_add(1, std::memory_order_relaxed);
        return r;  // (regop_only leaves *file, *offset as they are)
    }
    int rc_out = 1;
    void *arr[1] = {ranges};
    const int rc = check_batch(c, arr, nullptr, file, offset, 1, 1, &rc_out);
    return rc ? 1 : rc_out;  // errors are "not serializable"
}

extern "C" {

int hsc_regop_stats(hsc_ctx *c, uint64_t out[2])
{
    if (!c || !out) return HSC_EINVAL;
    out[0] = c->rg_fast.load(std::memory_order_relaxed);
    out[1] = c->rg_slow.load(std::memory_order_relaxed);
    return HSC_OK;
}

int hsc_small_stats(hsc_ctx *c, hsc_small_stats_t *out)
{
    if (!c || !out) return HSC_EINVAL;
    out->calls = c->sm_calls.load();
    out->marshal_ns = c->sm_marshal_ns.load();
    out->launch_ns = c->sm_launch_ns.load();
    out->wait_ns = c->sm_wait_ns.load();
    out->slot_waits = c->sm_slot_waits.load();
    out->lock_ns = c->sm_lock_ns.load();
    return HSC_OK;
}

int hsc_batch_stats(hsc_ctx *c, hsc_batch_stats_t *out)
{
    if (!c || !out) return HSC_EINVAL;
    out->marshals = c->mb_marshals.load();
    out->read_sets = c->mb_txns.load();
    out->ranges = c->mb_ranges.load();
    out->parts_ns = c->mb_parts_ns.load();
    out->alloc_ns = c->mb_alloc_ns.load();
    out->assemble_ns = c->mb_assemble_ns.load();
    out->launch_ns = c->mb_launch_ns.load();
    out->wait_ns = c->mb_wait_ns.load();
    return HSC_OK;
}

int hsc_set_threads(hsc_ctx *c, int n)
{
    if (!c || n < 0) return HSC_EINVAL;
    MuGuard g(c);
    c->threads = n ? std::min(n, 256) : default_threads();
    return HSC_OK;
}

int hsc_set_autocollect(hsc_ctx *c, int on)
{
    if (!c || (on != 0 && on != 1)) return HSC_EINVAL;
    c->autocollect.store(on, std::memory_order_relaxed);
    return HSC_OK;
}

// The context's collector, created by the first call that needs it (a racing
// creator keeps the winner's and drops its own).
static hsc_collector *auto_collector(hsc_ctx *c)
{
    hsc_collector *k = c->auto_col.load(std::memory_order_acquire);
    if (k) return k;
    hsc_collector *mine = nullptr;
    if (hsc_collector_create(c, 0, 0, &mine) != HSC_OK) return nullptr;
    if (c->auto_col.compare_exchange_strong(k, mine, std::memory_order_acq_rel)) return mine;
    hsc_collector_destroy(mine);
    return k;
}

int hip_bdb_osql_serial_check(void *ctx, void *ranges, unsigned int *file, unsigned int *offset,
                              int regop_only)
{
    if (!ranges) return 0;
    hsc_ctx *c = (hsc_ctx *)ctx;
    if (c && regop_only) return ctx_regop_probe(c, ranges, file, offset);  // never queued
    if (c && c->autocollect.load(std::memory_order_relaxed))
        if (hsc_collector *k = auto_collector(c)) return hsc_collector_check(k, ranges, file, offset, regop_only);
    int rc_out = 1;
    void *arr[1] = {ranges};
    int rc = hip_serial_check_batch(ctx, arr, file, offset, regop_only, 1, &rc_out);
    return rc ? 1 : rc_out;  // errors are "not serializable"
}

int hsc_probe_device(hsc_ctx *c, const hsc_probe_batch *b)
{
    if (!c || !b) return HSC_EINVAL;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    if (c->dirty) return fail(c, HSC_ESTATE, "window not built");
    return probe(c, b);
}

int hsc_pack_verdicts(hsc_ctx *c, const uint8_t *verdict, size_t n_txn, uint64_t *bitmap)
{
    if (!c || (n_txn && (!verdict || !bitmap)) || n_txn > 0xFFFFFFFFull) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    if (!c->host_only) (void)hipSetDevice(c->device);
    HIPCHK(c, launch_pack(verdict, (uint32_t)n_txn, bitmap, c->stream));
    return HSC_OK;
}

int hsc_or_bitmaps(hsc_ctx *c, const uint64_t *parts, int nparts, size_t words, uint64_t *out)
{
    if (!c || nparts < 1 || (words && (!parts || !out))) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    HIPCHK(c, launch_or_bitmaps(parts, nparts, words, out, c->stream));
    return HSC_OK;
}

int hsc_synchronize(hsc_ctx *c)
{
    if (!c) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return collect_timing(c);
}

int hsc_get_timing(hsc_ctx *c, hsc_timing *t)
{
    if (!c || !t) return HSC_EINVAL;
    *t = c->last;
    return HSC_OK;
}

int hsc_enable_timing(hsc_ctx *c, int on)
{
    if (!c) return HSC_EINVAL;
    c->timing = on != 0;
    return HSC_OK;
}

}  // extern "C"

// Build c->graph from device-resident ops (edges and CSR/CSC), timed with
// events.  Caller holds c->mu.
static int graph_build_timed(hsc_ctx *c, const GraphInput &in, bool full, float *build_ms)
{
    hipStream_t s = c->stream;
    GraphBufs &gb = c->graph;
    hipEvent_t e0, e1;
    HIPCHK(c, hipEventCreate(&e0));
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventRecord(e0, s));
    GraphInput gi = in;
    if (gb.n_extra && c->x_max_txn >= in.ntxn) {  // staged rows would index past the CSR arrays
        gb.n_extra = 0;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        return fail(c, HSC_EINVAL, "a staged rw pair names a txn >= the build's ntxn");
    }
    if (gb.n_extra) {  // staged edges join this build, once
        gi.x_rows = gb.x_rows.as<uint64_t>();
        gi.x_type = gb.x_type.as<uint64_t>();
        gi.n_extra = gb.n_extra;
        gb.n_extra = 0;
    }
    gb.edge_bad = nullptr;
    gb.post = nullptr;
    hipError_t e = graph_build(gi, gb, full, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    // with the sync: the backward rows listed and the edge pass's check of the
    // observed ids (in.check)
    uint32_t post[3] = {0, 0, 0};
    if (e == hipSuccess && gb.post) e = hipMemcpyAsync(post, gb.post - 1, 12, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) (void)hipEventElapsedTime(build_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIPCHK(c, e);
    if (post[0] && gb.writer_packed) return fail(c, HSC_EDEVICE, "graph build: the writer sort's look-back stalled");
    gb.back_n = post[1];
    const uint32_t ebad = gb.edge_bad ? post[2] : 0;
    gb.bad |= ebad;
    if (ebad & 1) {
        c->graph_ntxn = 0;
        return fail(c, HSC_EINVAL, "history op out of range");
    }
    c->graph_ntxn = in.ntxn;
    return HSC_OK;
}

// Upload a history and build its graph into c->graph (edges and CSR/CSC).
// Caller holds c->mu.
static int graph_upload_build(hsc_ctx *c, const hsc_history *h, bool full, float *build_ms,
                              bool skip_rw = false)
{
    if (!h || (h->nops && (!h->txn || !h->key || !h->is_write || !h->observed)) ||
        h->nops > 0x7FFFFFFFull)
        return HSC_EINVAL;
    if (c->host_only) return fail(c, HSC_EDEVICE, "host-only context");
    (void)hipSetDevice(c->device);
    for (size_t i = 0; i < h->nops; ++i)
        if (h->txn[i] >= h->ntxn || h->observed[i] >= (int64_t)h->ntxn || h->observed[i] < -1)
            return fail(c, HSC_EINVAL, "history op out of range");
    hipStream_t s = c->stream;
    GraphBufs &gb = c->graph;
    const size_t n = h->nops;
    std::vector<uint32_t> obs(std::max<size_t>(n, 1));
    for (size_t i = 0; i < n; ++i) obs[i] = h->observed[i] < 0 ? 0xFFFFFFFFu : (uint32_t)h->observed[i];
    HIPCHK(c, gb.h_txn.ensure(4 * std::max<size_t>(n, 1)));
    HIPCHK(c, gb.h_key.ensure(8 * std::max<size_t>(n, 1)));
    HIPCHK(c, gb.h_isw.ensure(std::max<size_t>(n, 1)));
    HIPCHK(c, gb.h_obs.ensure(4 * std::max<size_t>(n, 1)));
    if (n) {
        HIPCHK(c, hipMemcpyAsync(gb.h_txn.p, h->txn, 4 * n, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(gb.h_key.p, h->key, 8 * n, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(gb.h_isw.p, h->is_write, n, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(gb.h_obs.p, obs.data(), 4 * n, hipMemcpyHostToDevice, s));
    }
    GraphInput in{gb.h_txn.as<uint32_t>(), gb.h_key.as<uint64_t>(), gb.h_isw.as<uint8_t>(),
                  gb.h_obs.as<uint32_t>(), n, h->ntxn};
    in.skip_rw = skip_rw;
    return graph_build_timed(c, in, full, build_ms);
}

// Edge and edge-type counts of c->graph into st (none after a raw build).
static int graph_edge_stats(hsc_ctx *c, hsc_graph_stats *st)
{
    GraphBufs &gb = c->graph;
    st->edges = gb.ne;
    uint64_t t[3] = {0, 0, 0};
    HIPCHK(c, graph_type_counts(gb, t, c->stream));
    st->ww = t[0];
    st->wr = t[1];
    st->rw = t[2];
    return HSC_OK;
}

static void scc_size_stats(const uint32_t *scc, uint32_t ntxn, hsc_graph_stats *st)
{
    std::vector<uint32_t> sz(std::max<uint32_t>(ntxn, 1), 0);
    for (uint32_t v = 0; v < ntxn; ++v)
        if (scc[v] < ntxn) sz[scc[v]]++;
    for (uint32_t v = 0; v < ntxn; ++v)
        if (sz[v] > 1) {
            st->nontrivial_sccs++;
            st->txns_in_cycles += sz[v];
        }
}

extern "C" {

int hsc_dep_graph_scc(hsc_ctx *c, const hsc_history *h, uint32_t *scc_out, hsc_graph_stats *st)
{
    if (!c || !h || (h->ntxn && !scc_out)) return HSC_EINVAL;
    MuGuard g(c);
    float build_ms = 0;
    int rc = graph_upload_build(c, h, true, &build_ms);
    if (rc) return rc;
    hipStream_t s = c->stream;
    GraphBufs &gb = c->graph;
    hipEvent_t e1, e2;
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventCreate(&e2));
    HIPCHK(c, hipEventRecord(e1, s));
    uint32_t rounds = 0, iters = 0;
    HIPCHK(c, graph_scc(h->ntxn, gb, &rounds, &iters, s));
    HIPCHK(c, hipEventRecord(e2, s));
    if (h->ntxn)
        HIPCHK(c, hipMemcpyAsync(scc_out, gb.scc.p, 4 * (size_t)h->ntxn, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (st) {
        memset(st, 0, sizeof *st);
        st->build_ms = build_ms;
        (void)hipEventElapsedTime(&st->scc_ms, e1, e2);
        rc = graph_edge_stats(c, st);
        if (rc) return rc;
        scc_size_stats(scc_out, h->ntxn, st);
        st->rounds = rounds;
        st->iterations = iters;
    }
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    return HSC_OK;
}

int hsc_dep_graph_build(hsc_ctx *c, const hsc_history *h, int flags, hsc_graph_stats *st)
{
    if (!c || !h) return HSC_EINVAL;
    MuGuard g(c);
    float build_ms = 0;
    int rc = graph_upload_build(c, h, (flags & HSC_GRAPH_FULL) != 0, &build_ms,
                                (flags & HSC_GRAPH_NO_RW) != 0);
    if (rc || !st) return rc;
    memset(st, 0, sizeof *st);
    st->build_ms = build_ms;
    return graph_edge_stats(c, st);
}

int hsc_dep_graph_build_device(hsc_ctx *c, size_t nops, uint32_t ntxn, const uint32_t *txn_dev,
                               const uint64_t *key_dev, const uint8_t *is_write_dev,
                               const uint32_t *observed_dev, int flags, hsc_graph_stats *st)
{
    if (!c || (nops && (!txn_dev || !key_dev || !is_write_dev || !observed_dev)) ||
        nops > 0x7FFFFFFFull)
        return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    GraphInput in{txn_dev, key_dev, is_write_dev, observed_dev, nops, ntxn};
    in.skip_rw = (flags & HSC_GRAPH_NO_RW) != 0;
    in.check = true;  // the ids and the txn order, in the build's first pass
    float build_ms = 0;
    int rc = graph_build_timed(c, in, (flags & HSC_GRAPH_FULL) != 0, &build_ms);
    if (rc && (c->graph.bad & 1)) return fail(c, HSC_EINVAL, "history op out of range");
    if (rc || !st) return rc;
    memset(st, 0, sizeof *st);
    st->build_ms = build_ms;
    return graph_edge_stats(c, st);
}

int hsc_dep_graph_stage_rw_pairs(hsc_ctx *c, uint32_t nrs, const uint32_t *readset_txn,
                                 size_t ncommit, const uint64_t *commit_lsn,
                                 const uint32_t *commit_txn)
{
    if (!c || (nrs && !readset_txn) || (ncommit && (!commit_lsn || !commit_txn)))
        return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    for (size_t i = 1; i < ncommit; ++i)
        if (commit_lsn[i] <= commit_lsn[i - 1]) return fail(c, HSC_EINVAL, "commit LSNs not sorted");
    hipStream_t s = c->stream;
    GraphBufs &gb = c->graph;
    const size_t n = c->e_dev_n;
    gb.n_extra = 0;
    // every endpoint a pair can map to; graph_build_timed rejects the staged
    // rows if the build's ntxn does not cover them
    uint32_t xm = 0;
    for (uint32_t i = 0; i < nrs; ++i) xm = std::max(xm, readset_txn[i]);
    for (size_t i = 0; i < ncommit; ++i) xm = std::max(xm, commit_txn[i]);
    c->x_max_txn = xm;
    if (n == 0) return HSC_OK;
    // mapping tables next to each other: rs_txn[nrs] | commit_txn[ncommit] | commit_lsn[ncommit]
    const size_t o_ct = ((size_t)nrs + 1) & ~(size_t)1, o_cl = o_ct + ncommit + (ncommit & 1);
    HIPCHK(c, gb.x_map.ensure(4 * (o_cl + 2 * ncommit) + 64));
    uint32_t *m32 = gb.x_map.as<uint32_t>();
    uint64_t *cl = (uint64_t *)(m32 + o_cl);
    uint32_t *bad = m32 + o_cl + 2 * ncommit;
    if (nrs) HIPCHK(c, hipMemcpyAsync(m32, readset_txn, 4 * (size_t)nrs, hipMemcpyHostToDevice, s));
    if (ncommit) {
        HIPCHK(c, hipMemcpyAsync(m32 + o_ct, commit_txn, 4 * ncommit, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(cl, commit_lsn, 8 * ncommit, hipMemcpyHostToDevice, s));
    }
    HIPCHK(c, hipMemsetAsync(bad, 0, 4, s));
    HIPCHK(c, gb.x_rows.ensure(8 * n));
    HIPCHK(c, gb.x_type.ensure(8 * n));
    HIPCHK(c, graph_pairs_rows(n, c->e_dev_txn, c->e_dev_lsn, nrs, m32, ncommit, cl, m32 + o_ct,
                               gb.x_rows.as<uint64_t>(), gb.x_type.as<uint64_t>(), bad, s));
    uint32_t hb = 0;
    HIPCHK(c, hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (hb) return fail(c, HSC_EINVAL, "rw pair names a writer LSN or read set not in the map");
    gb.n_extra = n;
    return HSC_OK;
}

int hsc_dep_graph_scc_built(hsc_ctx *c, uint32_t *scc_out, hsc_graph_stats *st)
{
    if (!c) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    GraphBufs &gb = c->graph;
    const uint32_t nn = c->graph_ntxn;
    if (nn && !scc_out) return HSC_EINVAL;
    if (gb.raw) return fail(c, HSC_ESTATE, "last build kept raw rows only (no HSC_GRAPH_FULL)");
    hipStream_t s = c->stream;
    hipEvent_t e1, e2;
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventCreate(&e2));
    HIPCHK(c, hipEventRecord(e1, s));
    uint32_t rounds = 0, iters = 0;
    HIPCHK(c, graph_scc(nn, gb, &rounds, &iters, s));
    HIPCHK(c, hipEventRecord(e2, s));
    if (nn) HIPCHK(c, hipMemcpyAsync(scc_out, gb.scc.p, 4 * (size_t)nn, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (st) {
        memset(st, 0, sizeof *st);
        (void)hipEventElapsedTime(&st->scc_ms, e1, e2);
        const int rc = graph_edge_stats(c, st);
        if (rc) return rc;
        scc_size_stats(scc_out, nn, st);
        st->rounds = rounds;
        st->iterations = iters;
    }
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    return HSC_OK;
}

int hsc_dep_graph_cover(hsc_ctx *c, uint8_t *cover_dev)
{
    if (!c || (c->graph_ntxn && !cover_dev)) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    HIPCHK(c, graph_cover(c->graph, c->graph_ntxn, cover_dev, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return HSC_OK;
}

int hsc_dep_graph_cut(hsc_ctx *c, const uint8_t *cover_dev, uint64_t *rows_dev, size_t cap,
                      size_t *m)
{
    if (!c || !m || (c->graph_ntxn && !cover_dev)) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    HIPCHK(c, graph_cut(c->graph, cover_dev, m, c->stream));
    const size_t k = std::min(cap, *m);
    if (k && rows_dev)
        HIPCHK(c, hipMemcpyAsync(rows_dev, c->graph.cut.p, 8 * k, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return HSC_OK;
}

int hsc_dep_graph_scc_cut(hsc_ctx *c, uint32_t ntxn, const uint8_t *cover_dev,
                          const uint64_t *rows_dev, size_t m, uint32_t *scc_dev,
                          hsc_graph_stats *st)
{
    if (!c || (ntxn && (!cover_dev || !scc_dev)) || (m && !rows_dev) || m > 0xFFFFFFFFull)
        return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    hipStream_t s = c->stream;
    hipEvent_t e1, e2;
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventCreate(&e2));
    HIPCHK(c, hipEventRecord(e1, s));
    uint32_t rounds = 0, iters = 0, nc = 0;
    hipError_t e = graph_scc_rows(ntxn, cover_dev, rows_dev, m, c->subgraph, scc_dev, &nc, &rounds,
                                  &iters, s);
    if (e == hipErrorInvalidValue) {
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
        return fail(c, HSC_EINVAL, "cut row outside the cover");
    }
    HIPCHK(c, e);
    HIPCHK(c, hipEventRecord(e2, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (st) {
        memset(st, 0, sizeof *st);
        st->edges = c->subgraph.ne;
        (void)hipEventElapsedTime(&st->scc_ms, e1, e2);
        st->rounds = rounds;
        st->iterations = iters;
        st->cut_nodes = nc;
        // components of >= 2 txns live in the cut: its nc colours suffice
        std::vector<uint32_t> h(std::max<uint32_t>(nc, 1));
        if (nc) HIPCHK(c, hipMemcpy(h.data(), c->subgraph.scc.p, 4 * (size_t)nc, hipMemcpyDeviceToHost));
        scc_size_stats(h.data(), nc, st);
    }
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    return HSC_OK;
}

int hsc_dep_graph_edges(hsc_ctx *c, uint32_t *src, uint32_t *dst, uint32_t *type, size_t cap,
                        size_t *n)
{
    if (!c || !n) return HSC_EINVAL;
    if (c->host_only) return HSC_EDEVICE;
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    GraphBufs &gb = c->graph;
    *n = gb.ne;
    const size_t m = std::min(cap, gb.ne);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (m && src) HIPCHK(c, hipMemcpy(src, gb.src.p, 4 * m, hipMemcpyDeviceToHost));
    if (m && dst) HIPCHK(c, hipMemcpy(dst, gb.out_dst.p, 4 * m, hipMemcpyDeviceToHost));
    if (m && type) HIPCHK(c, hipMemcpy(type, gb.type.p, 4 * m, hipMemcpyDeviceToHost));
    return HSC_OK;
}

}  // extern "C"

// ---- internals the multi-GPU context drives its members with (hsc_ctx.h) ----
namespace hsc {
int ctx_fail(hsc_ctx *c, int code, const char *what, hipError_t e) { return fail(c, code, what, e); }
int ctx_window_words(hsc_ctx *c) { return window_words(c); }
void ctx_clear_window(hsc_ctx *c) { clear_window(c); }
int ctx_ensure_built(hsc_ctx *c) { return ensure_built(c); }
void ctx_add_write(hsc_ctx *c, int tid, int ix, const uint8_t *key, int keylen, bool has_key, uint64_t lsn)
{
    add_write(c, tid, ix, key, keylen, has_key, lsn);
}
int ctx_flush_appends(hsc_ctx *c, bool lazy) { return flush_appends(c, lazy); }
void ctx_raise_table_max(hsc_ctx *c, int tid, uint64_t lsn) { raise_table_max(c, tid, lsn); }
int ctx_probe(hsc_ctx *c, const hsc_probe_batch *b) { return probe(c, b); }
int ctx_default_threads() { return default_threads(); }
void ctx_par_for(hsc_ctx *c, int nwork, const std::function<void(int)> &f) { par_for(c, true, nwork, f, true); }

// The first and the last row of a built window: gid[2], words[2][W] (row
// 0's W words, then row n - 1's).
int ctx_edge_keys(hsc_ctx *c, uint32_t *gid, uint64_t *words)
{
    MuGuard g(c);
    if (c->dirty || !c->n || c->host_only) return fail(c, HSC_ESTATE, "no built window");
    (void)hipSetDevice(c->device);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t last = c->n - 1;
    HIPCHK(c, hipMemcpy(gid, c->d_gid.as<uint32_t>(), 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(gid + 1, c->d_gid.as<uint32_t>() + last, 4, hipMemcpyDeviceToHost));
    for (int j = 0; j < c->W; ++j) {
        HIPCHK(c, hipMemcpy(words + j, c->d_words.as<uint64_t>() + (size_t)j * c->cap, 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(words + c->W + j, c->d_words.as<uint64_t>() + (size_t)j * c->cap + last, 8,
                            hipMemcpyDeviceToHost));
    }
    return HSC_OK;
}

// The cut of the last build under cover (one pass: count + rows); *rows
// points into the context's own buffer until its next graph call.
int ctx_graph_cut(hsc_ctx *c, const uint8_t *cover, size_t *m, const uint64_t **rows, const uint32_t *op_txn,
                  const uint64_t *op_key, const uint8_t *op_isw)
{
    MuGuard g(c);
    (void)hipSetDevice(c->device);
    HIPCHK(c, graph_cut(c->graph, cover, m, c->stream, op_txn, op_key, op_isw, false));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *rows = c->graph.cut.as<uint64_t>();
    return HSC_OK;
}

bool ctx_small_fits(hsc_ctx *c, size_t n_txn, size_t n, size_t n_lock)
{
    return n_txn <= (size_t)kSmallMaxTxns && small_path(c, (int)n_txn) && n <= kSmallMaxRanges &&
           n_lock <= kSmallMaxRanges;
}

// A batch a multi context's front marshalled and routed to member c
// (hsc_multi.cpp, multi_check_stage).  A batch that fits the small path
// (st.coh: its arena is fine-grained with the slot's tail) takes one of c's
// slots -- its kernel reads the columns where the routing wrote them -- and
// *slot is the slot; else one staged upload + probe + verdict download on
// c->stream (*slot = -1).  Takes c->mu for the launch only.
int ctx_stage_launch(hsc_ctx *c, Stage &st, int *slot)
{
    std::unique_lock<std::mutex> lk(c->mu);
    (void)hipSetDevice(c->device);
    *slot = -1;
    if (c->dirty) return fail(c, HSC_ESTATE, "member window not built");
    if (st.coh && ctx_small_fits(c, st.n_txn, st.n, st.n_lock)) {
        const int k = small_launch(c, st);
        if (k < 0) return k;
        c->sm_calls.fetch_add(1, std::memory_order_relaxed);
        lk.unlock();
        if (const hipError_t e = small_fire(c, k); e != hipSuccess) {
            c->small[k].busy.store(false, std::memory_order_release);
            lk.lock();
            return fail(c, HSC_EDEVICE, "small batch launch", e);
        }
        *slot = k;
        return HSC_OK;
    }
    const int rc = launch_stage(c, st);
    if (rc) (void)hipStreamSynchronize(c->stream);
    return rc;
}

// The verdicts of ctx_stage_launch's batch: rc_out[t] = forced | conflict.
int ctx_stage_wait(hsc_ctx *c, Stage &st, int slot, int *rc_out)
{
    if (slot >= 0) {
        const char *why = nullptr;
        hipError_t herr = hipSuccess;
        const int rc = small_wait(c, slot, c->small[slot].stream, rc_out, &why, &herr);
        if (rc == HSC_OK) return HSC_OK;
        MuGuard g(c);
        return fail(c, rc, why, herr);
    }
    (void)hipSetDevice(c->device);
    return finish_stage(c, st, rc_out);
}
}  // namespace hsc
