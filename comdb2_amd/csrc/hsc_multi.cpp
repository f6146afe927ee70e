// hsc_multi.cpp -- the multi-GPU context (include/hip_serial.h, hsc_multi_*;
// SURVEY.md §8(e)).
//
// A multi context is an hsc_ctx like any other -- hip_serial_check_batch,
// hip_bdb_osql_serial_check, the collector, the log ingest and append entry
// points all take it -- whose window is cut into `world` contiguous pieces of
// the composite key space (gid, key words), one per member context.  The
// front context keeps what the reference keeps per check (the log decode, the
// dictionaries, the window rules of bdb/serializable.c:390-539) and marshals
// each batch on the host exactly as a one-GPU context does; the device work
// is spread over the members:
//
//   1. every member takes a share of the marshalled probes (its own read sets
//      on a per-rank context) and counts, per destination member, the probes
//      whose [lo, hi] overlaps that member's piece (k_route_count);
//   2. the counts go to every member (host memory in one process, an RCCL
//      all-gather across ranks): destination sizes and row offsets;
//   3. k_route_scatter copies every probe to its destinations -- straight
//      into their probe columns when the members share a process (peer
//      stores over xGMI, or plain stores on one GPU), else into one send
//      block per destination that RCCL sends (grouped ncclSend / ncclRecv)
//      and the receiver unpacks (k_route_unpack);
//   4. every member runs the one-GPU probe pipeline over what it received,
//      read sets numbered batch-wide, and packs its verdict bitmap;
//   5. the bitmaps are OR-ed per read-set owner (k_or_slices over the
//      members' bitmaps in one process; RCCL send / receive of each owner's
//      slice, then k_or_slices with the owner's own slice, across ranks).
// A read set's verdict is the OR of its probes' verdicts and a member holding
// none of a probe's keys cannot report a conflict for it, so the verdicts are
// those of one context holding the whole window.
#include "hsc_ctx.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

namespace hsc {

using SteadyClock = std::chrono::steady_clock;

// ---- RCCL, resolved at run time ---------------------------------------------
// librccl.so.1 is dlopen'ed on first use (the copy torch loaded, when it did),
// so the library itself loads on hosts without it (the CPU test suite).
struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*ErrorString)(ncclResult_t) = nullptr;
};

static Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.err = std::string("librccl not found: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto &f, const char *name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            if (!f) all = false;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.AllGather, "ncclAllGather");
        sym(r.AllReduce, "ncclAllReduce");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.ErrorString, "ncclGetErrorString");
        r.ok = all;
        if (!all) r.err = "librccl lacks an entry point";
    });
    return r;
}

constexpr int kMultiLanes = 2;  // batches in flight (hsc_multi_probe_device lanes)

// One member's scratch for one lane.
struct MLane {
    hipStream_t stream = nullptr;
    DBuf src;             // API path: the member's share of the batch (StageLayout `srcL`)
    StageLayout srcL;
    DBuf hist, totals, ctl;  // ctl: the scatter's cursors (zeroed by k_route_total)
    DBuf send, raw;       // RCCL: send blocks / received blocks
    DBuf recv;            // the probe columns routed to this member (StageLayout `recvL`)
    StageLayout recvL;
    DBuf verdict, bitmap; // this member's probe outputs over the batch-wide read sets
    DBuf gather, out;     // owner merge (RCCL gather) / the merged bitmap (API path)
    HBuf h_io;            // pinned: the merged bitmap's download (API path)
    HBuf h_cnt;           // fine-grained pinned: the counts the device publishes, + seq word
    uint32_t seq = 0;
    hipEvent_t ev_count = nullptr, ev_scatter = nullptr, ev_probe = nullptr, ev_done = nullptr;
    bool used = false;    // ev_done recorded
};

struct Multi {
    int world = 1;   // members of the partition
    int nlocal = 1;  // members in this process
    int rank = 0;    // global member index of local member 0
    bool rccl = false;
    hsc_ctx *mem[kMultiMax] = {};
    ncclComm_t comm[kMultiLanes] = {};
    MLane lane[kMultiLanes][kMultiMax];
    // partition: S = world - 1 splitters (gid, key words)
    bool sp_given = false;
    int sp_W = 1;
    std::vector<uint32_t> sp_gid;
    std::vector<uint64_t> sp_w;  // [sp_W][S]
    // the splitters as the routing uses them: exactly W words (zero-extended
    // or cut), the same on the host (rows, appends) and on the devices (probes)
    std::vector<uint64_t> eff_w;  // [d_sp_W][S]
    DBuf d_sp[kMultiMax];        // per local member: gid [S] then words [W][S] at d_sp_woff
    size_t d_sp_woff = 0;
    int d_sp_W = 0;              // words of the uploaded copy (0: stale)
    bool adopted = false;        // members' windows ingested directly (hsc_multi_adopt)
    // host copies of the last pipeline's counts
    std::vector<uint32_t> cnt;   // [world][world + 2]: per source s: to each d, n_lock, n_txn
    uint64_t batches = 0, routed = 0, probes = 0;
    // host phase split of run_pipeline (ns): waiting for the lane's previous
    // batch, launching the counts, waiting for them, enqueueing the rest
    uint64_t ns_lane = 0, ns_count = 0, ns_count_wait = 0, ns_enqueue = 0;
};

static int mfail(hsc_ctx *c, int code, const char *what, hipError_t e = hipSuccess)
{
    return ctx_fail(c, code, what, e);
}

#define MCHK(c, call)                                                       \
    do {                                                                    \
        hipError_t e_ = (call);                                             \
        if (e_ != hipSuccess) return mfail((c), HSC_EDEVICE, #call, e_);    \
    } while (0)
#define MRC(call)                          \
    do {                                   \
        const int rc_ = (call);            \
        if (rc_ != HSC_OK) return rc_;     \
    } while (0)
#define NCHK(c, call)                                                                    \
    do {                                                                                 \
        ncclResult_t r_ = (call);                                                        \
        if (r_ != ncclSuccess) {                                                         \
            std::string m_ = std::string(#call) + ": " + rccl().ErrorString(r_);        \
            return mfail((c), HSC_EDEVICE, m_.c_str());                                  \
        }                                                                                \
    } while (0)

static inline size_t r64(size_t x) { return (x + 63) & ~(size_t)63; }

// ---- composite keys ---------------------------------------------------------
// Row i of the front's host-staged window as (gid, W words).
static void row_key(const hsc_ctx *f, size_t i, int W, uint64_t *out)
{
    uint8_t buf[kMaxWords * 8];
    memset(buf, 0, (size_t)W * 8);
    const int klen = f->groups[f->h_gid[i]].klen;
    if (klen) memcpy(buf, f->h_keys.data() + f->h_keyoff[i], (size_t)std::min(klen, 8 * W));
    for (int j = 0; j < W; ++j) out[j] = load_be64(buf + 8 * j);
}

// composite (g, x[W]) vs splitter k as routed (eff_w, W = d_sp_W words)
static int sp_cmp(const Multi *M, uint32_t g, const uint64_t *x, int W, int k)
{
    const size_t S = M->sp_gid.size();
    if (g != M->sp_gid[k]) return g < M->sp_gid[k] ? -1 : 1;
    for (int j = 0; j < W; ++j) {
        const uint64_t b = M->eff_w[(size_t)j * S + k];
        if (x[j] != b) return x[j] < b ? -1 : 1;
    }
    return 0;
}

static int sp_owner(const Multi *M, uint32_t g, const uint64_t *x, int W)
{
    int lo = 0, hi = (int)M->sp_gid.size();
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sp_cmp(M, g, x, W, mid) >= 0)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Splitters at equal-count quantiles of the staged rows (every version
// counts: a row is probe-phase work of its member), from an evenly spaced
// sample of at most 2^16 rows; every rank of a per-rank context computes the
// same ones from the same log.
static void auto_splitters(hsc_ctx *f, Multi *M, int W)
{
    const size_t n = f->h_gid.size(), S = (size_t)M->world - 1;
    M->sp_W = W;
    M->sp_gid.assign(S, 0);
    M->sp_w.assign((size_t)W * S, 0);
    M->d_sp_W = 0;  // new splitters: upload again
    if (!S || !n) return;
    const size_t m = std::min<size_t>(n, 1u << 16);
    std::vector<uint64_t> keys(m * (size_t)(W + 1));
    for (size_t k = 0; k < m; ++k) {
        const size_t i = (size_t)((unsigned __int128)k * n / m);
        keys[k * (W + 1)] = f->h_gid[i];
        row_key(f, i, W, &keys[k * (W + 1) + 1]);
    }
    std::vector<uint32_t> ord(m);
    for (size_t k = 0; k < m; ++k) ord[k] = (uint32_t)k;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
        return std::lexicographical_compare(&keys[(size_t)a * (W + 1)], &keys[(size_t)a * (W + 1) + W + 1],
                                            &keys[(size_t)b * (W + 1)], &keys[(size_t)b * (W + 1) + W + 1]);
    });
    for (size_t s = 0; s < S; ++s) {
        const uint64_t *k = &keys[(size_t)ord[(s + 1) * m / (S + 1)] * (W + 1)];
        M->sp_gid[s] = (uint32_t)k[0];
        for (int j = 0; j < W; ++j) M->sp_w[(size_t)j * S + s] = k[1 + j];
    }
}

// The splitters on every local member's device, zero-extended to W words.
static int upload_splitters(hsc_ctx *f, Multi *M, int W)
{
    if (M->d_sp_W == W) return HSC_OK;
    const size_t S = M->sp_gid.size();
    std::vector<uint64_t> &w = M->eff_w;
    w.assign((size_t)W * std::max<size_t>(S, 1), 0);
    for (int j = 0; j < std::min(W, M->sp_W); ++j)
        for (size_t k = 0; k < S; ++k) w[(size_t)j * S + k] = M->sp_w[(size_t)j * S + k];
    M->d_sp_woff = (4 * std::max<size_t>(S, 1) + 15) & ~(size_t)15;
    for (int m = 0; m < M->nlocal; ++m) {
        MCHK(f, hipSetDevice(M->mem[m]->device));
        MCHK(f, M->d_sp[m].ensure(M->d_sp_woff + 8 * w.size()));
        if (S) {
            MCHK(f, hipMemcpy(M->d_sp[m].p, M->sp_gid.data(), 4 * S, hipMemcpyHostToDevice));
            MCHK(f, hipMemcpy(M->d_sp[m].as<uint8_t>() + M->d_sp_woff, w.data(), 8 * w.size(),
                              hipMemcpyHostToDevice));
        }
    }
    M->d_sp_W = W;
    return HSC_OK;
}

static RouteSplit split_view(const Multi *M, int m, int W)
{
    RouteSplit sp{};
    sp.S = (int)M->sp_gid.size();
    sp.W = W;
    sp.gid = M->d_sp[m].as<uint32_t>();
    sp.w = (const uint64_t *)(M->d_sp[m].as<uint8_t>() + M->d_sp_woff);
    return sp;
}

// ---- dictionaries -------------------------------------------------------------
// Members carry a copy of the front's dictionaries (same table ids, same
// gids, same key words), refreshed whenever the front's grow.
void multi_sync_dict(hsc_ctx *f)
{
    Multi *M = f->multi;
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        std::lock_guard<std::mutex> g(c->mu);
        if (c->table_names.size() != f->table_names.size() || c->groups.size() != f->groups.size())
            c->dict_epoch++;
        c->table_ids = f->table_ids;
        c->table_names = f->table_names;
        c->group_ids = f->group_ids;
        c->groups = f->groups;
        c->ix_groups = f->ix_groups;
        if (c->h_table_max.size() < f->h_table_max.size()) c->h_table_max.resize(f->h_table_max.size(), 0);
    }
}

// ---- window -------------------------------------------------------------------
// Build the members' windows from the front's host-staged rows (a decoded log
// or appended writes): the rows of each member's piece, in log order.
int multi_build(hsc_ctx *f)
{
    Multi *M = f->multi;
    if (!f->host_staged) {  // hsc_multi_adopt: the members' windows are the window
        if (!f->dirty) return HSC_OK;
        return mfail(f, HSC_ESTATE, "multi context: members were ingested directly; re-ingest them");
    }
    M->adopted = false;
    const int W = ctx_window_words(f);
    if (f->W != W) f->dict_epoch++;
    f->W = W;
    if (!M->sp_given) auto_splitters(f, M, W);
    MRC(upload_splitters(f, M, W));  // before the rows are placed: one routing rule
    multi_sync_dict(f);
    const size_t n = f->h_gid.size();
    std::vector<int> own(n);
    std::vector<uint64_t> x((size_t)W);
    for (size_t i = 0; i < n; ++i) {
        row_key(f, i, W, x.data());
        own[i] = sp_owner(M, f->h_gid[i], x.data(), W);
    }
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        const int me = M->rank + m;
        std::lock_guard<std::mutex> g(c->mu);
        (void)hipSetDevice(c->device);
        ctx_clear_window(c);
        c->end_lsn = f->end_lsn;
        c->h_table_max = f->h_table_max;
        c->max_commit = f->max_commit;
        for (size_t i = 0; i < n; ++i) {
            if (own[i] != me) continue;
            c->h_gid.push_back(f->h_gid[i]);
            c->h_keyoff.push_back(c->h_keys.size());
            const int klen = f->groups[f->h_gid[i]].klen;
            c->h_keys.insert(c->h_keys.end(), f->h_keys.data() + f->h_keyoff[i],
                             f->h_keys.data() + f->h_keyoff[i] + klen);
            c->h_lsn.push_back(f->h_lsn[i]);
        }
        const int rc = ctx_ensure_built(c);
        if (rc) return mfail(f, rc, ("member build: " + c->err).c_str());
        c->live = true;
        c->dirty = false;
    }
    size_t keys = 0;
    for (int m = 0; m < M->nlocal; ++m) keys += M->mem[m]->n;
    f->n = keys;
    f->dirty = false;
    f->live = true;
    f->merge_pending = false;
    f->ng_built = f->groups.size();
    f->app_gid.clear(), f->app_keys.clear(), f->app_koff.clear(), f->app_lsn.clear();
    f->app_tmax = false;
    return HSC_OK;
}

// Rows appended to a built window go to their owners' delta runs.
int multi_flush_appends(hsc_ctx *f)
{
    Multi *M = f->multi;
    if (!f->live) return HSC_OK;
    if (M->adopted) return mfail(f, HSC_ESTATE, "multi context: append to the members' windows directly");
    const int W = ctx_window_words(f);
    if (f->groups.size() > f->ng_built || W > f->W) {  // the pieces' tables were sized at the build
        f->dirty = true;
        f->app_gid.clear(), f->app_keys.clear(), f->app_koff.clear(), f->app_lsn.clear();
        return HSC_OK;
    }
    if (f->app_gid.empty() && !f->app_tmax) return HSC_OK;
    multi_sync_dict(f);
    std::vector<uint64_t> x((size_t)W);
    std::vector<std::vector<size_t>> rows(M->nlocal);
    for (size_t i = 0; i < f->app_gid.size(); ++i) {
        const int klen = f->groups[f->app_gid[i]].klen;
        uint8_t buf[kMaxWords * 8];
        memset(buf, 0, (size_t)W * 8);
        if (klen) memcpy(buf, f->app_keys.data() + f->app_koff[i], (size_t)klen);
        for (int j = 0; j < W; ++j) x[j] = load_be64(buf + 8 * j);
        const int o = sp_owner(M, f->app_gid[i], x.data(), W) - M->rank;
        if (o >= 0 && o < M->nlocal) rows[o].push_back(i);
    }
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        std::lock_guard<std::mutex> g(c->mu);
        (void)hipSetDevice(c->device);
        for (size_t t = 0; t < f->h_table_max.size(); ++t)
            if (f->h_table_max[t] > c->h_table_max[t]) c->h_table_max[t] = f->h_table_max[t], c->app_tmax = true;
        c->max_commit = std::max(c->max_commit, f->max_commit);
        c->end_lsn = f->end_lsn;
        for (size_t i : rows[m]) {
            const GroupInfo &gi = f->groups[f->app_gid[i]];
            ctx_add_write(c, gi.tid, gi.ix, f->app_keys.data() + f->app_koff[i], gi.klen, true, f->app_lsn[i]);
        }
        const int rc = ctx_flush_appends(c);
        if (rc) return mfail(f, rc, ("member append: " + c->err).c_str());
        if (c->dirty) {  // the member folds inline: rebuild it now (its rows are host-staged)
            const int rb = ctx_ensure_built(c);
            if (rb) return mfail(f, rb, ("member rebuild: " + c->err).c_str());
            c->live = true;
        }
    }
    f->app_gid.clear(), f->app_keys.clear(), f->app_koff.clear(), f->app_lsn.clear();
    f->app_tmax = false;
    return HSC_OK;
}

// ---- the routed probe pipeline -------------------------------------------------
struct MSource {          // one local member's source batch (device columns)
    ProbeView p;
    uint32_t n_txn;       // read sets this source numbers (its own: per-rank; the batch's: shared)
    uint64_t *out;        // the merged bitmap of the read sets it owns (nullptr: not an owner)
};

static int lane_stream(hsc_ctx *f, Multi *M, int L, int m)
{
    MLane &ml = M->lane[L][m];
    if (ml.stream) return HSC_OK;
    MCHK(f, hipSetDevice(M->mem[m]->device));
    MCHK(f, hipStreamCreateWithFlags(&ml.stream, hipStreamNonBlocking));
    for (hipEvent_t *e : {&ml.ev_count, &ml.ev_scatter, &ml.ev_probe, &ml.ev_done})
        MCHK(f, hipEventCreateWithFlags(e, hipEventDisableTiming));
    return HSC_OK;
}

// Probe columns of a StageLayout arena as a route target (stride = n).
static RouteTarget arena_target(uint8_t *base, const StageLayout &L, size_t n)
{
    RouteTarget t{};
    t.lo = (uint64_t *)(base + L.lo);
    t.hi = (uint64_t *)(base + L.hi);
    t.snap = (uint64_t *)(base + L.snap);
    t.gid = (uint32_t *)(base + L.gid);
    t.txn = (uint32_t *)(base + L.txn);
    t.stride = n;
    t.lock_snap = (uint64_t *)(base + L.lock_snap);
    t.lock_table = (uint32_t *)(base + L.lock_table);
    t.lock_txn = (uint32_t *)(base + L.lock_txn);
    return t;
}

// A send block (route_block_bytes layout) as a route target.
static RouteTarget block_target(uint8_t *b, int W, size_t n, size_t nl)
{
    RouteTarget t{};
    t.lo = (uint64_t *)b;
    t.hi = t.lo + (size_t)W * n;
    t.snap = t.hi + (size_t)W * n;
    t.gid = (uint32_t *)(t.snap + n);
    t.txn = t.gid + n;
    t.stride = n;
    t.lock_snap = (uint64_t *)(b + route_block_bytes(W, n, 0));
    t.lock_table = (uint32_t *)(t.lock_snap + nl);
    t.lock_txn = t.lock_table + nl;
    return t;
}

// shared: the local sources number the same read sets (one batch split by
// probe; member 0 owns every verdict); else each source numbers its own read
// sets and owns their verdicts (per-rank batches, hsc_multi_probe_device).
static int run_pipeline(hsc_ctx *f, int L, MSource *src, bool shared)
{
    Multi *M = f->multi;
    const int N = M->world, NL = M->nlocal, W = f->W;
    const int C = N + 2;
    const auto t0 = SteadyClock::now();
    if (M->d_sp_W != W) MRC(upload_splitters(f, M, W));
    for (int m = 0; m < NL; ++m) {
        MRC(lane_stream(f, M, L, m));
        MLane &ml = M->lane[L][m];
        if (ml.used) MCHK(f, hipEventSynchronize(ml.ev_done));  // this lane's last batch
    }
    const auto t1 = SteadyClock::now();
    Rccl &R = rccl();
    // 1. counts per destination: the count kernel's last block (or, across
    // ranks, a one-block copy after the all-gather) stores them to pinned host
    // memory with a sequence word the host spins on -- no copy, no event wait
    M->cnt.assign((size_t)N * C, 0);
    const bool gather = M->rccl && N > 1;
    const size_t hw = gather ? (size_t)C * N : (size_t)C;  // words published
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        hipStream_t s = ml.stream;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        const uint32_t nb = std::max<uint32_t>(route_blocks(src[m].p.n), 1);
        MCHK(f, ml.hist.ensure(4 * (size_t)nb * N));
        MCHK(f, ml.totals.ensure(4 * (size_t)C * (N + 1)));
        if (!ml.ctl.p) {
            MCHK(f, ml.ctl.ensure(4 * (2 * (size_t)kMultiMax + 2)));
            MCHK(f, hipMemsetAsync(ml.ctl.p, 0, ml.ctl.bytes, s));
        }
        if (ml.h_cnt.ensure(4 * ((size_t)C * kMultiMax + 1), true, true))
            return mfail(f, HSC_ENOMEM, "multi staging");
        uint32_t *hd = (uint32_t *)ml.h_cnt.dp;
        const RouteCountOut o{ml.ctl.as<uint32_t>(), ml.totals.as<uint32_t>(), gather ? nullptr : hd, ++ml.seq,
                              src[m].p.n_lock, src[m].n_txn};
        MCHK(f, launch_route_count(src[m].p, split_view(M, m, W), N, ml.hist.as<uint32_t>(), o, s));
        if (gather) {
            uint32_t *mat = ml.totals.as<uint32_t>() + C;
            NCHK(f, R.AllGather(ml.totals.p, mat, C, ncclUint32, M->comm[L], s));
            MCHK(f, launch_route_publish(mat, (uint32_t)hw, hd, ml.seq, s));
        }
        MCHK(f, hipEventRecord(ml.ev_count, s));
    }
    const auto t2 = SteadyClock::now();
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        volatile const uint32_t *h = ml.h_cnt.as<uint32_t>();
        for (uint32_t spin = 1; h[hw] != ml.seq; ++spin) {
            __builtin_ia32_pause();
            if ((spin & 4095) == 0) {  // a fault never publishes: ask the stream
                const hipError_t e = hipEventQuery(ml.ev_count);
                if (e == hipSuccess && h[hw] != ml.seq) return mfail(f, HSC_EDEVICE, "route counts not published");
                if (e != hipSuccess && e != hipErrorNotReady) return mfail(f, HSC_EDEVICE, "route count", e);
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (gather)
            for (size_t i = 0; i < (size_t)C * N; ++i) M->cnt[i] = h[i];
        else
            for (int i = 0; i < C; ++i) M->cnt[(size_t)(M->rank + m) * C + i] = h[i];
    }
    const auto t3 = SteadyClock::now();
    auto cnt = [&](int s, int d) -> size_t { return M->cnt[(size_t)s * C + d]; };
    auto nlk = [&](int s) -> size_t { return M->cnt[(size_t)s * C + N]; };
    auto ntx = [&](int s) -> size_t { return M->cnt[(size_t)s * C + N + 1]; };
    // 2. sizes, offsets, read-set numbering, owners
    std::vector<size_t> nd(N, 0), tbase(N + 1, 0), lbase(N + 1, 0);
    std::vector<size_t> off((size_t)N * N, 0);
    for (int d = 0; d < N; ++d)
        for (int s = 0; s < N; ++s) off[(size_t)s * N + d] = nd[d], nd[d] += cnt(s, d);
    for (int s = 0; s < N; ++s) {
        lbase[s + 1] = lbase[s] + nlk(s);
        tbase[s + 1] = shared ? 0 : tbase[s] + r64(ntx(s));
    }
    const size_t total = shared ? r64(ntx(0)) : tbase[N];  // batch-wide read sets (64-aligned)
    const size_t nlock = lbase[N];
    if (total > 0xFFFFFFFFull) return mfail(f, HSC_EINVAL, "multi batch too large");
    // owner o's verdict words: [ob[o], ob[o] + ow[o])
    auto ob = [&](int o) -> size_t { return shared ? 0 : tbase[o] / 64; };
    auto ow = [&](int o) -> size_t { return shared ? (o == 0 ? total / 64 : 0) : r64(ntx(o)) / 64; };
    // 3. destination buffers
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        const int d = M->rank + m;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        ml.recvL = stage_layout(W, nd[d], d == 0 ? nlock : 0);
        MCHK(f, ml.recv.ensure(std::max<size_t>(ml.recvL.total, 256)));
        MCHK(f, ml.verdict.ensure(std::max<size_t>(total, 64)));
        MCHK(f, ml.bitmap.ensure(std::max<size_t>(total / 8, 8)));
    }
    // 4. scatter
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        const int s = M->rank + m;
        hipStream_t st = ml.stream;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        RouteArgs a{};
        a.N = N;
        a.tbase = (uint32_t)tbase[s];
        uint32_t *hc = a.base;
        if (M->rccl) {
            // one send block per other rank; this rank's own probes go straight
            // into its probe columns, at the rows its unpack leaves for them
            size_t sb = 0;
            for (int d = 0; d < N; ++d)
                if (d != s) sb += route_block_bytes(W, cnt(s, d), d == 0 ? nlk(s) : 0);
            MCHK(f, ml.send.ensure(std::max<size_t>(sb, 256)));
            size_t o = 0;
            for (int d = 0; d < N; ++d) {
                if (d == s) {
                    a.t[d] = arena_target(ml.recv.as<uint8_t>(), ml.recvL, nd[d]);
                    hc[d] = (uint32_t)off[(size_t)s * N + d];
                    continue;
                }
                a.t[d] = block_target(ml.send.as<uint8_t>() + o, W, cnt(s, d), d == 0 ? nlk(s) : 0);
                o += route_block_bytes(W, cnt(s, d), d == 0 ? nlk(s) : 0);
                hc[d] = 0;
            }
            a.lock_base = 0;  // rank 0's own locks first in its lock columns, else a block's
        } else {
            for (int d = 0; d < N; ++d) {
                MLane &dl = M->lane[L][d];
                a.t[d] = arena_target(dl.recv.as<uint8_t>(), dl.recvL, nd[d]);
                hc[d] = (uint32_t)off[(size_t)s * N + d];
            }
            a.lock_base = (uint32_t)lbase[s];
        }
        MCHK(f, launch_route_scatter(src[m].p, split_view(M, m, W), a, ml.hist.as<uint32_t>(),
                                     ml.ctl.as<uint32_t>() + N + 1, st));
        MCHK(f, hipEventRecord(ml.ev_scatter, st));
    }
    // 5. exchange
    if (M->rccl) {
        MLane &ml = M->lane[L][0];
        const int me = M->rank;
        hipStream_t st = ml.stream;
        RouteUnpack u{};
        u.N = N;
        size_t rb = 0;
        for (int s = 0; s < N; ++s) {
            u.boff[s] = rb;
            u.n[s] = s == me ? 0 : (uint32_t)cnt(s, me);
            u.nl[s] = me == 0 && s != me ? (uint32_t)nlk(s) : 0;
            u.dst[s] = (uint32_t)off[(size_t)s * N + me];
            u.ldst[s] = (uint32_t)lbase[s];
            u.roff[s + 1] = u.roff[s] + u.n[s];
            u.loff[s + 1] = u.loff[s] + u.nl[s];
            rb += route_block_bytes(W, u.n[s], u.nl[s]);
        }
        if (N > 1) {
            MCHK(f, ml.raw.ensure(std::max<size_t>(rb, 256)));
            NCHK(f, R.GroupStart());
            size_t o = 0;
            for (int d = 0; d < N; ++d) {
                if (d == me) continue;
                const size_t b = route_block_bytes(W, cnt(me, d), d == 0 ? nlk(me) : 0);
                if (b) NCHK(f, R.Send(ml.send.as<uint8_t>() + o, b, ncclUint8, d, M->comm[L], st));
                o += b;
            }
            for (int s = 0; s < N; ++s) {
                const size_t b = route_block_bytes(W, u.n[s], u.nl[s]);
                if (b) NCHK(f, R.Recv(ml.raw.as<uint8_t>() + u.boff[s], b, ncclUint8, s, M->comm[L], st));
            }
            NCHK(f, R.GroupEnd());
            MCHK(f, launch_route_unpack(ml.raw.as<uint8_t>(), u,
                                        arena_target(ml.recv.as<uint8_t>(), ml.recvL, nd[me]), W, st));
        }
    } else {
        for (int d = 0; d < NL; ++d)
            for (int s = 0; s < NL; ++s)
                if (s != d) MCHK(f, hipStreamWaitEvent(M->lane[L][d].stream, M->lane[L][s].ev_scatter, 0));
    }
    // 6. every member probes what it received
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        const int d = M->rank + m;
        hsc_ctx *c = M->mem[m];
        hsc_probe_batch b{};
        uint8_t *base = ml.recv.as<uint8_t>();
        b.n = nd[d];
        b.lo = (const uint64_t *)(base + ml.recvL.lo);
        b.hi = (const uint64_t *)(base + ml.recvL.hi);
        b.gid = (const uint32_t *)(base + ml.recvL.gid);
        b.snap = (const uint64_t *)(base + ml.recvL.snap);
        b.txn = (const uint32_t *)(base + ml.recvL.txn);
        b.n_lock = d == 0 ? nlock : 0;
        b.lock_table = (const uint32_t *)(base + ml.recvL.lock_table);
        b.lock_snap = (const uint64_t *)(base + ml.recvL.lock_snap);
        b.lock_txn = (const uint32_t *)(base + ml.recvL.lock_txn);
        b.n_txn = total;
        b.verdict = ml.verdict.as<uint8_t>();
        b.bitmap = ml.bitmap.as<uint64_t>();
        std::lock_guard<std::mutex> g(c->mu);
        MCHK(f, hipSetDevice(c->device));
        if (c->dirty) return mfail(f, HSC_ESTATE, "multi context: a member's window is not built");
        if (c->app_last) MCHK(f, hipStreamWaitEvent(ml.stream, c->app_last, 0));  // its appends
        hipStream_t keep = c->stream;
        c->stream = ml.stream;
        const int rc = ctx_probe(c, &b);
        c->stream = keep;
        if (rc) return mfail(f, rc, ("member probe: " + c->err).c_str());
        MCHK(f, hipEventRecord(ml.ev_probe, ml.stream));
    }
    // 7. OR of the members' bitmaps per owner
    if (M->rccl) {
        MLane &ml = M->lane[L][0];
        const int me = M->rank;
        hipStream_t st = ml.stream;
        const size_t wme = ow(me);
        // the other ranks' verdicts on this rank's read sets, OR-ed with its own
        MCHK(f, ml.gather.ensure(8 * std::max<size_t>(wme * N, 1)));
        if (N > 1) {
            NCHK(f, R.GroupStart());
            for (int o = 0; o < N; ++o)
                if (o != me && ow(o))
                    NCHK(f, R.Send(ml.bitmap.as<uint64_t>() + ob(o), 8 * ow(o), ncclUint8, o, M->comm[L], st));
            if (wme)
                for (int d = 0; d < N; ++d)
                    if (d != me)
                        NCHK(f, R.Recv(ml.gather.as<uint64_t>() + (size_t)d * wme, 8 * wme, ncclUint8, d,
                                       M->comm[L], st));
            NCHK(f, R.GroupEnd());
        }
        if (src[0].out && wme) {
            RouteParts parts{};
            parts.n = N;
            for (int d = 0; d < N; ++d)
                parts.p[d] = d == me ? ml.bitmap.as<uint64_t>() + ob(me) : ml.gather.as<uint64_t>() + (size_t)d * wme;
            MCHK(f, launch_or_slices(parts, wme, src[0].out, st));
        }
        MCHK(f, hipEventRecord(ml.ev_done, st));
        ml.used = true;
    } else {
        for (int o = 0; o < NL; ++o) {
            MLane &ml = M->lane[L][o];
            MCHK(f, hipSetDevice(M->mem[o]->device));
            if (ow(o) && src[o].out) {
                RouteParts parts{};
                parts.n = NL;
                for (int d = 0; d < NL; ++d) {
                    if (d != o) MCHK(f, hipStreamWaitEvent(ml.stream, M->lane[L][d].ev_probe, 0));
                    parts.p[d] = M->lane[L][d].bitmap.as<uint64_t>() + ob(o);
                }
                MCHK(f, launch_or_slices(parts, ow(o), src[o].out, ml.stream));
            }
        }
        // a lane is done once every member's probe and every merge reading it ran
        for (int o = 0; o < NL; ++o) {
            MLane &ml = M->lane[L][o];
            MCHK(f, hipSetDevice(M->mem[o]->device));
            for (int d = 0; d < NL; ++d)
                if (d != o) MCHK(f, hipStreamWaitEvent(ml.stream, M->lane[L][d].ev_probe, 0));
            MCHK(f, hipEventRecord(ml.ev_done, ml.stream));
            ml.used = true;
        }
    }
    M->batches++;
    const auto t4 = SteadyClock::now();
    auto ns = [](SteadyClock::time_point a, SteadyClock::time_point b) {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    };
    M->ns_lane += ns(t0, t1);
    M->ns_count += ns(t1, t2);
    M->ns_count_wait += ns(t2, t3);
    M->ns_enqueue += ns(t3, t4);
    for (int d = 0; d < N; ++d) M->routed += nd[d];
    for (int m = 0; m < NL; ++m) M->probes += src[m].p.n;
    return HSC_OK;
}

// The front's marshalled batch (host staging st) through the members.
int multi_check_stage(hsc_ctx *f, Stage &st, int *rc_out)
{
    Multi *M = f->multi;
    const int W = f->W, NL = M->nlocal, L = 0;
    MSource src[kMultiMax] = {};
    const size_t n = st.n;
    for (int m = 0; m < NL; ++m) {
        MRC(lane_stream(f, M, L, m));
        MLane &ml = M->lane[L][m];
        if (ml.used) MCHK(f, hipEventSynchronize(ml.ev_done));
        const size_t a = n * m / NL, e = n * (m + 1) / NL, k = e - a;
        const size_t nl = m == 0 ? st.n_lock : 0;
        hipStream_t s = ml.stream;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        ml.srcL = stage_layout(W, k, nl);
        MCHK(f, ml.src.ensure(std::max<size_t>(ml.srcL.total, 256)));
        uint8_t *d = ml.src.as<uint8_t>();
        auto up = [&](size_t doff, size_t soff, size_t bytes) -> hipError_t {
            return bytes ? hipMemcpyAsync(d + doff, (uint8_t *)st.arena.p + soff, bytes, hipMemcpyHostToDevice, s)
                         : hipSuccess;
        };
        for (int j = 0; j < W; ++j) {
            MCHK(f, up(ml.srcL.lo + 8 * (size_t)j * k, st.L.lo + 8 * ((size_t)j * n + a), 8 * k));
            MCHK(f, up(ml.srcL.hi + 8 * (size_t)j * k, st.L.hi + 8 * ((size_t)j * n + a), 8 * k));
        }
        MCHK(f, up(ml.srcL.snap, st.L.snap + 8 * a, 8 * k));
        MCHK(f, up(ml.srcL.gid, st.L.gid + 4 * a, 4 * k));
        MCHK(f, up(ml.srcL.txn, st.L.txn + 4 * a, 4 * k));
        MCHK(f, up(ml.srcL.lock_snap, st.L.lock_snap, 8 * nl));
        MCHK(f, up(ml.srcL.lock_table, st.L.lock_table, 4 * nl));
        MCHK(f, up(ml.srcL.lock_txn, st.L.lock_txn, 4 * nl));
        ProbeView &p = src[m].p;
        p.lo = (const uint64_t *)(d + ml.srcL.lo);
        p.hi = (const uint64_t *)(d + ml.srcL.hi);
        p.gid = (const uint32_t *)(d + ml.srcL.gid);
        p.snap = (const uint64_t *)(d + ml.srcL.snap);
        p.txn = (const uint32_t *)(d + ml.srcL.txn);
        p.lock_table = (const uint32_t *)(d + ml.srcL.lock_table);
        p.lock_snap = (const uint64_t *)(d + ml.srcL.lock_snap);
        p.lock_txn = (const uint32_t *)(d + ml.srcL.lock_txn);
        p.n = (uint32_t)k;
        p.n_lock = (uint32_t)nl;
        src[m].n_txn = (uint32_t)st.n_txn;
        src[m].out = nullptr;
    }
    // the verdicts land on the owner: member 0 here (shared numbering), or
    // this rank's member for a per-rank context (its own read sets)
    MLane &o = M->lane[L][0];
    const size_t words = r64(st.n_txn) / 64;
    MCHK(f, hipSetDevice(M->mem[0]->device));
    MCHK(f, o.out.ensure(8 * std::max<size_t>(words, 1)));
    src[0].out = o.out.as<uint64_t>();
    MRC(run_pipeline(f, L, src, !M->rccl));
    if (o.h_io.ensure(8 * words + 64, true)) return mfail(f, HSC_ENOMEM, "multi staging");
    uint64_t *hb = o.h_io.as<uint64_t>();
    if (words) MCHK(f, hipMemcpyAsync(hb, o.out.p, 8 * words, hipMemcpyDeviceToHost, o.stream));
    MCHK(f, hipStreamSynchronize(o.stream));
    for (int m = 1; m < NL; ++m) MCHK(f, hipEventSynchronize(M->lane[L][m].ev_done));
    const uint8_t *fc = st.forced.as<uint8_t>();
    for (size_t t = 0; t < st.n_txn; ++t) rc_out[t] = (fc[t] || ((hb[t >> 6] >> (t & 63)) & 1)) ? 1 : 0;
    return HSC_OK;
}

void multi_destroy(hsc_ctx *f)
{
    Multi *M = f->multi;
    if (!M) return;
    for (int L = 0; L < kMultiLanes; ++L)
        for (int m = 0; m < M->nlocal; ++m) {
            MLane &ml = M->lane[L][m];
            if (!ml.stream) continue;
            (void)hipSetDevice(M->mem[m]->device);
            (void)hipStreamSynchronize(ml.stream);
            for (DBuf *b : {&ml.src, &ml.hist, &ml.totals, &ml.ctl, &ml.send, &ml.raw, &ml.recv,
                            &ml.verdict, &ml.bitmap, &ml.gather, &ml.out})
                b->release();
            ml.h_io.release();
            ml.h_cnt.release();
            for (hipEvent_t e : {ml.ev_count, ml.ev_scatter, ml.ev_probe, ml.ev_done})
                if (e) (void)hipEventDestroy(e);
            (void)hipStreamDestroy(ml.stream);
        }
    if (M->rccl && rccl().ok)
        for (auto &c : M->comm)
            if (c) (void)rccl().CommDestroy(c);
    for (int m = 0; m < M->nlocal; ++m) {
        if (!M->mem[m]) continue;
        (void)hipSetDevice(M->mem[m]->device);
        M->d_sp[m].release();
        hsc_ctx_destroy(M->mem[m]);
    }
    delete M;
    f->multi = nullptr;
}

static hsc_ctx *front_new(int device)
{
    hsc_ctx *f = new (std::nothrow) hsc_ctx();
    if (!f) return nullptr;
    f->device = device;
    f->host_only = true;  // no window of its own: dictionaries, decode, rules, marshal
    f->threads = ctx_default_threads();
    f->multi = new (std::nothrow) Multi();
    if (!f->multi) {
        delete f;
        return nullptr;
    }
    return f;
}

}  // namespace hsc

extern "C" {

int hsc_multi_create(const int *devices, int n, hsc_ctx **out)
{
    if (!out || !devices || n < 1 || n > kMultiMax) return HSC_EINVAL;
    *out = nullptr;
    const int nd = hsc_device_count();
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= nd) return HSC_EDEVICE;
    // members on different GPUs store into each other's memory (the exchange)
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            if (devices[i] == devices[j]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) != hipSuccess || !can) return HSC_EDEVICE;
            (void)hipSetDevice(devices[i]);
            const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return HSC_EDEVICE;
            (void)hipGetLastError();
        }
    hsc_ctx *f = front_new(devices[0]);
    if (!f) return HSC_ENOMEM;
    Multi *M = f->multi;
    M->world = M->nlocal = n;
    M->rank = 0;
    for (int i = 0; i < n; ++i) {
        const int rc = hsc_ctx_create(devices[i], &M->mem[i]);
        if (rc) {
            hsc_ctx_destroy(f);
            return rc;
        }
    }
    (void)hipSetDevice(devices[0]);
    *out = f;
    return HSC_OK;
}

int hsc_multi_unique_ids(void *out, size_t bytes)
{
    if (!out || bytes < (size_t)kMultiLanes * NCCL_UNIQUE_ID_BYTES) return HSC_EINVAL;
    Rccl &R = rccl();
    if (!R.ok) return HSC_EDEVICE;
    for (int L = 0; L < kMultiLanes; ++L) {
        ncclUniqueId id;
        if (R.GetUniqueId(&id) != ncclSuccess) return HSC_EDEVICE;
        memcpy((uint8_t *)out + (size_t)L * NCCL_UNIQUE_ID_BYTES, &id, NCCL_UNIQUE_ID_BYTES);
    }
    return HSC_OK;
}

int hsc_multi_create_rank(int device, int rank, int world, const void *ids, size_t bytes, hsc_ctx **out)
{
    if (!out || !ids || world < 1 || world > kMultiMax || rank < 0 || rank >= world ||
        bytes < (size_t)kMultiLanes * NCCL_UNIQUE_ID_BYTES)
        return HSC_EINVAL;
    *out = nullptr;
    Rccl &R = rccl();
    if (!R.ok) return HSC_EDEVICE;
    hsc_ctx *f = front_new(device);
    if (!f) return HSC_ENOMEM;
    Multi *M = f->multi;
    M->world = world;
    M->nlocal = 1;
    M->rank = rank;
    M->rccl = true;
    int rc = hsc_ctx_create(device, &M->mem[0]);
    if (rc) {
        hsc_ctx_destroy(f);
        return rc;
    }
    (void)hipSetDevice(device);
    for (int L = 0; L < kMultiLanes; ++L) {
        ncclUniqueId id;
        memcpy(&id, (const uint8_t *)ids + (size_t)L * NCCL_UNIQUE_ID_BYTES, NCCL_UNIQUE_ID_BYTES);
        if (R.CommInitRank(&M->comm[L], world, id, rank) != ncclSuccess) {
            hsc_ctx_destroy(f);
            return HSC_EDEVICE;
        }
    }
    *out = f;
    return HSC_OK;
}

int hsc_multi_world(hsc_ctx *f) { return f && f->multi ? f->multi->world : 0; }
int hsc_multi_rank(hsc_ctx *f) { return f && f->multi ? f->multi->rank : -1; }
int hsc_multi_local(hsc_ctx *f) { return f && f->multi ? f->multi->nlocal : 0; }

hsc_ctx *hsc_multi_member(hsc_ctx *f, int i)
{
    if (!f || !f->multi || i < 0 || i >= f->multi->nlocal) return nullptr;
    return f->multi->mem[i];
}

int hsc_multi_set_splitters(hsc_ctx *f, size_t S, const uint32_t *gid, const uint64_t *words, int W)
{
    if (!f || !f->multi) return HSC_EINVAL;
    Multi *M = f->multi;
    if (S != (size_t)M->world - 1 || W < 1 || W > kMaxWords || (S && (!gid || !words))) return HSC_EINVAL;
    std::lock_guard<std::mutex> g(f->mu);
    for (size_t k = 1; k < S; ++k) {  // ascending (equal: an empty piece)
        int c = gid[k - 1] < gid[k] ? -1 : gid[k - 1] > gid[k] ? 1 : 0;
        for (int j = 0; j < W && !c; ++j)
            if (words[(size_t)j * S + k - 1] != words[(size_t)j * S + k])
                c = words[(size_t)j * S + k - 1] < words[(size_t)j * S + k] ? -1 : 1;
        if (c > 0) return mfail(f, HSC_EINVAL, "splitters not ascending");
    }
    M->sp_given = true;
    M->sp_W = W;
    M->sp_gid.assign(gid, gid + S);
    M->sp_w.assign(words, words + (size_t)W * S);
    M->d_sp_W = 0;
    f->dirty = true;  // a host-staged window is re-partitioned at the next check
    return HSC_OK;
}

int hsc_multi_adopt(hsc_ctx *f)
{
    if (!f || !f->multi) return HSC_EINVAL;
    Multi *M = f->multi;
    std::lock_guard<std::mutex> g(f->mu);
    // table maxima: every member answers lock probes with the global ones
    std::vector<uint64_t> tm(f->h_table_max);
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        if (c->dirty) return mfail(f, HSC_ESTATE, "adopt: a member's window is not built");
        if (c->groups.size() != f->groups.size()) return mfail(f, HSC_EINVAL, "adopt: member groups differ");
        for (size_t t = 0; t < std::min(tm.size(), c->h_table_max.size()); ++t)
            tm[t] = std::max(tm[t], c->h_table_max[t]);
    }
    if (M->rccl && !tm.empty()) {
        hsc_ctx *c = M->mem[0];
        MCHK(f, hipSetDevice(c->device));
        MRC(lane_stream(f, M, 0, 0));
        MLane &ml = M->lane[0][0];
        MCHK(f, ml.gather.ensure(8 * tm.size()));
        MCHK(f, hipMemcpy(ml.gather.p, tm.data(), 8 * tm.size(), hipMemcpyHostToDevice));
        NCHK(f, rccl().AllReduce(ml.gather.p, ml.gather.p, tm.size(), ncclUint64, ncclMax, M->comm[0], ml.stream));
        MCHK(f, hipStreamSynchronize(ml.stream));
        MCHK(f, hipMemcpy(tm.data(), ml.gather.p, 8 * tm.size(), hipMemcpyDeviceToHost));
    }
    f->h_table_max = tm;
    for (uint64_t v : tm) f->max_commit = std::max(f->max_commit, v);
    for (int m = 0; m < M->nlocal; ++m) {
        const int rc = hsc_merge_table_max(M->mem[m], tm.data(), (int)std::min(tm.size(), M->mem[m]->table_names.size()));
        if (rc) return mfail(f, rc, "adopt: table maxima");
        f->end_lsn = std::max(f->end_lsn, M->mem[m]->end_lsn);
    }
    int W = 1;
    for (int m = 0; m < M->nlocal; ++m) W = std::max(W, M->mem[m]->W);
    f->W = W;
    size_t keys = 0;
    for (int m = 0; m < M->nlocal; ++m) keys += M->mem[m]->n;
    f->n = keys;
    M->adopted = true;
    M->d_sp_W = 0;
    f->host_staged = false;
    f->dirty = false;
    f->live = false;
    f->ng_built = f->groups.size();
    return HSC_OK;
}

int hsc_multi_probe_device(hsc_ctx *f, const hsc_probe_batch *b, int lane)
{
    if (!f || !f->multi || !b || lane < 0 || lane >= kMultiLanes) return HSC_EINVAL;
    Multi *M = f->multi;
    std::lock_guard<std::mutex> g(f->mu);
    if (f->dirty) return mfail(f, HSC_ESTATE, "window not built");
    MSource src[kMultiMax] = {};
    for (int m = 0; m < M->nlocal; ++m) {
        if (b[m].n > 0xFFFFFFFFull || b[m].n_lock > 0xFFFFFFFFull || b[m].n_txn > 0x7FFFFFFFull ||
            (b[m].n_txn && !b[m].bitmap))
            return mfail(f, HSC_EINVAL, "multi probe batch");
        ProbeView &p = src[m].p;
        p.lo = b[m].lo, p.hi = b[m].hi, p.gid = b[m].gid, p.snap = b[m].snap, p.txn = b[m].txn;
        p.lock_table = b[m].lock_table, p.lock_snap = b[m].lock_snap, p.lock_txn = b[m].lock_txn;
        p.n = (uint32_t)b[m].n;
        p.n_lock = (uint32_t)b[m].n_lock;
        src[m].n_txn = (uint32_t)b[m].n_txn;
        src[m].out = b[m].bitmap;
    }
    return run_pipeline(f, lane, src, false);
}

int hsc_multi_stats(hsc_ctx *f, uint64_t out[4])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    Multi *M = f->multi;
    out[0] = M->batches;
    out[1] = M->probes;
    out[2] = M->routed;
    out[3] = M->nlocal;
    return HSC_OK;
}

int hsc_multi_phase_stats(hsc_ctx *f, double out[5])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    Multi *M = f->multi;
    const double b = (double)std::max<uint64_t>(M->batches, 1) * 1e3;
    out[0] = (double)M->batches;
    out[1] = (double)M->ns_lane / b;
    out[2] = (double)M->ns_count / b;
    out[3] = (double)M->ns_count_wait / b;
    out[4] = (double)M->ns_enqueue / b;
    return HSC_OK;
}

// counts[s * world + d]: probes source s sent to destination d in the last
// routed batch (host copy)
int hsc_multi_last_counts(hsc_ctx *f, uint32_t *counts, int n)
{
    if (!f || !f->multi || !counts) return HSC_EINVAL;
    Multi *M = f->multi;
    const int N = M->world, C = N + 2;
    if (n < N * N) return HSC_EINVAL;
    for (int s = 0; s < N; ++s)
        for (int d = 0; d < N; ++d)
            counts[s * N + d] = M->cnt.empty() ? 0 : M->cnt[(size_t)s * C + d];
    return HSC_OK;
}

}  // extern "C"
