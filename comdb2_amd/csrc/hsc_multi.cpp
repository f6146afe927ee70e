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
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // timed: around this member's probe (hsc_multi_enable_timing)
    bool timed = false;
    bool used = false;    // the lane ran a batch (ev_done recorded when nlocal > 1)
};

struct Multi {
    int world = 1;   // members of the partition
    int nlocal = 1;  // members in this process
    int rank = 0;    // global member index of local member 0
    int ndev = 1;    // distinct GPUs of the local members
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
    // in-process members exchanging like ranks (hsc_multi_set_transport):
    // send blocks moved by peer copies, unpacked, owner slices gathered
    bool loop = false;
    // routing on the host (multi_check_stage, hsc_multi_marshal_routed)
    Stage mst[kMultiMax];        // each member's share of the last routed batch (hsc_multi_marshal_routed)
    // the drop-in entries' routed shares: one set per call in flight (the
    // front lock is dropped once a batch is routed; its set is the call's
    // until the members' verdicts are in)
    struct StageSet {
        Stage s[kMultiMax];
    };
    std::mutex set_mu;
    std::vector<std::unique_ptr<StageSet>> sets;
    std::vector<StageSet *> free_sets;
    std::vector<uint8_t> h_own;  // per probe: first | last member << 4
    std::vector<uint32_t> h_cw;  // per chunk and member: counts, then offsets
    std::vector<int> h_rc;       // one member's verdicts
    uint64_t h_calls = 0, h_routed = 0, h_probes = 0, ns_route = 0;
    // accumulated after the front lock is dropped
    std::atomic<uint64_t> ns_launch_a{0}, ns_wait{0}, members_run{0};
    std::atomic<uint64_t> part_epoch{0};  // bumped before the members' pieces change
    // sharded SCC (hsc_multi_graph_scc): per local member its cover, its cut
    // rows and (the SCC's member) every member's cut rows
    DBuf g_cover[kMultiMax], g_rows[kMultiMax], g_all[kMultiMax], g_sz[kMultiMax];
    double g_ms[4] = {};  // host ms of its last call: build + cover, cover merge, cuts + gather, SCC
    // window placement (hsc_multi_set_mode): pieces or replicas
    int mode = HSC_MULTI_AUTO;
    bool replicated = false;            // in force since the last build / adopt
    std::atomic<int> inflight[kMultiMax] = {};  // replicas: drop-in batches running per member
    std::atomic<uint32_t> rr{0};
    std::atomic<uint64_t> rep_calls{0}, rep_sliced{0};
    bool timing = false;  // events around every member's probe (per-member probe times)
    int last_lane = 0;
    // host copies of the last pipeline's counts
    std::vector<uint32_t> cnt;   // [world][world + 2]: per source s: to each d, n_lock, n_txn
    uint64_t batches = 0, routed = 0, probes = 0;
    // host phase split of run_pipeline (ns): waiting for the lane's previous
    // batch, launching the counts, waiting for them, enqueueing the rest
    uint64_t ns_lane = 0, ns_count = 0, ns_count_wait = 0, ns_enqueue = 0;
    uint64_t pr_batches = 0, ns_pr = 0;  // hsc_multi_probe_routed: batches, host time enqueueing them
    // its split: lane_acquire (the members' cross-lane event waits), the
    // members' probe launches, the owners' merges + done events
    uint64_t ns_pr_lane = 0, ns_pr_probe = 0, ns_pr_merge = 0;
    uint64_t ns_pm_probe = 0, ns_pm_merge = 0;  // probe_merge's last call: probes, merges
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
            // (a NULL-stream copy from pageable memory may return before it
            // lands; the route kernels run on non-blocking lane streams)
            MCHK(f, hipDeviceSynchronize());
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
        MuGuard g(c);
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
// Placement of a host-staged window of n rows of W key words: replicas when
// asked, or (AUTO) when n x (8 W + 16) bytes fit an eighth of the smallest
// local member's device memory (every rank of a per-rank context sees the
// same log and the same GPUs, so all choose alike).
static bool choose_replicas(hsc_ctx *f, Multi *M, size_t n, int W)
{
    if (M->mode != HSC_MULTI_AUTO) return M->mode == HSC_MULTI_REPLICAS;
    if (M->sp_given) return false;  // splitters were set: the caller cut pieces
    size_t lim = ~(size_t)0;
    for (int m = 0; m < M->nlocal; ++m) {
        size_t fr = 0, tot = 0;
        if (hipSetDevice(M->mem[m]->device) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
        lim = std::min(lim, tot / 8);
    }
    (void)hipSetDevice(f->device);
    return (double)n * (8.0 * W + 16.0) <= (double)lim;
}


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
    M->part_epoch.fetch_add(1, std::memory_order_acq_rel);
    const int W = ctx_window_words(f);
    if (f->W != W) f->dict_epoch++;
    f->W = W;
    const size_t n = f->h_gid.size();
    M->replicated = choose_replicas(f, M, n, W);
    std::vector<int> own(M->replicated ? 0 : n);
    if (!M->replicated) {
        if (!M->sp_given) auto_splitters(f, M, W);
        MRC(upload_splitters(f, M, W));  // before the rows are placed: one routing rule
        std::vector<uint64_t> x((size_t)W);
        for (size_t i = 0; i < n; ++i) {
            row_key(f, i, W, x.data());
            own[i] = sp_owner(M, f->h_gid[i], x.data(), W);
        }
    }
    multi_sync_dict(f);
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        const int me = M->rank + m;
        MuGuard g(c);
        (void)hipSetDevice(c->device);
        ctx_clear_window(c);
        c->end_lsn = f->end_lsn;
        c->h_table_max = f->h_table_max;
        c->max_commit = f->max_commit;
        for (size_t i = 0; i < n; ++i) {
            if (!M->replicated && own[i] != me) continue;  // (replicas: every row)
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
    f->n = M->replicated ? M->mem[0]->n : keys;
    f->dirty = false;
    f->live = true;
    f->merge_pending = false;
    f->ng_built = f->groups.size();
    f->app_gid.clear(), f->app_keys.clear(), f->app_koff.clear(), f->app_lsn.clear();
    f->app_tmax = false;
    return HSC_OK;
}

// Rows appended to a built window go to their owners' delta runs.
int multi_flush_appends(hsc_ctx *f, bool lazy)
{
    Multi *M = f->multi;
    if (M->adopted) return mfail(f, HSC_ESTATE, "multi context: append to the members' windows directly");
    if (!f->live) return HSC_OK;
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
        if (M->replicated) {  // every member holds every row
            for (int m = 0; m < M->nlocal; ++m) rows[m].push_back(i);
            continue;
        }
        const int o = sp_owner(M, f->app_gid[i], x.data(), W) - M->rank;
        if (o >= 0 && o < M->nlocal) rows[o].push_back(i);
    }
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        MuGuard g(c);
        (void)hipSetDevice(c->device);
        for (size_t t = 0; t < f->h_table_max.size(); ++t)  // (mirrored by a pending tail)
            ctx_raise_table_max(c, (int)t, f->h_table_max[t]);
        c->max_commit = std::max(c->max_commit, f->max_commit);
        c->end_lsn = f->end_lsn;
        for (size_t i : rows[m]) {
            const GroupInfo &gi = f->groups[f->app_gid[i]];
            ctx_add_write(c, gi.tid, gi.ix, f->app_keys.data() + f->app_koff[i], gi.klen, true, f->app_lsn[i]);
        }
        const int rc = ctx_flush_appends(c, lazy);  // lazy: a small batch's pending tail
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

// Lane L's next batch runs after its previous one on every local member:
// each member's lane stream waits (on the device, no host wait) for every
// member's done event of the lane -- a member's buffers of the lane are
// written by the others' scatters / copies and read by their merges.
static int lane_acquire(hsc_ctx *f, Multi *M, int L)
{
    for (int m = 0; m < M->nlocal; ++m) MRC(lane_stream(f, M, L, m));
    for (int m = 0; m < M->nlocal; ++m) {
        MLane &ml = M->lane[L][m];
        MCHK(f, hipSetDevice(M->mem[m]->device));
        for (int d = 0; d < M->nlocal; ++d)  // (its own stream is in order)
            if (d != m && M->lane[L][d].used) MCHK(f, hipStreamWaitEvent(ml.stream, M->lane[L][d].ev_done, 0));
    }
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

static hsc_probe_batch arena_batch(uint8_t *base, const StageLayout &L, size_t n, size_t nl)
{
    hsc_probe_batch b{};
    b.n = n;
    b.lo = (const uint64_t *)(base + L.lo);
    b.hi = (const uint64_t *)(base + L.hi);
    b.gid = (const uint32_t *)(base + L.gid);
    b.snap = (const uint64_t *)(base + L.snap);
    b.txn = (const uint32_t *)(base + L.txn);
    b.n_lock = nl;
    b.lock_table = (const uint32_t *)(base + L.lock_table);
    b.lock_snap = (const uint64_t *)(base + L.lock_snap);
    b.lock_txn = (const uint32_t *)(base + L.lock_txn);
    return b;
}

static hsc_probe_batch view_batch(const ProbeView &p)
{
    hsc_probe_batch b{};
    b.n = p.n;
    b.lo = p.lo, b.hi = p.hi, b.gid = p.gid, b.snap = p.snap, b.txn = p.txn;
    b.n_lock = p.n_lock;
    b.lock_table = p.lock_table, b.lock_snap = p.lock_snap, b.lock_txn = p.lock_txn;
    return b;
}

// Steps 6-7 of every pipeline: local member m probes in[m] (read sets
// numbered batch-wide, tb[N] of them; owner o owns [tb[o], tb[o+1]), every
// bound a multiple of 64), then each owner's slice of the members' verdict
// bitmaps is OR-ed into out[m] of the owner's local member.  The members'
// streams already hold whatever produced in[m] (routing, exchange).
static int probe_merge(hsc_ctx *f, int L, hsc_probe_batch *in, const size_t *tb, uint64_t *const *out)
{
    Multi *M = f->multi;
    const int N = M->world, NL = M->nlocal;
    const size_t total = tb[N];
    auto ob = [&](int o) -> size_t { return tb[o] / 64; };
    auto ow = [&](int o) -> size_t { return (tb[o + 1] - tb[o]) / 64; };
    const bool direct = !M->rccl && !M->loop;
    // 6. every member probes what it holds -- the members' launches issued
    // from one host thread each (a probe is several launches; eight GPUs'
    // worth from one thread would outlast the probes themselves)
    auto probe_one = [&](int m) -> int {
        MLane &ml = M->lane[L][m];
        hsc_ctx *c = M->mem[m];
        hsc_probe_batch b = in[m];
        b.n_txn = total;
        MCHK(c, hipSetDevice(c->device));
        MCHK(c, ml.verdict.ensure(std::max<size_t>(total, 64)));
        b.verdict = ml.verdict.as<uint8_t>();
        if (N == 1) {  // one piece: its bitmap is the result
            b.bitmap = out[0];
        } else if (direct) {  // in process: the owners OR the verdict bytes themselves
            b.bitmap = nullptr;
        } else {
            MCHK(c, ml.bitmap.ensure(std::max<size_t>(total / 8, 8)));
            b.bitmap = ml.bitmap.as<uint64_t>();
        }
        MuGuard g(c);
        if (c->dirty) return ctx_fail(c, HSC_ESTATE, "window not built");
        if (c->app_last) MCHK(c, hipStreamWaitEvent(ml.stream, c->app_last, 0));  // its appends
        ml.timed = M->timing;
        if (ml.timed) {
            if (!ml.ev_t0) MCHK(c, hipEventCreate(&ml.ev_t0));
            if (!ml.ev_t1) MCHK(c, hipEventCreate(&ml.ev_t1));
            MCHK(c, hipEventRecord(ml.ev_t0, ml.stream));
        }
        hipStream_t keep = c->stream;
        MCHK(c, ctx_switch_stream(c, ml.stream));
        const int rc = ctx_probe(c, &b);
        MCHK(c, ctx_switch_stream(c, keep));  // (fences the member's lane of ml.stream)
        if (rc) return rc;
        if (ml.timed) MCHK(c, hipEventRecord(ml.ev_t1, ml.stream));
        // (not the context's own lane event: a concurrent caller of the member
        // may take that lane and record it again before the merges wait);
        // only other local members' streams wait on it
        if (NL > 1) MCHK(c, hipEventRecord(ml.ev_probe, ml.stream));
        return HSC_OK;
    };
    int prc[kMultiMax] = {};
    const auto tp0 = SteadyClock::now();
    // (members sharing a GPU: one thread -- its launches serialise anyway;
    // HSC_MULTI_PAR_LAUNCH=1 issues them from the pool there too, an A/B)
    static const bool par_env = getenv("HSC_MULTI_PAR_LAUNCH") != nullptr;
    if (M->ndev > 1 || (par_env && NL > 1))
        ctx_par_for(f, NL, [&](int m) { prc[m] = probe_one(m); });
    else
        for (int m = 0; m < NL; ++m) prc[m] = probe_one(m);
    for (int m = 0; m < NL; ++m)
        if (prc[m]) return mfail(f, prc[m], ("member probe: " + M->mem[m]->err).c_str());
    const auto tp1 = SteadyClock::now();
    M->last_lane = L;
    // 7. OR of the members' bitmaps per owner
    if (N == 1) {
    } else if (M->rccl) {
        Rccl &R = rccl();
        MLane &ml = M->lane[L][0];
        const int me = M->rank;
        hipStream_t st = ml.stream;
        const size_t wme = ow(me);
        // the other ranks' verdicts on this rank's read sets, OR-ed with its own
        MCHK(f, ml.gather.ensure(8 * std::max<size_t>(wme * N, 1)));
        NCHK(f, R.GroupStart());
        for (int o = 0; o < N; ++o)
            if (o != me && ow(o))
                NCHK(f, R.Send(ml.bitmap.as<uint64_t>() + ob(o), 8 * ow(o), ncclUint8, o, M->comm[L], st));
        if (wme)
            for (int d = 0; d < N; ++d)
                if (d != me)
                    NCHK(f, R.Recv(ml.gather.as<uint64_t>() + (size_t)d * wme, 8 * wme, ncclUint8, d, M->comm[L],
                                   st));
        NCHK(f, R.GroupEnd());
        if (out[0] && wme) {
            RouteParts parts{};
            parts.n = N;
            for (int d = 0; d < N; ++d)
                parts.p[d] = d == me ? ml.bitmap.as<uint64_t>() + ob(me) : ml.gather.as<uint64_t>() + (size_t)d * wme;
            MCHK(f, launch_or_slices(parts, wme, out[0], st));
        }
    } else if (M->loop) {
        // the per-rank merge with peer copies in place of RCCL send / receive:
        // owner o gathers every other member's slice of its read sets into its
        // gather buffer, then ORs them with its own slice
        for (int o = 0; o < NL; ++o) {
            MLane &ol = M->lane[L][o];
            const size_t wo = ow(o);
            MCHK(f, hipSetDevice(M->mem[o]->device));
            MCHK(f, ol.gather.ensure(8 * std::max<size_t>(wo * N, 1)));
            if (!wo) continue;
            RouteParts parts{};
            parts.n = N;
            for (int d = 0; d < NL; ++d) {
                if (d == o) {
                    parts.p[d] = ol.bitmap.as<uint64_t>() + ob(o);
                    continue;
                }
                MLane &dl = M->lane[L][d];
                uint64_t *dst = ol.gather.as<uint64_t>() + (size_t)d * wo;
                MCHK(f, hipStreamWaitEvent(ol.stream, dl.ev_probe, 0));
                MCHK(f, hipMemcpyPeerAsync(dst, M->mem[o]->device, dl.bitmap.as<uint64_t>() + ob(o),
                                           M->mem[d]->device, 8 * wo, ol.stream));
                parts.p[d] = dst;
            }
            if (out[o]) MCHK(f, launch_or_slices(parts, wo, out[o], ol.stream));
        }
    } else {
        for (int o = 0; o < NL; ++o) {
            MLane &ml = M->lane[L][o];
            MCHK(f, hipSetDevice(M->mem[o]->device));
            if (ow(o) && out[o]) {
                RouteBytes parts{};
                parts.n = NL;
                for (int d = 0; d < NL; ++d) {
                    if (d != o) MCHK(f, hipStreamWaitEvent(ml.stream, M->lane[L][d].ev_probe, 0));
                    parts.p[d] = M->lane[L][d].verdict.as<uint8_t>() + tb[o];
                }
                MCHK(f, launch_or_bytes(parts, ow(o), out[o], ml.stream));
            }
        }
    }
    // a lane is done once every member's probe and every merge reading it ran
    // (an owner whose merge read every member has waited for them already)
    for (int o = 0; o < NL; ++o) {
        MLane &ml = M->lane[L][o];
        MCHK(f, hipSetDevice(M->mem[o]->device));
        const bool merged = (M->loop || (!M->rccl && !M->loop && out[o])) && ow(o);
        if (!M->rccl && !merged)
            for (int d = 0; d < NL; ++d)
                if (d != o) MCHK(f, hipStreamWaitEvent(ml.stream, M->lane[L][d].ev_probe, 0));
        // (only the other local members' next use of the lane waits on it: one
        // member orders its lane by its stream alone -- the world-1 step 51 ->
        // 48 us without the probe event, r05x)
        if (NL > 1) MCHK(f, hipEventRecord(ml.ev_done, ml.stream));
        ml.used = true;
    }
    M->batches++;
    const auto tp2 = SteadyClock::now();
    M->ns_pm_probe = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tp1 - tp0).count();
    M->ns_pm_merge = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tp2 - tp1).count();
    return HSC_OK;
}

// The device-routed pipeline (batches resident on the GPUs, not routed when
// they were marshalled).  shared: the local sources number the same read
// sets (one batch split by probe; member 0 owns every verdict); else each
// source numbers its own read sets and owns their verdicts (per-rank batches,
// hsc_multi_probe_device).
static int run_pipeline(hsc_ctx *f, int L, MSource *src, bool shared)
{
    Multi *M = f->multi;
    const int N = M->world, NL = M->nlocal, W = f->W;
    const int C = N + 2;
    const auto t0 = SteadyClock::now();
    if (M->d_sp_W != W) MRC(upload_splitters(f, M, W));
    MRC(lane_acquire(f, M, L));
    const auto t1 = SteadyClock::now();
    uint64_t *outs[kMultiMax] = {};
    for (int m = 0; m < NL; ++m) outs[m] = src[m].out;
    if (N == 1) {  // one piece: no routing, the batch is probed where it is
        hsc_probe_batch b = view_batch(src[0].p);
        const size_t tb[2] = {0, r64(src[0].n_txn)};
        MRC(probe_merge(f, L, &b, tb, outs));
        M->ns_lane += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        M->routed += src[0].p.n, M->probes += src[0].p.n;
        return HSC_OK;
    }
    Rccl &R = rccl();
    const bool blocks = M->rccl || M->loop;  // send blocks + unpack (per-rank form)
    // 1. counts per destination: the count kernel's last block (or, across
    // ranks, a one-block copy after the all-gather) stores them to pinned host
    // memory with a sequence word the host spins on -- no copy, no event wait
    M->cnt.assign((size_t)N * C, 0);
    const bool gather = M->rccl;
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
    std::vector<size_t> nd(N, 0), tbase(N + 1, 0), lbase(N + 1, 0), tb(N + 1, 0);
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
    for (int o = 0; o <= N; ++o) tb[o] = shared ? (o == 0 ? 0 : total) : tbase[o];
    // 3. destination buffers
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        const int d = M->rank + m;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        ml.recvL = stage_layout(W, nd[d], d == 0 ? nlock : 0);
        MCHK(f, ml.recv.ensure(std::max<size_t>(ml.recvL.total, 256)));
    }
    // send blocks (per-rank form): one per other destination, in destination
    // order; u[m]: the unpack of what local member m receives
    std::vector<std::vector<size_t>> soff(NL, std::vector<size_t>(N + 1, 0));
    std::vector<RouteUnpack> u(NL);
    std::vector<size_t> rbytes(NL, 0);
    if (blocks)
        for (int m = 0; m < NL; ++m) {
            const int me = M->rank + m;
            for (int d = 0; d < N; ++d)
                soff[m][d + 1] = soff[m][d] + (d == me ? 0 : route_block_bytes(W, cnt(me, d), d == 0 ? nlk(me) : 0));
            RouteUnpack &x = u[m];
            x = RouteUnpack{};
            x.N = N;
            size_t rb = 0;
            for (int s = 0; s < N; ++s) {
                x.boff[s] = rb;
                x.n[s] = s == me ? 0 : (uint32_t)cnt(s, me);
                x.nl[s] = me == 0 && s != me ? (uint32_t)nlk(s) : 0;
                x.dst[s] = (uint32_t)off[(size_t)s * N + me];
                x.ldst[s] = (uint32_t)lbase[s];
                x.roff[s + 1] = x.roff[s] + x.n[s];
                x.loff[s + 1] = x.loff[s] + x.nl[s];
                rb += route_block_bytes(W, x.n[s], x.nl[s]);
            }
            rbytes[m] = rb;
            MLane &ml = M->lane[L][m];
            MCHK(f, hipSetDevice(M->mem[m]->device));
            MCHK(f, ml.send.ensure(std::max<size_t>(soff[m][N], 256)));
            MCHK(f, ml.raw.ensure(std::max<size_t>(rb, 256)));
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
        if (blocks) {
            // one send block per other destination; this member's own probes go
            // straight into its probe columns, at the rows its unpack leaves
            for (int d = 0; d < N; ++d) {
                if (d == s) {
                    a.t[d] = arena_target(ml.recv.as<uint8_t>(), ml.recvL, nd[d]);
                    hc[d] = (uint32_t)off[(size_t)s * N + d];
                    continue;
                }
                a.t[d] = block_target(ml.send.as<uint8_t>() + soff[m][d], W, cnt(s, d), d == 0 ? nlk(s) : 0);
                hc[d] = 0;
            }
            a.lock_base = 0;  // member 0's own locks first in its lock columns, else a block's
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
        NCHK(f, R.GroupStart());
        for (int d = 0; d < N; ++d) {
            const size_t b = soff[0][d + 1] - soff[0][d];
            if (b) NCHK(f, R.Send(ml.send.as<uint8_t>() + soff[0][d], b, ncclUint8, d, M->comm[L], st));
        }
        for (int s = 0; s < N; ++s) {
            const size_t b = route_block_bytes(W, u[0].n[s], u[0].nl[s]);
            if (b) NCHK(f, R.Recv(ml.raw.as<uint8_t>() + u[0].boff[s], b, ncclUint8, s, M->comm[L], st));
        }
        NCHK(f, R.GroupEnd());
        MCHK(f, launch_route_unpack(ml.raw.as<uint8_t>(), u[0], arena_target(ml.recv.as<uint8_t>(), ml.recvL, nd[me]),
                                    W, st));
    } else if (M->loop) {
        // the same blocks moved by peer copies: member d's stream waits for
        // every source's scatter and copies its block in, then unpacks
        for (int d = 0; d < NL; ++d) {
            MLane &dl = M->lane[L][d];
            MCHK(f, hipSetDevice(M->mem[d]->device));
            for (int s = 0; s < NL; ++s) {
                if (s == d) continue;
                const size_t b = soff[s][d + 1] - soff[s][d];
                if (!b) continue;
                MCHK(f, hipStreamWaitEvent(dl.stream, M->lane[L][s].ev_scatter, 0));
                MCHK(f, hipMemcpyPeerAsync(dl.raw.as<uint8_t>() + u[d].boff[s], M->mem[d]->device,
                                           M->lane[L][s].send.as<uint8_t>() + soff[s][d], M->mem[s]->device, b,
                                           dl.stream));
            }
            MCHK(f, launch_route_unpack(dl.raw.as<uint8_t>(), u[d],
                                        arena_target(dl.recv.as<uint8_t>(), dl.recvL, nd[d]), W, dl.stream));
        }
    } else {
        for (int d = 0; d < NL; ++d)
            for (int s = 0; s < NL; ++s)
                if (s != d) MCHK(f, hipStreamWaitEvent(M->lane[L][d].stream, M->lane[L][s].ev_scatter, 0));
    }
    // 6-7. every member probes what it received; OR per owner
    hsc_probe_batch in[kMultiMax];
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        const int d = M->rank + m;
        in[m] = arena_batch(ml.recv.as<uint8_t>(), ml.recvL, nd[d], d == 0 ? nlock : 0);
    }
    MRC(probe_merge(f, L, in, tb.data(), outs));
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

// ---- routing on the host, at marshal time ---------------------------------------
// The front's marshalled batch st goes to the members by the same rule as the
// device routing -- member d gets every probe whose [g || lo, g || hi]
// overlaps its piece, i.e. owner(g || lo) <= d <= owner(g || hi); the table
// locks go to member 0, whose table maxima are the global ones -- while the
// host still has the columns it just wrote.  out[d] receives
// member d's columns (txn + txn_base), sized with the small path's slot tail
// when small(d, n_d, nl_d) says so; member 0 only, or every member.
constexpr size_t kRouteHostChunk = 16384;

static int route_host(hsc_ctx *f, const Stage &st, Stage *out, int only, uint32_t txn_base,
                      const std::function<bool(int, size_t, size_t)> &small)
{
    Multi *M = f->multi;
    const int N = M->world, W = f->W;
    if (M->d_sp_W != W) MRC(upload_splitters(f, M, W));
    const size_t n = st.n, nl = st.n_lock;
    const int S = (int)M->sp_gid.size();
    const uint64_t *lo = st.col<uint64_t>(st.L.lo), *hi = st.col<uint64_t>(st.L.hi);
    const uint64_t *sn = st.col<uint64_t>(st.L.snap);
    const uint32_t *gid = st.col<uint32_t>(st.L.gid), *txn = st.col<uint32_t>(st.L.txn);
    const int nw = (int)((n + kRouteHostChunk - 1) / kRouteHostChunk);
    std::vector<uint8_t> &own = M->h_own;  // ra | rb << 4 per probe (world <= 16)
    own.resize(std::max<size_t>(n, 1));
    std::vector<uint32_t> &cw = M->h_cw;   // [chunk][N] counts, then offsets
    cw.assign((size_t)std::max(nw, 1) * N, 0);
    auto owner = [&](uint32_t g, const uint64_t *x, size_t i) {
        int a = 0, b = S;
        while (a < b) {
            const int mid = (a + b) >> 1;
            int c = g == M->sp_gid[mid] ? 0 : (g < M->sp_gid[mid] ? -1 : 1);
            for (int j = 0; j < W && !c; ++j) {
                const uint64_t v = x[(size_t)j * n + i], s = M->eff_w[(size_t)j * S + mid];
                if (v != s) c = v < s ? -1 : 1;
            }
            if (c >= 0)
                a = mid + 1;
            else
                b = mid;
        }
        return a;
    };
    auto pass1 = [&](int w) {
        const size_t a = (size_t)w * kRouteHostChunk, e = std::min(n, a + kRouteHostChunk);
        uint32_t *k = &cw[(size_t)w * N];
        for (size_t i = a; i < e; ++i) {
            const int ra = S ? owner(gid[i], lo, i) : 0, rb = S ? owner(gid[i], hi, i) : 0;
            own[i] = (uint8_t)(ra | rb << 4);
            for (int d = ra; d <= rb; ++d) k[d]++;
        }
    };
    if (nw > 1 && n >= 65536)
        ctx_par_for(f, nw, pass1);
    else
        for (int w = 0; w < nw; ++w) pass1(w);
    std::vector<size_t> nd(N, 0);
    for (int w = 0; w < nw; ++w)
        for (int d = 0; d < N; ++d) {
            const uint32_t k = cw[(size_t)w * N + d];
            cw[(size_t)w * N + d] = (uint32_t)nd[d];
            nd[d] += k;
        }
    for (int d = 0; d < N; ++d) {
        if (only >= 0 && d != only) continue;
        Stage &o = out[d];
        const size_t ol = d == 0 ? nl : 0;
        o.L = stage_layout(W, nd[d], ol);
        o.n = nd[d], o.n_lock = ol, o.n_txn = st.n_txn;
        o.coh = small && small(d, nd[d], ol);
        if (o.arena.ensure(std::max<size_t>(o.L.total + (o.coh ? small_tail(st.n_txn) : 0), 256), true, o.coh) ||
            o.forced.ensure(std::max<size_t>(st.n_txn, 1), true))
            return mfail(f, HSC_ENOMEM, "multi routing staging");
        memset(o.forced.p, 0, std::max<size_t>(st.n_txn, 1));  // the front's forced verdicts are OR-ed in
        if (ol) {
            memcpy(o.col<uint32_t>(o.L.lock_table), st.col<uint32_t>(st.L.lock_table), 4 * ol);
            memcpy(o.col<uint64_t>(o.L.lock_snap), st.col<uint64_t>(st.L.lock_snap), 8 * ol);
            uint32_t *lt = o.col<uint32_t>(o.L.lock_txn);
            const uint32_t *sl = st.col<uint32_t>(st.L.lock_txn);
            for (size_t i = 0; i < ol; ++i) lt[i] = sl[i] + txn_base;
        }
    }
    auto pass2 = [&](int w) {
        const size_t a = (size_t)w * kRouteHostChunk, e = std::min(n, a + kRouteHostChunk);
        uint32_t k[kMultiMax];
        for (int d = 0; d < N; ++d) k[d] = cw[(size_t)w * N + d];
        for (size_t i = a; i < e; ++i) {
            const int ra = own[i] & 15, rb = own[i] >> 4;
            for (int d = ra; d <= rb; ++d) {
                const size_t r = k[d]++;
                if (only >= 0 && d != only) continue;
                Stage &o = out[d];
                const size_t m = o.n;
                uint64_t *olo = o.col<uint64_t>(o.L.lo), *ohi = o.col<uint64_t>(o.L.hi);
                for (int j = 0; j < W; ++j) {
                    olo[(size_t)j * m + r] = lo[(size_t)j * n + i];
                    ohi[(size_t)j * m + r] = hi[(size_t)j * n + i];
                }
                o.col<uint64_t>(o.L.snap)[r] = sn[i];
                o.col<uint32_t>(o.L.gid)[r] = gid[i];
                o.col<uint32_t>(o.L.txn)[r] = txn[i] + txn_base;
            }
        }
    };
    if (nw > 1 && n >= 65536)
        ctx_par_for(f, nw, pass2);
    else
        for (int w = 0; w < nw; ++w) pass2(w);
    for (int d = 0; d < N; ++d) M->h_routed += nd[d];
    M->h_probes += n;
    return HSC_OK;
}

// The front's marshalled batch through the members (the drop-in entries on
// a multi context).  In one process the batch is routed on the host and
// every member that holds any of its probes checks its share through its own
// one-GPU path -- a read set touching one member launches that member's
// small kernel only -- and the verdicts are OR-ed on the host.  A per-rank
// context has only its own member here: its batch goes through the device
// routing and the RCCL exchange.
static int check_stage_device(hsc_ctx *f, Stage &st, int *rc_out);

// ---- replicas: whole batches (or read-set slices) to single members ------------
// The member with the fewest drop-in batches in flight, round robin among
// equals (a lone caller alternates members; concurrent callers spread).
static int pick_member(Multi *M)
{
    const int NL = M->nlocal;
    const int start = (int)(M->rr.fetch_add(1, std::memory_order_relaxed) % (uint32_t)NL);
    int best = start, bv = M->inflight[start].load(std::memory_order_relaxed);
    for (int k = 1; k < NL && bv > 0; ++k) {
        const int m = (start + k) % NL;
        const int x = M->inflight[m].load(std::memory_order_relaxed);
        if (x < bv) best = m, bv = x;
    }
    return best;
}

// Read sets [t0, t1) of the marshalled batch st into o for member c: the
// probes (and lock probes) whose read set falls in the slice, in the batch's
// order -- which is NOT read-set order in general (the marshal lays a key
// length's points after its ranges, config 3), so the slice is a filter, not
// a subrange -- read sets renumbered from 0, sized for c's small path when it
// fits.  A whole batch (t0 = 0, t1 = T) copies the columns as they are.
static int replica_slice(hsc_ctx *f, hsc_ctx *c, const Stage &st, size_t t0, size_t t1, Stage &o)
{
    const int W = f->W;
    const size_t n = st.n, nl = st.n_lock, T = t1 - t0;
    const uint32_t *txn = st.col<uint32_t>(st.L.txn), *ltx = st.col<uint32_t>(st.L.lock_txn);
    const bool whole = t0 == 0 && t1 >= st.n_txn;
    static thread_local std::vector<uint32_t> pi, li;
    pi.clear(), li.clear();
    if (!whole) {
        for (size_t i = 0; i < n; ++i)
            if (txn[i] >= t0 && txn[i] < t1) pi.push_back((uint32_t)i);
        for (size_t i = 0; i < nl; ++i)
            if (ltx[i] >= t0 && ltx[i] < t1) li.push_back((uint32_t)i);
    }
    const size_t k = whole ? n : pi.size(), kl = whole ? nl : li.size();
    o.L = stage_layout(W, k, kl);
    o.n = k, o.n_lock = kl, o.n_txn = T;
    o.coh = ctx_small_fits(c, T, k, kl);
    if (o.arena.ensure(std::max<size_t>(o.L.total + (o.coh ? small_tail(T) : 0), 256), true, o.coh) ||
        o.forced.ensure(std::max<size_t>(T, 1), true))
        return mfail(f, HSC_ENOMEM, "multi replica staging");
    memset(o.forced.p, 0, std::max<size_t>(T, 1));  // the front's forced verdicts are OR-ed in
    if (whole) {
        for (int j = 0; j < W; ++j) {
            memcpy(o.col<uint64_t>(o.L.lo) + (size_t)j * k, st.col<uint64_t>(st.L.lo) + (size_t)j * n, 8 * k);
            memcpy(o.col<uint64_t>(o.L.hi) + (size_t)j * k, st.col<uint64_t>(st.L.hi) + (size_t)j * n, 8 * k);
        }
        memcpy(o.col<uint64_t>(o.L.snap), st.col<uint64_t>(st.L.snap), 8 * k);
        memcpy(o.col<uint32_t>(o.L.gid), st.col<uint32_t>(st.L.gid), 4 * k);
        memcpy(o.col<uint32_t>(o.L.txn), txn, 4 * k);
        memcpy(o.col<uint64_t>(o.L.lock_snap), st.col<uint64_t>(st.L.lock_snap), 8 * kl);
        memcpy(o.col<uint32_t>(o.L.lock_table), st.col<uint32_t>(st.L.lock_table), 4 * kl);
        memcpy(o.col<uint32_t>(o.L.lock_txn), ltx, 4 * kl);
        return HSC_OK;
    }
    for (int j = 0; j < W; ++j) {
        const uint64_t *slo = st.col<uint64_t>(st.L.lo) + (size_t)j * n, *shi = st.col<uint64_t>(st.L.hi) + (size_t)j * n;
        uint64_t *dlo = o.col<uint64_t>(o.L.lo) + (size_t)j * k, *dhi = o.col<uint64_t>(o.L.hi) + (size_t)j * k;
        for (size_t i = 0; i < k; ++i) dlo[i] = slo[pi[i]], dhi[i] = shi[pi[i]];
    }
    const uint64_t *ssn = st.col<uint64_t>(st.L.snap);
    const uint32_t *sg = st.col<uint32_t>(st.L.gid);
    uint64_t *osn = o.col<uint64_t>(o.L.snap);
    uint32_t *og = o.col<uint32_t>(o.L.gid), *ot = o.col<uint32_t>(o.L.txn);
    for (size_t i = 0; i < k; ++i) osn[i] = ssn[pi[i]], og[i] = sg[pi[i]], ot[i] = txn[pi[i]] - (uint32_t)t0;
    const uint64_t *sls = st.col<uint64_t>(st.L.lock_snap);
    const uint32_t *slt = st.col<uint32_t>(st.L.lock_table);
    uint64_t *ols = o.col<uint64_t>(o.L.lock_snap);
    uint32_t *olt = o.col<uint32_t>(o.L.lock_table), *olx = o.col<uint32_t>(o.L.lock_txn);
    for (size_t i = 0; i < kl; ++i) ols[i] = sls[li[i]], olt[i] = slt[li[i]], olx[i] = ltx[li[i]] - (uint32_t)t0;
    return HSC_OK;
}

// A drop-in batch on a replicated window: one member checks it whole when it
// fits the small path (one member kernel per call), else its read sets are
// cut into one slice per local member.  The members' verdicts land in their
// slices of rc_out (no OR across members: each read set is checked once).
static int replica_check(hsc_ctx *f, Stage &st, int *rc_out, std::unique_lock<std::mutex> *lk)
{
    Multi *M = f->multi;
    const int NL = M->nlocal;
    const size_t T = st.n_txn;
    const auto t0 = SteadyClock::now();
    Multi::StageSet *set = nullptr;
    {
        std::lock_guard<std::mutex> g(M->set_mu);
        if (M->free_sets.empty()) {
            M->sets.emplace_back(new (std::nothrow) Multi::StageSet());
            if (!M->sets.back()) {
                M->sets.pop_back();
                return mfail(f, HSC_ENOMEM, "multi replica staging");
            }
            M->free_sets.push_back(M->sets.back().get());
        }
        set = M->free_sets.back();
        M->free_sets.pop_back();
    }
    auto give_back = [&] {
        std::lock_guard<std::mutex> g(M->set_mu);
        M->free_sets.push_back(set);
    };
    const uint64_t epoch = M->part_epoch.load(std::memory_order_acquire);
    int parts = 1, mem_of[kMultiMax];
    size_t tb[kMultiMax + 1] = {0, T};
    if (NL > 1 && !ctx_small_fits(M->mem[0], T, st.n, st.n_lock)) {
        parts = (int)std::min<size_t>((size_t)NL, std::max<size_t>(1, T / 64));
        const int first = (int)(M->rr.fetch_add(1, std::memory_order_relaxed) % (uint32_t)NL);
        for (int p = 0; p < parts; ++p) mem_of[p] = (first + p) % NL, tb[p] = T * (size_t)p / (size_t)parts;
        tb[parts] = T;
        M->rep_sliced.fetch_add(1, std::memory_order_relaxed);
    } else {
        mem_of[0] = pick_member(M);
    }
    Stage *ms = set->s;
    int rc = HSC_OK;
    for (int p = 0; p < parts && rc == HSC_OK; ++p) rc = replica_slice(f, M->mem[mem_of[p]], st, tb[p], tb[p + 1], ms[p]);
    if (rc) {
        give_back();
        return rc;
    }
    const uint8_t *fc = st.forced.as<uint8_t>();
    for (size_t t = 0; t < T; ++t) rc_out[t] = fc[t] ? 1 : 0;
    const auto t1 = SteadyClock::now();
    M->h_calls++;
    M->ns_route += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    M->rep_calls.fetch_add(1, std::memory_order_relaxed);
    if (lk) lk->unlock();  // the batch is in the call's own set
    int slot[kMultiMax];
    bool run[kMultiMax] = {};
    int nrun = 0, fail_p = -1;
    for (int p = 0; p < parts && rc == HSC_OK; ++p) {
        M->inflight[mem_of[p]].fetch_add(1, std::memory_order_relaxed);
        rc = ctx_stage_launch(M->mem[mem_of[p]], ms[p], &slot[p]);
        if (rc == HSC_OK) {
            run[p] = true, nrun++;
        } else {
            M->inflight[mem_of[p]].fetch_sub(1, std::memory_order_relaxed);
            fail_p = p;
        }
    }
    const auto t2 = SteadyClock::now();
    static thread_local std::vector<int> rcm;
    for (int p = 0; p < parts; ++p) {
        if (!run[p]) continue;
        rcm.resize(std::max<size_t>(tb[p + 1] - tb[p], 1));
        const int r = ctx_stage_wait(M->mem[mem_of[p]], ms[p], slot[p], rcm.data());
        M->inflight[mem_of[p]].fetch_sub(1, std::memory_order_relaxed);
        if (r) {
            if (rc == HSC_OK) rc = r, fail_p = p;
            continue;
        }
        for (size_t t = tb[p]; t < tb[p + 1]; ++t) rc_out[t] |= rcm[t - tb[p]];
    }
    give_back();
    const auto t3 = SteadyClock::now();
    M->ns_launch_a.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count(),
                             std::memory_order_relaxed);
    M->ns_wait.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t3 - t2).count(),
                         std::memory_order_relaxed);
    M->members_run.fetch_add((uint64_t)nrun, std::memory_order_relaxed);
    const bool moved = M->part_epoch.load(std::memory_order_acquire) != epoch;
    if (rc == HSC_OK && !moved) return HSC_OK;
    if (lk) lk->lock();
    if (rc == HSC_OK) return mfail(f, HSC_ESTATE, "multi context re-placed during the check");
    return mfail(f, rc, ("member check: " + M->mem[mem_of[fail_p < 0 ? 0 : fail_p]]->err).c_str());
}

// Device-resident batches on a replicated window (hsc_multi_probe_device):
// each local member probes its own batch against its replica; its verdict
// bits go straight to b[m].bitmap (no routing, no exchange, no merge).
static int replica_probe_device(hsc_ctx *f, const hsc_probe_batch *b, int L)
{
    Multi *M = f->multi;
    const int NL = M->nlocal;
    for (int m = 0; m < NL; ++m)
        if (b[m].n > 0xFFFFFFFFull || b[m].n_lock > 0xFFFFFFFFull || b[m].n_txn > 0x7FFFFFFFull ||
            (b[m].n_txn && !b[m].bitmap))
            return mfail(f, HSC_EINVAL, "multi probe batch");
    MRC(lane_acquire(f, M, L));
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
        hsc_ctx *c = M->mem[m];
        hsc_probe_batch x = b[m];
        MCHK(f, hipSetDevice(c->device));
        MCHK(f, ml.verdict.ensure(std::max<size_t>(x.n_txn, 64)));
        x.verdict = ml.verdict.as<uint8_t>();
        MuGuard g(c);
        if (c->dirty) return mfail(f, HSC_ESTATE, "member window not built");
        if (c->app_last) MCHK(f, hipStreamWaitEvent(ml.stream, c->app_last, 0));
        hipStream_t keep = c->stream;
        MCHK(f, ctx_switch_stream(c, ml.stream));
        const int rc = ctx_probe(c, &x);
        MCHK(f, ctx_switch_stream(c, keep));
        if (rc) return mfail(f, rc, ("member probe: " + c->err).c_str());
        if (NL > 1) MCHK(f, hipEventRecord(ml.ev_done, ml.stream));
        ml.used = true;
        M->probes += x.n, M->routed += x.n;
    }
    M->last_lane = L;
    M->batches++;
    return HSC_OK;
}

int multi_check_stage(hsc_ctx *f, Stage &st, int *rc_out, std::unique_lock<std::mutex> *lk)
{
    Multi *M = f->multi;
    if (M->replicated) return replica_check(f, st, rc_out, lk);
    if (M->rccl) return check_stage_device(f, st, rc_out);
    const int N = M->world;
    const size_t T = st.n_txn;
    const auto t0 = SteadyClock::now();
    Multi::StageSet *set = nullptr;
    {
        std::lock_guard<std::mutex> g(M->set_mu);
        if (M->free_sets.empty()) {
            M->sets.emplace_back(new (std::nothrow) Multi::StageSet());
            if (!M->sets.back()) {
                M->sets.pop_back();
                return mfail(f, HSC_ENOMEM, "multi routing staging");
            }
            M->free_sets.push_back(M->sets.back().get());
        }
        set = M->free_sets.back();
        M->free_sets.pop_back();
    }
    auto give_back = [&] {
        std::lock_guard<std::mutex> g(M->set_mu);
        M->free_sets.push_back(set);
    };
    Stage *ms = set->s;
    const uint64_t epoch = M->part_epoch.load(std::memory_order_acquire);
    int rc = route_host(f, st, ms, -1, 0, [&](int d, size_t n, size_t nl) {
        return ctx_small_fits(M->mem[d], T, n, nl);
    });
    if (rc) {
        give_back();
        return rc;
    }
    const auto t1 = SteadyClock::now();
    const uint8_t *fc = st.forced.as<uint8_t>();
    for (size_t t = 0; t < T; ++t) rc_out[t] = fc[t] ? 1 : 0;
    M->h_calls++;
    M->ns_route += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    // the batch is in the call's own set now: the next caller marshals and
    // routes while this one launches and waits (the members take their own
    // locks; the window cannot change under a check: every change takes the
    // front lock and waits for the members' slots)
    if (lk) lk->unlock();
    int slot[kMultiMax];
    bool run[kMultiMax] = {};
    int nrun = 0;
    for (int d = 0; d < N && rc == HSC_OK; ++d) {
        if (!ms[d].n && !ms[d].n_lock) continue;  // nothing of this batch lives there
        rc = ctx_stage_launch(M->mem[d], ms[d], &slot[d]);
        if (rc == HSC_OK) run[d] = true, nrun++;
    }
    const auto t2 = SteadyClock::now();
    // every launched member is waited for, also after a failed launch
    static thread_local std::vector<int> rcm;
    rcm.resize(std::max<size_t>(T, 1));
    int fail_d = rc ? N : -1;
    for (int d = 0; d < N; ++d) {
        if (!run[d]) continue;
        const int r = ctx_stage_wait(M->mem[d], ms[d], slot[d], rcm.data());
        if (r) {
            if (rc == HSC_OK) rc = r, fail_d = d;
            continue;
        }
        for (size_t t = 0; t < T; ++t) rc_out[t] |= rcm[t];
    }
    give_back();
    const auto t3 = SteadyClock::now();
    M->ns_launch_a.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count(),
                             std::memory_order_relaxed);
    M->ns_wait.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t3 - t2).count(),
                         std::memory_order_relaxed);
    M->members_run.fetch_add((uint64_t)nrun, std::memory_order_relaxed);
    // a re-partition (new splitters, a rebuild) between the routing and the
    // launches would have sent ranges to members that no longer hold them:
    // fail closed
    const bool moved = M->part_epoch.load(std::memory_order_acquire) != epoch;
    if (rc == HSC_OK && !moved) return HSC_OK;  // (lk stays released)
    if (lk) lk->lock();  // the caller's contract: failures are recorded under the lock
    if (rc == HSC_OK) return mfail(f, HSC_ESTATE, "multi context re-partitioned during the check");
    for (int d = 0; d < N; ++d)  // the failing member's message
        if (d == fail_d || (fail_d == N && !run[d] && (ms[d].n || ms[d].n_lock)))
            return mfail(f, rc, ("member check: " + M->mem[d]->err).c_str());
    return mfail(f, rc, "member check");
}

// Per-rank context: this rank's read sets, uploaded to its member and routed
// on the devices (count, scatter, RCCL exchange), verdicts back to this rank.
static int check_stage_device(hsc_ctx *f, Stage &st, int *rc_out)
{
    Multi *M = f->multi;
    const int W = f->W, NL = M->nlocal, L = 0;
    MSource src[kMultiMax] = {};
    const size_t n = st.n;
    MRC(lane_acquire(f, M, L));
    for (int m = 0; m < NL; ++m) {
        MLane &ml = M->lane[L][m];
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
    // the verdicts land on this rank's member (its own read sets)
    MLane &o = M->lane[L][0];
    const size_t words = r64(st.n_txn) / 64;
    MCHK(f, hipSetDevice(M->mem[0]->device));
    MCHK(f, o.out.ensure(8 * std::max<size_t>(words, 1)));
    src[0].out = o.out.as<uint64_t>();
    MRC(run_pipeline(f, L, src, false));
    if (o.h_io.ensure(8 * words + 64, true)) return mfail(f, HSC_ENOMEM, "multi staging");
    uint64_t *hb = o.h_io.as<uint64_t>();
    if (words) MCHK(f, hipMemcpyAsync(hb, o.out.p, 8 * words, hipMemcpyDeviceToHost, o.stream));
    MCHK(f, hipStreamSynchronize(o.stream));
    const uint8_t *fc = st.forced.as<uint8_t>();
    for (size_t t = 0; t < st.n_txn; ++t) rc_out[t] = (fc[t] || ((hb[t >> 6] >> (t & 63)) & 1)) ? 1 : 0;
    return HSC_OK;
}

bool multi_adopted(const hsc_ctx *f) { return f && f->multi && f->multi->adopted; }

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
            for (hipEvent_t e : {ml.ev_count, ml.ev_scatter, ml.ev_probe, ml.ev_done, ml.ev_t0, ml.ev_t1})
                if (e) (void)hipEventDestroy(e);
            (void)hipStreamDestroy(ml.stream);
        }
    if (M->rccl && rccl().ok)
        for (auto &c : M->comm)
            if (c) (void)rccl().CommDestroy(c);
    for (Stage &st : M->mst) st.release();
    for (auto &ss : M->sets)
        for (Stage &st : ss->s) st.release();
    for (int m = 0; m < M->nlocal; ++m) {
        if (!M->mem[m]) continue;
        (void)hipSetDevice(M->mem[m]->device);
        for (DBuf *b : {&M->g_cover[m], &M->g_rows[m], &M->g_all[m], &M->g_sz[m]}) b->release();
    }
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
    M->ndev = 0;
    for (int i = 0; i < n; ++i) {
        bool seen = false;
        for (int j = 0; j < i; ++j) seen |= devices[j] == devices[i];
        M->ndev += !seen;
    }
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
    MuGuard g(f);
    for (size_t k = 1; k < S; ++k) {  // ascending (equal: an empty piece)
        int c = gid[k - 1] < gid[k] ? -1 : gid[k - 1] > gid[k] ? 1 : 0;
        for (int j = 0; j < W && !c; ++j)
            if (words[(size_t)j * S + k - 1] != words[(size_t)j * S + k])
                c = words[(size_t)j * S + k - 1] < words[(size_t)j * S + k] ? -1 : 1;
        if (c > 0) return mfail(f, HSC_EINVAL, "splitters not ascending");
    }
    M->part_epoch.fetch_add(1, std::memory_order_acq_rel);
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
    MuGuard g(f);
    const bool rep = M->mode == HSC_MULTI_REPLICAS;
    // the routing of every probe follows the splitters: without them all
    // probes would go to member 0 and the other pieces' keys never be probed
    if (M->world > 1 && !M->sp_given && !rep)
        return mfail(f, HSC_ESTATE, "adopt: set the splitters the members' pieces were cut at first");
    // one key width: a probe's bound words are those of the front
    const int W = M->mem[0]->W;
    for (int m = 1; m < M->nlocal; ++m)
        if (M->mem[m]->W != W) return mfail(f, HSC_EINVAL, "adopt: members' key widths differ");
    // table maxima: every member answers lock probes with the global ones
    std::vector<uint64_t> tm(f->h_table_max);
    for (int m = 0; m < M->nlocal; ++m) {
        hsc_ctx *c = M->mem[m];
        if (c->dirty) return mfail(f, HSC_ESTATE, "adopt: a member's window is not built");
        if (c->groups.size() != f->groups.size()) return mfail(f, HSC_EINVAL, "adopt: member groups differ");
        for (size_t t = 0; t < std::min(tm.size(), c->h_table_max.size()); ++t)
            tm[t] = std::max(tm[t], c->h_table_max[t]);
    }
    // replicas: every member holds the same window (its row count and first
    // and last keys); pieces: every member's rows inside its piece
    if (rep) {
        uint32_t g0[2];
        uint64_t w0[2 * kMaxWords];
        for (int m = 0; m < M->nlocal; ++m) {
            hsc_ctx *c = M->mem[m];
            if (c->n != M->mem[0]->n) return mfail(f, HSC_EINVAL, "adopt: replicas hold different rows");
            if (!c->n) continue;
            uint32_t kg[2];
            uint64_t kw[2 * kMaxWords];
            const int rc = ctx_edge_keys(c, kg, kw);
            if (rc) return mfail(f, rc, ("adopt: member keys: " + c->err).c_str());
            if (m == 0) {
                memcpy(g0, kg, sizeof g0), memcpy(w0, kw, sizeof w0);
            } else if (memcmp(g0, kg, sizeof g0) || memcmp(w0, kw, 16 * (size_t)W)) {
                return mfail(f, HSC_EINVAL, "adopt: replicas hold different rows");
            }
        }
    } else if (M->world > 1) {
        f->W = W;
        MRC(upload_splitters(f, M, W));
        for (int m = 0; m < M->nlocal; ++m) {
            hsc_ctx *c = M->mem[m];
            if (!c->n) continue;
            uint32_t kg[2];
            uint64_t kw[2 * kMaxWords];
            const int rc = ctx_edge_keys(c, kg, kw);
            if (rc) return mfail(f, rc, ("adopt: member keys: " + c->err).c_str());
            const int me = M->rank + m;
            if (sp_owner(M, kg[0], kw, W) != me || sp_owner(M, kg[1], kw + W, W) != me)
                return mfail(f, HSC_EINVAL, "adopt: a member holds keys outside its piece");
        }
    }
    if (M->rccl && !tm.empty()) {
        hsc_ctx *c = M->mem[0];
        MCHK(f, hipSetDevice(c->device));
        MRC(lane_stream(f, M, 0, 0));
        MLane &ml = M->lane[0][0];
        MCHK(f, ml.gather.ensure(8 * tm.size()));
        MCHK(f, hipMemcpyAsync(ml.gather.p, tm.data(), 8 * tm.size(), hipMemcpyHostToDevice, ml.stream));
        NCHK(f, rccl().AllReduce(ml.gather.p, ml.gather.p, tm.size(), ncclUint64, ncclMax, M->comm[0], ml.stream));
        MCHK(f, hipMemcpyAsync(tm.data(), ml.gather.p, 8 * tm.size(), hipMemcpyDeviceToHost, ml.stream));
        MCHK(f, hipStreamSynchronize(ml.stream));
    }
    f->h_table_max = tm;
    for (uint64_t v : tm) f->max_commit = std::max(f->max_commit, v);
    for (int m = 0; m < M->nlocal; ++m) {
        const int rc = hsc_merge_table_max(M->mem[m], tm.data(), (int)std::min(tm.size(), M->mem[m]->table_names.size()));
        if (rc) return mfail(f, rc, "adopt: table maxima");
        f->end_lsn = std::max(f->end_lsn, M->mem[m]->end_lsn);
    }
    f->W = W;
    size_t keys = 0;
    for (int m = 0; m < M->nlocal; ++m) keys += M->mem[m]->n;
    f->n = rep ? M->mem[0]->n : keys;
    M->part_epoch.fetch_add(1, std::memory_order_acq_rel);
    M->adopted = true;
    M->replicated = rep;
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
    MuGuard g(f);
    if (f->dirty) return mfail(f, HSC_ESTATE, "window not built");
    if (M->replicated) return replica_probe_device(f, b, lane);
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

int hsc_multi_phase_stats(hsc_ctx *f, double out[7])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    Multi *M = f->multi;
    const uint64_t routed_dev = M->batches - M->pr_batches;  // run_pipeline batches
    const double b = (double)std::max<uint64_t>(routed_dev, 1) * 1e3;
    out[0] = (double)routed_dev;
    out[1] = (double)M->ns_lane / b;
    out[2] = (double)M->ns_count / b;
    out[3] = (double)M->ns_count_wait / b;
    out[4] = (double)M->ns_enqueue / b;
    out[5] = (double)M->pr_batches;
    out[6] = (double)M->ns_pr / ((double)std::max<uint64_t>(M->pr_batches, 1) * 1e3);
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

int hsc_multi_set_transport(hsc_ctx *f, int transport)
{
    if (!f || !f->multi || transport < HSC_MULTI_DIRECT || transport > HSC_MULTI_LOOPBACK) return HSC_EINVAL;
    Multi *M = f->multi;
    MuGuard g(f);
    if (M->rccl) return transport == HSC_MULTI_DIRECT ? HSC_OK : mfail(f, HSC_EINVAL, "per-rank context: RCCL");
    for (int L = 0; L < kMultiLanes; ++L)  // nothing of the other form in flight
        for (int m = 0; m < M->nlocal; ++m)
            if (M->lane[L][m].used)
                MCHK(f, M->nlocal > 1 ? hipEventSynchronize(M->lane[L][m].ev_done)
                                      : hipStreamSynchronize(M->lane[L][m].stream));
    M->loop = transport == HSC_MULTI_LOOPBACK;
    return HSC_OK;
}

int hsc_multi_routed_phase_stats(hsc_ctx *f, double out[4])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    Multi *M = f->multi;
    const double b = (double)std::max<uint64_t>(M->pr_batches, 1) * 1e3;
    out[0] = (double)M->pr_batches;
    out[1] = (double)M->ns_pr_lane / b;
    out[2] = (double)M->ns_pr_probe / b;
    out[3] = (double)M->ns_pr_merge / b;
    return HSC_OK;
}

int hsc_multi_set_mode(hsc_ctx *f, int mode)
{
    if (!f || !f->multi || mode < HSC_MULTI_AUTO || mode > HSC_MULTI_REPLICAS) return HSC_EINVAL;
    Multi *M = f->multi;
    MuGuard g(f);
    if (M->mode == mode) return HSC_OK;
    M->mode = mode;
    M->part_epoch.fetch_add(1, std::memory_order_acq_rel);
    if (f->host_staged) f->dirty = true;  // re-placed at the next check
    return HSC_OK;
}

int hsc_multi_mode(hsc_ctx *f)
{
    if (!f || !f->multi) return HSC_EINVAL;
    return f->multi->replicated ? HSC_MULTI_REPLICAS : HSC_MULTI_PIECES;
}

int hsc_multi_probe_routed(hsc_ctx *f, const hsc_probe_batch *b, const uint64_t *owner_base, int lane)
{
    if (!f || !f->multi || !b || !owner_base || lane < 0 || lane >= kMultiLanes) return HSC_EINVAL;
    Multi *M = f->multi;
    const int N = M->world, NL = M->nlocal;
    MuGuard g(f);
    if (f->dirty) return mfail(f, HSC_ESTATE, "window not built");
    if (M->replicated) return mfail(f, HSC_ESTATE, "replicated window: probe each member (hsc_probe_device)");
    size_t tb[kMultiMax + 1];
    for (int o = 0; o <= N; ++o) {
        tb[o] = (size_t)owner_base[o];
        if ((o && tb[o] < tb[o - 1]) || (tb[o] & 63) || (o == 0 && tb[0]) || tb[o] > 0xFFFFFFFFull)
            return mfail(f, HSC_EINVAL, "owner bases: ascending multiples of 64 from 0");
    }
    hsc_probe_batch in[kMultiMax];
    uint64_t *outs[kMultiMax] = {};
    for (int m = 0; m < NL; ++m) {
        const int o = M->rank + m;
        if (b[m].n > 0xFFFFFFFFull || b[m].n_lock > 0xFFFFFFFFull || ((tb[o + 1] > tb[o]) && !b[m].bitmap) ||
            (b[m].n_lock && o != 0))
            return mfail(f, HSC_EINVAL, "multi routed batch (locks go to member 0)");
        in[m] = b[m];
        outs[m] = b[m].bitmap;
    }
    const auto t0 = SteadyClock::now();
    MRC(lane_acquire(f, M, lane));
    const auto t1 = SteadyClock::now();
    MRC(probe_merge(f, lane, in, tb, outs));
    for (int m = 0; m < NL; ++m) M->routed += b[m].n, M->probes += b[m].n;
    M->pr_batches++;
    M->ns_pr += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(SteadyClock::now() - t0).count();
    M->ns_pr_lane += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    M->ns_pr_probe += M->ns_pm_probe;
    M->ns_pr_merge += M->ns_pm_merge;
    return HSC_OK;
}

int hsc_multi_marshal_routed(hsc_ctx *f, const hsc_readsets *rs, int member, uint32_t txn_base,
                             const hsc_marshalled **out)
{
    if (!f || !f->multi || !rs || !out || member < -1 || member >= f->multi->world) return HSC_EINVAL;
    const hsc_marshalled *m = nullptr;
    int rc = hsc_marshal_readsets(f, rs, &m);
    if (rc) return rc;
    Multi *M = f->multi;
    MuGuard g(f);
    Stage &st = f->stage[0];
    rc = route_host(f, st, M->mst, member, txn_base, nullptr);
    if (rc) return rc;
    return hsc_multi_routed_member(f, member < 0 ? 0 : member, out);
}

int hsc_multi_routed_member(hsc_ctx *f, int member, const hsc_marshalled **out)
{
    if (!f || !f->multi || !out || member < 0 || member >= f->multi->world) return HSC_EINVAL;
    Multi *M = f->multi;
    const Stage &st = f->stage[0];
    const Stage &o = M->mst[member];
    static thread_local hsc_marshalled r;
    r = hsc_marshalled{};
    r.n = o.n;
    r.n_lock = o.n_lock;
    r.n_txn = o.n_txn;
    r.words = f->W;
    r.lo = o.col<uint64_t>(o.L.lo);
    r.hi = o.col<uint64_t>(o.L.hi);
    r.gid = o.col<uint32_t>(o.L.gid);
    r.snap = o.col<uint64_t>(o.L.snap);
    r.txn = o.col<uint32_t>(o.L.txn);
    r.lock_table = o.col<uint32_t>(o.L.lock_table);
    r.lock_snap = o.col<uint64_t>(o.L.lock_snap);
    r.lock_txn = o.col<uint32_t>(o.L.lock_txn);
    r.forced = st.forced.as<uint8_t>();
    *out = &r;
    return HSC_OK;
}

int hsc_multi_enable_timing(hsc_ctx *f, int on)
{
    if (!f || !f->multi) return HSC_EINVAL;
    f->multi->timing = on != 0;
    return HSC_OK;
}

int hsc_multi_member_probe_ms(hsc_ctx *f, float *out, int n)
{
    if (!f || !f->multi || !out || n < f->multi->nlocal) return HSC_EINVAL;
    Multi *M = f->multi;
    for (int m = 0; m < M->nlocal; ++m) {
        MLane &ml = M->lane[M->last_lane][m];
        out[m] = 0;
        if (!ml.timed || !ml.ev_t1) continue;
        MCHK(f, hipSetDevice(M->mem[m]->device));
        MCHK(f, hipEventSynchronize(ml.ev_t1));
        MCHK(f, hipEventElapsedTime(&out[m], ml.ev_t0, ml.ev_t1));
    }
    return HSC_OK;
}

int hsc_multi_route_stats(hsc_ctx *f, double out[8])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    Multi *M = f->multi;
    const double c = M->h_calls ? (double)M->h_calls : 1.0;
    out[0] = (double)M->h_calls;
    out[1] = (double)M->members_run.load();
    out[2] = (double)M->h_probes;
    out[3] = (double)M->h_routed;
    out[4] = (double)M->ns_route / c * 1e-3;
    out[5] = (double)M->world;
    out[6] = (double)M->ns_launch_a.load() / c * 1e-3;
    out[7] = (double)M->ns_wait.load() / c * 1e-3;
    return HSC_OK;
}

int hsc_multi_graph_scc(hsc_ctx *f, const hsc_ops_dev *ops, uint32_t ntxn, uint32_t *const *scc_dev,
                        hsc_graph_stats *st)
{
    if (!f || !f->multi || !ops || !scc_dev || !scc_dev[0]) return HSC_EINVAL;
    Multi *M = f->multi;
    const int N = M->world, NL = M->nlocal;
    MuGuard g(f);
    const auto t0 = SteadyClock::now();
    for (int m = 0; m < NL; ++m) MRC(lane_stream(f, M, 0, m));
    const size_t cb = r64(std::max<uint32_t>(ntxn, 1));  // cover bytes, whole u64 words
    float build_ms = 0;
    // 1. every member builds the raw edges of its key shard and its cover
    for (int m = 0; m < NL; ++m) {
        hsc_ctx *c = M->mem[m];
        hsc_graph_stats bs{};
        int rc = hsc_dep_graph_build_device(c, ops[m].nops, ntxn, ops[m].txn, ops[m].key, ops[m].is_write,
                                            ops[m].observed, 0, &bs);
        if (rc) return mfail(f, rc, ("graph build: " + c->err).c_str());
        build_ms = std::max(build_ms, bs.build_ms);
        MCHK(f, hipSetDevice(c->device));
        MCHK(f, M->g_cover[m].ensure(cb));
        // on the member's stream, ahead of its cover kernels (a NULL-stream
        // memset is not ordered with the members' non-blocking streams)
        MCHK(f, hipMemsetAsync(M->g_cover[m].p, 0, cb, c->stream));
        rc = hsc_dep_graph_cover(c, M->g_cover[m].as<uint8_t>());
        if (rc) return mfail(f, rc, ("graph cover: " + c->err).c_str());
    }
    const auto t1 = SteadyClock::now();
    // 2. the covers OR-ed (0 / 1 bytes: MAX) over every member
    Rccl &R = rccl();
    MLane &l0 = M->lane[0][0];
    if (M->rccl) {
        if (N > 1) {
            MCHK(f, hipSetDevice(M->mem[0]->device));
            NCHK(f, R.AllReduce(M->g_cover[0].p, M->g_cover[0].p, cb, ncclUint8, ncclMax, M->comm[0], l0.stream));
            MCHK(f, hipStreamSynchronize(l0.stream));
        }
    } else if (NL > 1) {
        RouteParts parts{};
        parts.n = NL;
        for (int d = 0; d < NL; ++d) parts.p[d] = M->g_cover[d].as<uint64_t>();
        MCHK(f, hipSetDevice(M->mem[0]->device));
        MCHK(f, launch_or_slices(parts, cb / 8, M->g_cover[0].as<uint64_t>(), l0.stream));
        for (int d = 1; d < NL; ++d)
            MCHK(f, hipMemcpyPeerAsync(M->g_cover[d].p, M->mem[d]->device, M->g_cover[0].p, M->mem[0]->device, cb,
                                       l0.stream));
        MCHK(f, hipStreamSynchronize(l0.stream));
    }
    const auto t2 = SteadyClock::now();
    // 3. every member's edges between covered txns
    size_t k[kMultiMax] = {};
    const uint64_t *cut[kMultiMax] = {};
    for (int m = 0; m < NL; ++m) {
        hsc_ctx *c = M->mem[m];
        // (the build's ops are the caller's, live for this call)
        const int rc = ctx_graph_cut(c, M->g_cover[m].as<uint8_t>(), &k[m], &cut[m], ops[m].txn, ops[m].key,
                                     ops[m].is_write);
        if (rc) return mfail(f, rc, ("graph cut: " + c->err).c_str());
    }
    // 4. the union of the cuts where the SCC runs: every rank (all-gather,
    // each rank's rows padded with ~0 to the largest), or member 0 here
    const uint64_t *rows = cut[0];
    size_t total = k[0], cut_rows = k[0];
    if (M->rccl && N > 1) {
        MCHK(f, hipSetDevice(M->mem[0]->device));
        MCHK(f, M->g_sz[0].ensure(8 * (size_t)(N + 1)));
        uint64_t mine = k[0];
        MCHK(f, hipMemcpyAsync(M->g_sz[0].p, &mine, 8, hipMemcpyHostToDevice, l0.stream));
        NCHK(f, R.AllGather(M->g_sz[0].p, M->g_sz[0].as<uint64_t>() + 1, 1, ncclUint64, M->comm[0], l0.stream));
        std::vector<uint64_t> sz(N);
        MCHK(f, hipMemcpyAsync(sz.data(), M->g_sz[0].as<uint64_t>() + 1, 8 * (size_t)N, hipMemcpyDeviceToHost,
                               l0.stream));
        MCHK(f, hipStreamSynchronize(l0.stream));
        size_t mx = 1;
        cut_rows = 0;
        for (int r = 0; r < N; ++r) mx = std::max<size_t>(mx, sz[r]), cut_rows += sz[r];
        MCHK(f, M->g_rows[0].ensure(8 * mx));
        if (k[0]) MCHK(f, hipMemcpyAsync(M->g_rows[0].p, cut[0], 8 * k[0], hipMemcpyDeviceToDevice, l0.stream));
        if (mx > k[0]) MCHK(f, hipMemsetAsync(M->g_rows[0].as<uint64_t>() + k[0], 0xFF, 8 * (mx - k[0]), l0.stream));
        MCHK(f, M->g_all[0].ensure(8 * mx * (size_t)N));
        NCHK(f, R.AllGather(M->g_rows[0].p, M->g_all[0].p, mx, ncclUint64, M->comm[0], l0.stream));
        MCHK(f, hipStreamSynchronize(l0.stream));
        rows = M->g_all[0].as<uint64_t>();
        total = mx * (size_t)N;
    } else if (NL > 1) {
        total = 0;
        for (int d = 0; d < NL; ++d) total += k[d];
        cut_rows = total;
        MCHK(f, hipSetDevice(M->mem[0]->device));
        MCHK(f, M->g_all[0].ensure(8 * std::max<size_t>(total, 1)));
        size_t o = 0;
        for (int d = 0; d < NL; ++d) {
            if (k[d])
                MCHK(f, hipMemcpyPeerAsync(M->g_all[0].as<uint64_t>() + o, M->mem[0]->device, cut[d],
                                           M->mem[d]->device, 8 * k[d], l0.stream));
            o += k[d];
        }
        MCHK(f, hipStreamSynchronize(l0.stream));  // (the SCC runs on member 0's own stream)
        rows = M->g_all[0].as<uint64_t>();
    }
    const auto t3 = SteadyClock::now();
    // 5. SCC of the cut union (components of >= 2 txns live there)
    hsc_graph_stats ss{};
    int rc = hsc_dep_graph_scc_cut(M->mem[0], ntxn, M->g_cover[0].as<uint8_t>(), rows, total, scc_dev[0], &ss);
    if (rc) return mfail(f, rc, ("graph scc: " + M->mem[0]->err).c_str());
    for (int d = 1; d < NL; ++d)  // in process: the same components on every member that asked
        if (scc_dev[d])
            MCHK(f, hipMemcpyPeerAsync(scc_dev[d], M->mem[d]->device, scc_dev[0], M->mem[0]->device,
                                       4 * (size_t)ntxn, l0.stream));
    if (NL > 1) MCHK(f, hipStreamSynchronize(l0.stream));
    const auto t4 = SteadyClock::now();
    if (st) {
        *st = ss;
        st->build_ms = build_ms;
        st->edges = cut_rows;  // rows of the cut union (every shard's)
    }
    auto ms = [](SteadyClock::time_point a, SteadyClock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    M->g_ms[0] = ms(t0, t1), M->g_ms[1] = ms(t1, t2), M->g_ms[2] = ms(t2, t3), M->g_ms[3] = ms(t3, t4);
    return HSC_OK;
}

int hsc_multi_graph_phase_ms(hsc_ctx *f, double out[4])
{
    if (!f || !f->multi || !out) return HSC_EINVAL;
    for (int i = 0; i < 4; ++i) out[i] = f->multi->g_ms[i];
    return HSC_OK;
}

}  // extern "C"
