// hsc_ctx.h -- the validator context (struct hsc_ctx) and the host-side
// types it holds, shared by hsc_host.cpp (single-GPU context) and
// hsc_multi.cpp (the multi-GPU context built from member contexts).
#pragma once
#include "../../include/hip_serial.h"
#include "hsc_internal.h"

#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <memory>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace hsc {


struct GroupInfo {
    int tid, ix, klen;
};

inline uint64_t load_be64(const uint8_t *b)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | b[i];
    return v;
}

inline uint64_t ixkey(int tid, int ix) { return ((uint64_t)(uint32_t)tid << 32) | (uint32_t)ix; }

// Host staging buffer: pinned (hipHostMalloc) on a device context, so that
// uploads and verdict downloads are DMA from / to it; malloc on a host-only
// one.  Grows, never shrinks.
struct HBuf {
    void *p = nullptr;
    void *dp = nullptr;  // coherent buffers: the device's address of p
    size_t bytes = 0;
    bool pinned = false, coherent = false;
    // 0 or -1 (out of memory).  coherent: fine-grained pinned memory the GPU
    // maps (kernels read and write it directly, the host sees their
    // system-scope stores while they run).
    int ensure(size_t want, bool pin, bool coh = false)
    {
        if (want <= bytes && pin == pinned && coh == coherent) return 0;
        release();
        const size_t b = want + want / 8 + 256;
        if (pin) {
            const unsigned flags = coh ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault;
            if (hipHostMalloc(&p, b, flags) != hipSuccess) {
                p = nullptr;
                return -1;
            }
            if (coh && hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
                (void)hipHostFree(p);
                p = dp = nullptr;
                return -1;
            }
        } else if (!(p = malloc(b))) {
            return -1;
        }
        bytes = b;
        pinned = pin;
        coherent = coh && pin;
        return 0;
    }
    void release()
    {
        if (p) {
            if (pinned)
                (void)hipHostFree(p);
            else
                free(p);
        }
        p = dp = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return (T *)p; }
};

// One marshalled batch (or pipeline chunk) in host memory: probe SoA,
// forced verdicts, and the verdict bytes read back.
// Byte offsets of a marshalled batch's columns inside one staging arena (and
// the device arena it is uploaded to with ONE copy): a small batch -- the
// collector's usual tens of read sets -- pays one transfer, not eight.
struct StageLayout {
    size_t lo = 0, hi = 0, snap = 0, lock_snap = 0, gid = 0, txn = 0, lock_table = 0,
           lock_txn = 0, total = 0;
};

inline StageLayout stage_layout(int W, size_t n, size_t nl)
{
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    StageLayout L;
    size_t o = 0;
    L.lo = o, o = al(o + 8 * (size_t)W * n);
    L.hi = o, o = al(o + 8 * (size_t)W * n);
    L.snap = o, o = al(o + 8 * n);
    L.lock_snap = o, o = al(o + 8 * nl);
    L.gid = o, o = al(o + 4 * n);
    L.txn = o, o = al(o + 4 * n);
    L.lock_table = o, o = al(o + 4 * nl);
    L.lock_txn = o, o = al(o + 4 * nl);
    L.total = o;
    return L;
}

// Room a small batch's slot needs past the columns: the verdict bytes and the
// done word, each 64-byte aligned (hsc_ctx::SmallSlot).
inline size_t small_tail(size_t n_txn) { return 64 + ((n_txn + 63) & ~(size_t)63) + 64; }

struct Stage {
    HBuf arena, forced, verdict;
    StageLayout L;
    size_t n = 0, n_lock = 0, n_txn = 0;
    // the small-batch stage: its arena is fine-grained pinned memory with room
    // for the slot's verdicts and done word, and moves into the slot at launch
    // (the kernel reads the columns where the marshal wrote them)
    bool coh = false;
    hipEvent_t done = nullptr;  // the chunk's verdict download
    template <class T>
    T *col(size_t off) const
    {
        return (T *)((uint8_t *)arena.p + off);
    }
    void release()
    {
        for (HBuf *b : {&arena, &forced, &verdict}) b->release();
        if (done) (void)hipEventDestroy(done);
        done = nullptr;
    }
};

constexpr int kMarshalTxns = 2048;         // read sets per marshal work item
enum { kFoldIdle = 0, kFoldRunning = 1, kFoldDone = 2 };  // hsc_ctx::fold_state
constexpr int kMarshalParallelMin = 4096;  // fewer read sets: marshal on the caller's thread
constexpr int kPipeTxns = 32768;           // read sets per pipeline chunk of a large batch


// One table of a read set: islocked of its first range (db/sqlglue.c:322-326)
// and its index spans [b, e] in array order (:327-349), spans[s0 .. s0 + ns).
struct TxnTable {
    int tid, islocked, s0, ns;
};
struct IdxSpan {
    int idx, b, e;
    const std::vector<int> *groups;  // the (table, index)'s key groups, null: none
};

// Growable array of trivially copyable T whose growth does not initialise
// the new elements (the marshal writes every one it keeps).
template <class T>
struct PodVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    PodVec() = default;
    PodVec(const PodVec &) = delete;
    PodVec &operator=(const PodVec &) = delete;
    PodVec(PodVec &&o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr, o.n = o.cap = 0; }
    ~PodVec() { free(p); }
    void reserve(size_t k)
    {
        if (k <= cap) return;
        const size_t c = std::max(k, 2 * cap + 64);
        T *q = (T *)realloc(p, c * sizeof(T));
        if (!q) throw std::bad_alloc();
        p = q, cap = c;
    }
    void resize(size_t k) { reserve(k), n = k; }
    void clear() { n = 0; }
    size_t size() const { return n; }
    T *data() { return p; }
    const T *data() const { return p; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
    void push_back(const T &v) { reserve(n + 1), p[n++] = v; }
    void append(const T *src, size_t k)
    {
        reserve(n + k);
        if (k) memcpy(p + n, src, k * sizeof(T));
        n += k;
    }
    void append_fill(size_t k, const T &v)
    {
        reserve(n + k);
        for (size_t i = 0; i < k; ++i) p[n + i] = v;
        n += k;
    }
};

// Append-only array of trivially copyable T for the stores that grow with
// every commit (the log records, the host-staged rows): its pages are mapped
// directly and grown with mremap, which moves page tables instead of copying
// the contents, so an append never pays a copy of everything before it
// (std::vector's doubling cost a 0.6-1.2 ms stall per doubling at 2^17 and
// 2^18 records of a commit stream).
template <class T>
struct MapVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    MapVec() = default;
    MapVec(const MapVec &) = delete;
    MapVec &operator=(const MapVec &) = delete;
    ~MapVec()
    {
        if (p) munmap(p, cap * sizeof(T));
    }
    // The first reserve maps a large range of address space without
    // reserving memory (MAP_NORESERVE: pages are backed as they are first
    // written), so the store never moves; an mremap of tens of MB of page
    // tables still cost an append ~0.3 ms (r06e).  If the system refuses the
    // range, the store grows by mremap as before.
    static constexpr size_t kVirtBytes = (size_t)1 << 36;
    void reserve(size_t k)
    {
        if (k <= cap) return;
        const size_t page = 4096 / sizeof(T) ? 4096 / sizeof(T) : 1;
        if (!p) {
            const size_t cv = std::max(k, kVirtBytes / sizeof(T)) / page * page;
            void *q = mmap(nullptr, cv * sizeof(T), PROT_READ | PROT_WRITE,
                           MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
            if (q != MAP_FAILED && cv >= k) {
                // 4 KiB pages: a transparent huge page is zeroed whole at its
                // first write -- a 0.3 ms stall of the append that crosses
                // into the next 2 MiB of the store (r06f, scripts/fold_diag.py)
                (void)madvise(q, cv * sizeof(T), MADV_NOHUGEPAGE);
                p = (T *)q, cap = cv;
                return;
            }
            if (q != MAP_FAILED) munmap(q, cv * sizeof(T));
        }
        size_t c = std::max(k, std::max(2 * cap, (size_t)65536));
        c = (c + page - 1) / page * page;
        void *q = p ? mremap(p, cap * sizeof(T), c * sizeof(T), MREMAP_MAYMOVE)
                    : mmap(nullptr, c * sizeof(T), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(q, c * sizeof(T), MADV_NOHUGEPAGE);
        p = (T *)q, cap = c;
    }
    void push_back(const T &v)
    {
        if (n == cap) reserve(n + 1);
        p[n++] = v;
    }
    // append [a, b) (pos must be end())
    void insert(T *pos, const T *a, const T *b)
    {
        (void)pos;
        const size_t k = (size_t)(b - a);
        if (!k) return;
        reserve(n + k);
        memcpy(p + n, a, k * sizeof(T));
        n += k;
    }
    void clear() { n = 0; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    T *data() { return p; }
    const T *data() const { return p; }
    T *begin() { return p; }
    T *end() { return p + n; }
    const T *begin() const { return p; }
    const T *end() const { return p + n; }
    T &back() { return p[n - 1]; }
    const T &back() const { return p[n - 1]; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

// One worker's share of a marshal (read sets [t0, t1) of the batch): probes
// as AoS rows (W words of lo, W of hi) plus the scratch of the span builder.
// One range of a read set as the marshal reads it (window table id, -1 if
// the table was never written).
struct RangeRef {
    int tid;
    int idxnum;
    const uint8_t *lkey, *rkey;
    int lkeylen, rkeylen, lflag, rflag, islocked;
};
struct alignas(128) MarshalPart {  // one per worker: no shared cache lines
    PodVec<uint64_t> lohi;  // [n][2W]
    PodVec<uint64_t> snap, lock_snap;
    PodVec<uint32_t> gid, txn, lock_table, lock_txn;
    std::vector<TxnTable> tabs;
    std::vector<IdxSpan> spans;
    std::vector<RangeRef> refs;  // the read set's ranges, read once
    uint64_t ix_last = ~0ull;    // cache of the last (table, index) group lookup
    const std::vector<int> *ix_groups = nullptr;
    size_t out0 = 0, lock0 = 0;  // output offsets (assembly)
    void clear()
    {
        lohi.clear(), snap.clear(), lock_snap.clear(), gid.clear(), txn.clear();
        lock_table.clear(), lock_txn.clear();
        ix_last = ~0ull;  // the dictionary may have changed since the last marshal
        ix_groups = nullptr;
    }
};

struct Multi;  // hsc_multi.cpp: the members of a multi-GPU context

// Persistent marshal workers (one pool per context, created on first use):
// run(nwork, f) calls f(0 .. nwork - 1) on the pool's threads and the
// caller's, dynamically scheduled, and returns when all are done.  A large
// batch runs two parallel phases per pipeline chunk; spawning threads for
// each cost tens of microseconds per thread.
class WorkPool {
  public:
    explicit WorkPool(int nthreads) : size_(std::max(1, nthreads))
    {
        for (int i = 1; i < size_; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~WorkPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return size_; }
    // f(0 .. nwork - 1), dynamically scheduled
    void run(int nwork, const std::function<void(int)> &f) { go(nwork, f, false); }
    // f(i) on participant i % size() (0 = the caller): two runs over the same
    // items touch each item's data from the same core
    void run_static(int nwork, const std::function<void(int)> &f) { go(nwork, f, true); }

  private:
    void go(int nwork, const std::function<void(int)> &f, bool stat)
    {
        if (nwork <= 0) return;
        if (th_.empty() || nwork == 1) {
            for (int i = 0; i < nwork; ++i) f(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            nwork_ = nwork;
            static_ = stat;
            next_.store(0, std::memory_order_relaxed);
            busy_.store((int)th_.size(), std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        if (sleeping_.load(std::memory_order_acquire)) cv_.notify_all();
        work(0);
        // the workers finish their share (they spin between back-to-back jobs)
        while (busy_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
        job_ = nullptr;
    }
    void work(int me)
    {
        if (static_) {
            for (int i = me; i < nwork_; i += size_) (*job_)(i);
        } else {
            for (int i = next_.fetch_add(1); i < nwork_; i = next_.fetch_add(1)) (*job_)(i);
        }
    }
    // A worker spins up to kSpin for the next job (a marshal runs its phases
    // back to back: a futex wake per phase cost tens of microseconds on a
    // large host), then sleeps on the condition variable.
    void loop(int me)
    {
        uint64_t seen = 0;
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            while (gen_.load(std::memory_order_acquire) == seen &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(kSpinUs))
                __builtin_ia32_pause();
            if (gen_.load(std::memory_order_acquire) == seen) {
                std::unique_lock<std::mutex> lk(m_);
                sleeping_.fetch_add(1, std::memory_order_acq_rel);
                cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_acquire) != seen; });
                sleeping_.fetch_sub(1, std::memory_order_acq_rel);
            }
            {
                std::lock_guard<std::mutex> g(m_);
                if (stop_) return;
                seen = gen_.load(std::memory_order_acquire);
            }
            work(me);
            busy_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    static constexpr int kSpinUs = 200;
    const int size_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    const std::function<void(int)> *job_ = nullptr;
    std::atomic<int> next_{0}, busy_{0}, sleeping_{0};
    std::atomic<uint64_t> gen_{0};
    int nwork_ = 0;
    bool static_ = false;
    bool stop_ = false;
};

}  // namespace hsc

using namespace hsc;


// The dictionaries a marshal reads (key words, groups, table ids) as an
// immutable snapshot: a collector's callers marshal their own read set
// against it before they queue (premarshal, no context lock), and a batch
// takes those rows only if the context's dictionary epoch has not moved.
struct MarshalDict {
    uint64_t epoch = 0;
    int W = 1;
    std::unordered_map<std::string, int> table_ids;
    std::vector<GroupInfo> groups;
    std::unordered_map<uint64_t, std::vector<int>> ix_groups;
};

struct hsc_ctx {
    int device = 0;
    bool host_only = false;
    // multi-GPU context (hsc_multi_create*): this context keeps the
    // dictionaries, the log decode, the window rules and the marshal; its
    // window lives on the member contexts of `multi` (hsc_multi.cpp)
    Multi *multi = nullptr;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    std::mutex mu;  // one check at a time per context (re-entrant callers queue)

    // dictionaries
    std::unordered_map<std::string, int> table_ids;
    std::vector<std::string> table_names;
    std::unordered_map<uint64_t, int> group_ids;                    // (tid,ix,klen)
    std::vector<GroupInfo> groups;
    std::unordered_map<uint64_t, std::vector<int>> ix_groups;       // (tid,ix) -> gids
    uint64_t dict_epoch = 1;  // bumped when a table, a group or W changes
    // the dictionary snapshot callers premarshal against, published under mu;
    // read without a lock (one atomic load: the shared_ptr atomics go through
    // one global spinlock that hundreds of concurrent callers contend on).
    // Every version stays alive until the context is destroyed (a new one is
    // published only when a table, group or the key width changes).
    std::atomic<const MarshalDict *> dict_cur{nullptr};
    std::vector<std::unique_ptr<MarshalDict>> dict_all;
    std::vector<uint8_t> gcls;   // marshal: key-length class of every group (gcls_epoch)
    uint64_t gcls_epoch = ~0ull;

    // host staging of the window (host ingest paths)
    MapVec<uint32_t> h_gid;
    MapVec<uint64_t> h_keyoff;
    MapVec<uint8_t> h_keys;
    MapVec<uint64_t> h_lsn;
    std::vector<uint64_t> h_table_max;
    bool host_staged = true;
    bool dirty = true;
    uint64_t end_lsn = 0, max_commit = 0;
    uint64_t poison_regop = 0;  // max regop LSN whose prev record cannot be read
    uint64_t poison_chain = 0;  // max commit LSN whose logical chain is broken
    // the log a log-based window was decoded from (record LSNs for the
    // DB_SET rule, records for chain walks of txns committed by appends);
    // table = window table id
    struct LogStore {
        MapVec<uint64_t> lsn, prev, key_off;
        MapVec<uint32_t> rectype;
        MapVec<int16_t> isabort, ix;
        MapVec<int32_t> table, keylen;
        MapVec<uint8_t> keys;
        void clear()
        {
            lsn.clear(), prev.clear(), key_off.clear(), rectype.clear(), isabort.clear();
            ix.clear(), table.clear(), keylen.clear(), keys.clear();
        }
    } lg;
    bool lg_rule = false;  // every record LSN of the window is in lg (DB_SET rule on)
    uint64_t last_append_lsn = 0;
    // The regop_only answer's inputs (end_lsn, max_commit, poison_regop,
    // lg_rule), republished by MuGuard whenever a mutating entry releases mu
    // and read lock-free by the regop_only probes (a seqlock: odd while a
    // writer stores).  db/toblock.c:4779-4785 runs that probe under the
    // commit_lock write lock, so it must not queue or wait for mu.
    std::atomic<uint64_t> rg_seq{0}, rg_end{0}, rg_max{0}, rg_poison{0};
    std::atomic<uint32_t> rg_lgrule{0};
    std::atomic<uint64_t> rg_fast{0}, rg_slow{0};  // regop probes answered without / with mu
    // incremental window (hsc_delta.hip): writes committed after the last
    // build, kept on the device as a sorted delta run probed beside the main
    // window; live = a built window takes appends into the delta
    bool live = false, merge_pending = false;
    size_t ng_built = 0;  // groups the per-group device tables were sized for
    DBuf d_dgid[2], d_dwords[2], d_dlsn[2], d_dbmax;
    DBuf d_agid;  // an append's upload: rows + table maxima (stage_bytes layout)
    size_t dn = 0, dcap = 0;
    int dcur = 0;
    std::vector<uint32_t> app_gid;   // appended rows not yet on the device
    std::vector<uint8_t> app_keys;   // their key bytes (klen of the group each)
    std::vector<uint64_t> app_koff, app_lsn;
    bool app_tmax = false;           // table maxima changed since the last upload
    // pinned staging of appended rows / table maxima: a ring of two, each
    // reused only after the copies that read it ran (its event), so an append
    // returns without waiting for its upload and delta merge
    HBuf h_appq[2];
    hipEvent_t app_ev[2] = {};
    int app_i = 0;
    HBuf *h_app = nullptr;          // the buffer of the append being staged
    hipEvent_t app_last = nullptr;  // recorded behind the last append's device work
    // pending tail (narrow windows, the small-batch path): an append's rows
    // and raised table maxima are mirrored into mapped pinned memory that
    // k_small_narrow scans beside the delta runs, and stay in app_* until
    // kPendRows of them (or a batch that is not small) merge them into the
    // live run with one launch.  A ring of two: a buffer is refilled only
    // after the launch that retired it ran (its event); rows [0, pend_n) of
    // the current one never change while it is current.
    HBuf h_pend[2];
    hipEvent_t pend_ev[2] = {};
    int pend_i = 0;
    uint32_t pend_n = 0, pend_t = 0;   // rows / table entries mirrored
    std::vector<uint32_t> app_tchg;    // tables whose maximum rose since the last mirror
    uint64_t pend_appends = 0, pend_merges = 0;
    ProbeView raw_probe{};           // the batch being probed, untransformed (delta probe)
    // background fold: once the live run holds fold_rows rows it
    // is frozen, and a shadow context rebuilds the main window from the main
    // window's versions + the frozen run on its own stream and host thread;
    // checks probe main + frozen + live runs until a call after the build
    // swaps the shadow's window in (fold_poll).  fold_bg = false: the run is
    // merged inline by the next check instead (the pre-fold behaviour).
    hsc_ctx *shadow = nullptr;     // created by the fold worker (its stream too)
    std::thread fold_thread;       // the fold worker: one per context, started by its first fold
    std::mutex fold_mu;
    std::condition_variable fold_cv;
    bool fold_job = false, fold_quit = false;
    struct FoldJob {  // one fold, captured by fold_start on the caller's thread
        size_t nm = 0, nf = 0, cap = 0, dcap = 0;
        int W = 1, layout = 0;
        unsigned paths = 0;
        const void *gid2 = nullptr, *lsn2 = nullptr, *words2 = nullptr;  // main window versions
        const void *fgid = nullptr, *flsn = nullptr, *fwords = nullptr;  // the frozen run
        std::vector<GroupInfo> groups;
        std::vector<std::string> table_names;
        std::vector<uint64_t> table_max;
    } fold_jobv;
    std::atomic<int> fold_state{0};  // kFoldIdle / kFoldRunning / kFoldDone
    int fold_rc = 0;
    std::string fold_err;
    DBuf f_dgid, f_dwords, f_dlsn, f_dbmax;  // the frozen run (fn rows, stride dcap)
    size_t fn = 0;
    size_t fold_rows = kDeltaCap / 2;
    bool fold_bg = true;
    hipEvent_t fold_ev = nullptr;  // the old window's last readers (the next fold waits)
    uint64_t folds_started = 0, folds_swapped = 0, folds_inline = 0;
    bool merge_is_fold = false;  // merge_pending for a full delta run (not a new group / wider key)
    float fold_ms = 0;  // build time of the last background fold

    // device window
    int W = 1;
    size_t n = 0, cap = 0;
    uint32_t ntiles = 0;
    int log2T = 11, levels = 0;
    int layout = HSC_LAYOUT_AUTO;  // hsc_set_layout
    bool narrow = false;           // 64-bit codes + 16-ary index (hsc_narrow.hip)
    int lw = 0, tz = 0;  // least significant varying limb / its constant low bits
    bool ncomp = false;  // narrow over compressed codes (NarrowView::comp)
    uint64_t nc0 = 0;
    DBuf d_ncmeta;       // its per-limb masks, patterns, compress moves
    DBuf d_nkeys, d_nmaxs, d_nbase;
    NarrowView nv{};
    // the narrow window as one-word tile rows (codes) for the tile pipeline
    WinView wn{};
    DBuf d_nzero, d_ntmax, d_nsp_g, d_nsp_w, d_ngs, d_nscratch;
    DBuf p_code_lo, p_code_hi, p_zero;
    uint32_t probe_ntiles = 0;  // tiles of the view the last probe ran on
    bool probe_buckets = false; // the last probe ran the narrow tiles (fixed-capacity buckets)
    // narrow tiles: u32 key deltas + commit ranks (dense batches)
    bool ntiles32 = false;
    DBuf d_trad2;  // the other bucket-table mode (narrow_trad_pick)
    DBuf d_commits, d_cdir, d_tdir, d_trad, d_done, w_vflags, d_key32, d_rank32, d_ctmp[4];
    Dir16 cdir{}, tdir{};
    uint32_t trad_m = 0;       // tile bucket table size (0: none)
    bool trad_log = false;     // the table is in log mode (narrow_trad_pick)
    uint32_t ncommit = 0;      // distinct commit LSNs in d_commits (built only for the rank directory)
    bool has_commits = false;  // the window has rows and a commit span (narrow / compact tiles)
    uint64_t commit_span[2] = {0, 0};  // oldest / newest distinct commit LSN of the window
    bool rank_lsn32 = false;   // narrow tiles: rows carry lsn - rank_base + 1 (NarrowTiles)
    uint64_t rank_base = 0;
    DBuf w_tcode, w_tcode2, w_trecs;
    DBuf d_gid, d_words, d_lsn, d_gid2, d_words2, d_lsn2, d_flags, d_scratch;
    DBuf d_pk[2];              // packed-key sort: the keys, ping-pong (hsc_ingest.hip)
    bool packed_sort = false;  // the last build sorted packed keys
    DBuf d_gstart, d_gend, d_tmax, d_table_max, d_group_table, d_count, d_sp_g, d_sp_w;
    uint32_t nt_dev = 0;  // tables whose maxima d_table_max holds (later ones: the pending tail)
    // compact codes of a wide window (hsc_compact.hip): WinView wc over them
    bool compact = false;
    CompactTables ct{};
    WinView wc{};
    DBuf d_cmask, d_cpat, d_cmv, d_cbits, d_cwords, d_ctmax, d_csp_g, d_csp_w;
    // the code sort's tables and keys (device_build: wide rows whose per-group
    // varying bits fit 3 words)
    DBuf d_csrep, d_csmask, d_cspat, d_csmv, d_csbits, d_cskeys[2], d_cssplit;
    bool code_sorted = false;  // the last build sorted by compact codes
    int cs_codes_wc = 0;       // its unpack wrote the distinct rows' codes (d_cwords) of this width
    std::vector<uint64_t> cs_mask;     // its varying bits per (group, word) (host copy)
    std::vector<uint8_t> cs_has_rows;  // its groups with rows
    std::vector<uint32_t> cs_bits_h;   // host sources of its table uploads
    std::vector<uint64_t> cs_mv_h;
    int ct_maxbits = 0;  // most varying bits of any group
    // compact tiles (hsc_ctiles.hip): the compact window as gid || code keys
    bool ctiles = false;
    CTiles ctv{};
    DBuf d_ckey, d_crank, d_cfirst, d_crel, d_ctrad, d_ctb;
    DBuf d_cph;               // the tiles' point index (PointHash), cph_nb buckets
    uint64_t cph_nb = 0;
    uint32_t cph_ep = 0;      // its epoch (1..2^24-1; 0 = the buffer was never cleared)

    // probe workspace
    DBuf p_lo, p_hi, p_gid, p_snap, p_txn, p_lock_table, p_lock_snap, p_lock_txn;
    DBuf p_arena;  // a staged batch's columns, uploaded in one copy (StageLayout)
    DBuf p_verdict, p_bitmap;
    DBuf w_code, w_hist, w_counts, w_bucket, w_cursor, w_items, w_item_tile, w_item_desc, w_recs;

    // marshal output: staging sets (two: a large batch is checked as a
    // pipeline of chunks, one marshalled while the other is on the GPU),
    // per-worker parts, host threads
    hsc_marshalled m{};
    Stage stage[2];
    // the drop-in entry's own collector (hsc_set_autocollect), created at the
    // first collected call
    std::atomic<int> autocollect{1};
    std::atomic<hsc_collector *> auto_col{nullptr};
    std::vector<MarshalPart> parts;
    std::vector<std::vector<uint8_t>> parts_cls;  // per part: probe class (length, point) in marshal_into
    int threads = 1;
    std::unique_ptr<WorkPool> pool;  // `threads` workers (created by the first parallel marshal)

    // raw log / wire decode output
    DecodedLog decoded;
    PhysStore phys;  // records key reconstruction walks may visit (hsc_logdec.cpp)
    DecodedReadSets wire;

    // rw conflict pairs: every window version (pre-dedupe rows in d_*2)
    size_t n_all = 0;
    DBuf e_span, e_cnt, e_txn, e_lsn, e_txn2, e_lsn2, e_gid, e_scratch, e_flags, e_after;
    std::vector<uint32_t> e_out_txn;
    std::vector<uint64_t> e_out_lsn;
    const uint32_t *e_dev_txn = nullptr;  // the last hsc_rw_edges pairs, on the device
    const uint64_t *e_dev_lsn = nullptr;
    size_t e_dev_n = 0;

    // replicant coalesce: device inputs / working arrays, host outputs
    DBuf co_dev[25];
    std::vector<int64_t> co_off;
    std::vector<int32_t> co_i32[7];
    std::vector<uint64_t> co_u64[2];

    // dependency graph
    GraphBufs graph;
    GraphBufs subgraph;  // the graph induced on a cover (sharded SCC)
    uint32_t graph_ntxn = 0;
    uint32_t x_max_txn = 0;  // largest txn id a staged rw pair can name (stage_rw_pairs)

    // Probe lanes: the probe scratch above belongs to the active lane; other
    // lanes park theirs here.  A lane is bound to the stream that last used
    // it, so batches on different streams never share scratch and can run
    // concurrently; a lane taken over by another stream first waits for the
    // lane's last batch (its done event).
    // The done event is recorded when the context leaves the lane's stream
    // (hsc_set_stream, the multi context's member probes), not after every
    // batch: batches on one stream are ordered by it, and a record per batch
    // cost a one-stream config-2 batch 3 us (r05ab: 0.683 -> 0.718 of peak).
    // pend: batches on the stream since the last record.
    struct Lane {
        DBuf b[20];
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint64_t tick = 0;
        bool pend = false;
    };
    static constexpr int kLanes = 4;
    Lane lanes[kLanes];
    int lane = 0;
    uint64_t lane_tick = 0;

    // small batches (k_small_narrow): a ring of slots, each with the probe
    // columns, verdict bytes and done word in fine-grained pinned memory and
    // its own block counter.  A slot belongs to one call from its launch
    // (under mu) until that call has read its verdicts (without mu), so a
    // second call can marshal and launch while the first one's kernel runs.
    static constexpr int kSmallSlots = 8;
    struct SmallSlot {
        HBuf io;
        std::vector<uint8_t> forced;
        size_t n_txn = 0, vo = 0, dn = 0;
        uint32_t seq = 0;
        hipStream_t stream = nullptr;  // the stream its kernel was launched on
        hipEvent_t wait_ev = nullptr;  // the stream waits on it before the launch (appends)
        // the launch's arguments, captured under c->mu (the launch itself is
        // issued after the lock is dropped: small_fire)
        NarrowView nv{};
        DeltaView d{}, d2{};
        PendView pd{};
        ProbeView p{};
        std::atomic<bool> busy{false};
    };
    SmallSlot small[kSmallSlots];
    // Small batches run on side streams of their own, one per slot, so that
    // concurrent ones overlap on the device instead of queueing behind each
    // other on c->stream.  What they read of the window is complete when they
    // launch -- builds, folds and table-maxima uploads synchronize -- except
    // an append's merge / upload, so a slot's stream waits on app_last once
    // per append (app_seq); every window change waits on the host until no
    // slot is in flight (wait_small), so a kernel never overlaps a change.
    hipStream_t small_side[kSmallSlots] = {};
    uint64_t small_app_seq[kSmallSlots] = {};
    uint64_t app_seq = 0;  // appends whose device work app_last follows
    Stage small_st;  // marshal target of the small path (coh: its arena swaps into a slot)
    // collector batches assembled from premarshalled rows before the context
    // lock (check_batch_assembled): a stage per batch in flight
    std::mutex pre_mu;
    std::vector<std::unique_ptr<Stage>> pre_stages;
    std::vector<Stage *> pre_free;
    DBuf small_blocks;
    bool small_blocks_zeroed = false;
    bool no_small = false;  // hsc_set_paths(HSC_PATH_NO_SMALL): the staged path
    unsigned paths = 0;     // hsc_set_paths flags (tests, A/B)
    uint32_t small_seq = 0;
    // small-path phase times (hsc_small_stats)
    // marshal / batch phase totals (hsc_batch_stats)
    std::atomic<uint64_t> mb_marshals{0}, mb_txns{0}, mb_ranges{0}, mb_parts_ns{0}, mb_alloc_ns{0},
        mb_assemble_ns{0}, mb_launch_ns{0}, mb_wait_ns{0};
    std::atomic<uint64_t> sm_calls{0}, sm_marshal_ns{0}, sm_launch_ns{0}, sm_wait_ns{0},
        sm_slot_waits{0}, sm_lock_ns{0};

    // timing
    bool timing = false;
    hipEvent_t ev[8] = {};
    hsc_timing last{};
};

namespace hsc {
// hsc_host.cpp internals the multi-GPU context (hsc_multi.cpp) drives its
// member contexts with
int ctx_fail(hsc_ctx *c, int code, const char *what, hipError_t e = hipSuccess);
int ctx_window_words(hsc_ctx *c);
void ctx_clear_window(hsc_ctx *c);
int ctx_ensure_built(hsc_ctx *c);
void ctx_add_write(hsc_ctx *c, int tid, int ix, const uint8_t *key, int keylen, bool has_key, uint64_t lsn);
int ctx_flush_appends(hsc_ctx *c, bool lazy = false);
void ctx_raise_table_max(hsc_ctx *c, int tid, uint64_t lsn);
int ctx_probe(hsc_ctx *c, const hsc_probe_batch *b);
// c->stream := s, the active lane's batches on the stream left fenced by its
// done event first (callers hold c->mu)
hipError_t ctx_switch_stream(hsc_ctx *c, hipStream_t s);
int ctx_default_threads();
void ctx_par_for(hsc_ctx *c, int nwork, const std::function<void(int)> &f);
bool ctx_small_fits(hsc_ctx *c, size_t n_txn, size_t n, size_t n_lock);
int ctx_edge_keys(hsc_ctx *c, uint32_t *gid, uint64_t *words);
// op_txn: the last build's ops' txn array when still live (the op-range cut)
int ctx_graph_cut(hsc_ctx *c, const uint8_t *cover, size_t *m, const uint64_t **rows,
                  const uint32_t *op_txn = nullptr, const uint64_t *op_key = nullptr,
                  const uint8_t *op_isw = nullptr);
int ctx_stage_launch(hsc_ctx *c, Stage &st, int *slot);
int ctx_stage_wait(hsc_ctx *c, Stage &st, int slot, int *rc_out);
bool multi_adopted(const hsc_ctx *f);
// hsc_multi.cpp: the front context's hooks (c->multi != nullptr)
int multi_build(hsc_ctx *f);
int multi_flush_appends(hsc_ctx *f, bool lazy);
// lk (may be null): the caller's hold on f->mu; released while the members'
// small kernels run when every member of the batch took that path
int multi_check_stage(hsc_ctx *f, Stage &st, int *rc_out, std::unique_lock<std::mutex> *lk = nullptr);
void multi_sync_dict(hsc_ctx *f);
void multi_destroy(hsc_ctx *f);

// Publish the regop_only inputs (caller holds c->mu; the only writer).
inline void ctx_publish_regop(hsc_ctx *c)
{
    const uint64_t s = c->rg_seq.load(std::memory_order_relaxed);
    c->rg_seq.store(s + 1, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    c->rg_end.store(c->end_lsn, std::memory_order_relaxed);
    c->rg_max.store(c->max_commit, std::memory_order_relaxed);
    c->rg_poison.store(c->poison_regop, std::memory_order_relaxed);
    c->rg_lgrule.store(c->lg_rule ? 1u : 0u, std::memory_order_relaxed);
    c->rg_seq.store(s + 2, std::memory_order_release);
}

// The published (end, max commit, poison, lg_rule), consistent with each other.
inline void ctx_read_regop(const hsc_ctx *c, uint64_t *end, uint64_t *mx, uint64_t *po, uint32_t *lg)
{
    for (;;) {
        const uint64_t s1 = c->rg_seq.load(std::memory_order_acquire);
        if (s1 & 1) {
            __builtin_ia32_pause();
            continue;
        }
        *end = c->rg_end.load(std::memory_order_relaxed);
        *mx = c->rg_max.load(std::memory_order_relaxed);
        *po = c->rg_poison.load(std::memory_order_relaxed);
        *lg = c->rg_lgrule.load(std::memory_order_relaxed);
        std::atomic_thread_fence(std::memory_order_acquire);
        if (c->rg_seq.load(std::memory_order_relaxed) == s1) return;
    }
}

// regop_only (bdb/serializable.c:382-416, 531-534) without mu: S at or past
// the end -> 0 (DB_SET finds nothing); a committed write txn (or an
// unreadable regop) after S -> 1, whether or not S is a record LSN; else 0,
// unless the DB_SET-on-a-non-record rule needs the log's record LSNs: -1
// (the caller takes mu and answers from the log).
inline int ctx_regop_fast(const hsc_ctx *c, uint64_t S)
{
    uint64_t end, mx, po;
    uint32_t lg;
    ctx_read_regop(c, &end, &mx, &po, &lg);
    if (S >= end) return 0;
    if (mx > S || po > S) return 1;
    return lg ? -1 : 0;
}

// std::lock_guard on c->mu for the entries that change the window: the
// regop_only snapshot is republished before mu is released.
class MuGuard {
  public:
    explicit MuGuard(hsc_ctx *c) : c_(c), g_(c->mu) {}
    ~MuGuard() { ctx_publish_regop(c_); }
    MuGuard(const MuGuard &) = delete;
    MuGuard &operator=(const MuGuard &) = delete;

  private:
    hsc_ctx *c_;
    std::lock_guard<std::mutex> g_;
};
}  // namespace hsc
