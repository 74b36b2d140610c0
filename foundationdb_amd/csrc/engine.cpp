// engine.cpp — host side of the MI355X conflict-resolution engine and its C-ABI
// (include/fdb_conflict_set.h).
//
// Mirrors the reference ConflictSet / ConflictBatch lifecycle (fdbserver/SkipList.cpp:730-890):
// addTransaction packs each transaction's conflict ranges into flat SoA buffers of normalized
// key prefixes plus a tail arena; detectConflicts uploads the batch with one pinned H2D copy,
// enqueues the kernel pipeline on the set's stream, and copies back one verdict byte per
// transaction.  No CPU fallback exists: without a usable HIP device every entry point fails.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <cxxabi.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/fdb_conflict_set.h"
#include "engine.h"

using namespace fdbcs;

#define HIPOK(expr)                                                                                   \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess) {                                                                       \
            fprintf(stderr, "fdbcs: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(_e), __FILE__, \
                    __LINE__);                                                                        \
            return FDBCS_E_DEVICE;                                                                    \
        }                                                                                             \
    } while (0)

// Base-tier size from which the read check splits by default (FDBCS_SPLIT_CHECK=2).
constexpr int64_t kSplitCheckMinBase = 16 << 20;

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr int64_t kTailSlack = 64;  // bytes past a tail arena's capacity (dkey.h tail_word reads aligned words)
// History tails are 8-byte aligned and addressed in 8-byte units by the uint32 Hist::lt.y: the
// arena holds up to 32 GiB of tail bytes per conflict set (detect refuses a batch past that).
constexpr int64_t kTailLimit = (int64_t)8 << 32;
constexpr int64_t kTailReclaimDefault = kTailLimit / 2;  // force the GC repack past half of that

// Grow-only device allocation.
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return FDBCS_OK;
        size_t want = std::max(bytes, cap + cap / 2);
        want = align_up(want < 256 ? 256 : want, 256);
        if (p) HIPOK(hipFree(p));
        p = nullptr;
        cap = 0;
        HIPOK(hipMalloc(&p, want));
        cap = want;
        return FDBCS_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Grow-only pinned host allocation; `mapped` buffers are fine-grained and written by kernels directly.
struct HBuf {
    void* p = nullptr;
    void* dp = nullptr;  // device view (mapped buffers)
    size_t cap = 0;
    int ensure(size_t bytes, bool mapped = false, bool noncoherent = false) {
        if (bytes <= cap) return FDBCS_OK;
        size_t want = align_up(std::max(bytes, cap + cap / 2), 4096);
        if (p) HIPOK(hipHostFree(p));
        p = dp = nullptr;
        cap = 0;
        const unsigned fl = !mapped ? hipHostMallocDefault
                                    : (hipHostMallocMapped | (noncoherent ? hipHostMallocNonCoherent : hipHostMallocCoherent));
        HIPOK(hipHostMalloc(&p, want, fl));
        if (mapped) HIPOK(hipHostGetDevicePointer(&dp, p, 0));
        cap = want;
        return FDBCS_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = dp = nullptr;
        cap = 0;
    }
};

enum Phase {
    kPhStart, kPhUpload, kPhSort, kPhEdges, kPhCheck, kPhIntra, kPhCombine, kPhCopyBegin, kPhCopyEnd, kPhMerge,
    kPhCompBegin, kPhCompEnd, kPhCompact, kPhGc, kPhEpilogue, kPhEnd,
    kPhCheckBegin, kPhCheckEnd, kPhSortBegin, kPhSortEnd, kPhCount
};

}  // namespace

struct fdbcs_batch;
struct BatchSlot;

// ws[k] slots: ensure_workspace TAKEs [0, kWsTileSlot); then the copy-tile index and the scan arena.
constexpr int kWsTileSlot = 54, kWsArenaSlot = 55;
// Batch workspaces in rotation: stage A can run up to two batches ahead of stage B, so each
// workspace is reused every third batch.
constexpr int kNumWork = 3;
constexpr int kGcEveryCompactions = 4;  // removeBefore cadence of size-triggered compactions

// FDBCS_HOST_TRACE=<path>: host-side spans of the pipeline (steady_clock ns, the clock rocprofv3
// timestamps use), written as CSV when the set is destroyed: per batch sequence number the detect
// call (D), the helper's issue of stage A (A) and of a Y half (Y), the calling thread's issue of an
// X half (X) and the wait for the completion flag (W).  scripts/host_trace.py joins them with a
// rocprofv3 kernel trace: when each chain's launches were issued against when they ran.
struct HSpan {
    uint32_t seq;
    char kind;
    int64_t t0, t1;
};
inline int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Host threads for addTransaction of whole batches (fdbcs_batch_add_packed): the endpoint keys'
// validation and normalization into pinned staging split over chunks of transactions.  The
// calling thread works too.  A ticket carries the job's generation, so a worker that wakes late
// never takes a ticket of a later job with the earlier job's function.  Between jobs a worker
// sleeps on the condition variable (spinning ~300 us for the next job measured no better:
// DESIGN.md §5).
struct AddPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv;
    std::atomic<uint64_t> ticket{0};  // generation << 32 | next ticket
    std::atomic<int> done{0};         // tickets finished in the current generation
    std::atomic<uint32_t> gen{0};
    std::atomic<int> sleepers{0};
    int n = 0;
    const std::function<void(int)>* job = nullptr;
    bool stop = false;

    // std::thread's constructor throws (std::system_error) at the process's thread limit: the
    // workers already started are stopped and joined before the exception leaves, so the caller
    // can fall back to the serial loop
    explicit AddPool(int workers) {
        try {
            for (int i = 0; i < workers; i++) th.emplace_back([this] { worker(); });
        } catch (...) {
            shutdown();
            throw;
        }
    }
    ~AddPool() { shutdown(); }
    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
            gen.fetch_add(1);
        }
        cv.notify_all();
        for (auto& t : th)
            if (t.joinable()) t.join();
    }
    void run(uint32_t g, int nn, const std::function<void(int)>* fn) {
        uint64_t cur = ticket.load(std::memory_order_acquire);
        for (;;) {
            if ((uint32_t)(cur >> 32) != g || (int)(cur & 0xffffffffu) >= nn) return;
            if (ticket.compare_exchange_weak(cur, cur + 1, std::memory_order_acq_rel)) {
                (*fn)((int)(cur & 0xffffffffu));
                done.fetch_add(1, std::memory_order_acq_rel);
                cur = ticket.load(std::memory_order_acquire);
            }
        }
    }
    void worker() {
        uint32_t seen = 0;
        for (;;) {
            uint32_t g;
            int nn;
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> lk(m);
                if (gen.load(std::memory_order_relaxed) == seen && !stop) {
                    sleepers.fetch_add(1);
                    cv.wait(lk, [&] { return stop || gen.load(std::memory_order_relaxed) != seen; });
                    sleepers.fetch_sub(1);
                }
                if (stop) return;
                seen = g = gen.load(std::memory_order_relaxed);
                nn = n;
                fn = job;
            }
            run(g, nn, fn);
        }
    }
    // fn(c) for c in [0, tickets), in ticket order across the workers and the calling thread;
    // returns when all are done.
    void parallel_for(int tickets, const std::function<void(int)>& fn) {
        uint32_t g;
        {
            std::lock_guard<std::mutex> lk(m);
            g = gen.load(std::memory_order_relaxed) + 1;
            n = tickets;
            job = &fn;
            done.store(0, std::memory_order_relaxed);
            ticket.store((uint64_t)g << 32, std::memory_order_release);
            gen.store(g, std::memory_order_release);
        }
        if (sleepers.load(std::memory_order_acquire) > 0) cv.notify_all();
        run(g, tickets, &fn);
        while (done.load(std::memory_order_acquire) < tickets) __builtin_ia32_pause();
    }
};

struct fdbcs_conflict_set {
    int device = 0;
    hipStream_t stream = nullptr;   // stage B: everything that reads or writes the history, in batch order
    hipStream_t astream = nullptr;  // stage A (and every upload): history-independent sort and edges
    hipStream_t cstream = nullptr;  // split read check: the base-tier half (history-independent between
                                    // compactions) beside stage A
    hipEvent_t ev_c[kNumWork] = {}; // base-tier check of the batch using workspace k is done
    hipEvent_t ev_cmp = nullptr;    // stage B of the last batch that rewrote the base (compaction / GC)
    bool cmp_recorded = false;
    // FDBCS_SPLIT_CHECK: 0 = one read check over both tiers in stage B, 1 = the base-tier half on
    // its own stream beside stage A, 2 (default) = split only over a large base tier (>= 16M
    // boundaries): there the base check is long (C4: ~150 us) and must leave the batch-order
    // chain; over a 5M base (C2) the single launch measured faster (device-resident 34.0M vs
    // 32.1M txns/s: one launch and two cross-stream events fewer, no third stream competing)
    int split_check = 2;
    hipStream_t ustream = nullptr;  // batch uploads (k_upload over PCIe), so batch i+1's upload overlaps
                                    // batch i's stage A; stage A waits for the upload's event
    hipEvent_t ev_a[kNumWork] = {}; // stage A of the batch using workspace k is done
    hipEvent_t ev_b[kNumWork] = {}; // stage B (epilogue) of the batch using workspace k is done
    // Stage B in two halves on two streams: X (`stream`: read check, resolution, D.Combine) and Y
    // (`ystream`: merge into the delta, compaction / GC, epilogue).  The check of batch i + 1 runs
    // against the delta before batch i's merge plus batch i's union segments (PrevSegs), so it does
    // not wait for that merge: Y(i) overlaps X(i + 1).
    hipStream_t ystream = nullptr;
    hipEvent_t ev_res[kNumWork] = {};   // X of the batch using workspace k is done (Y waits for it)
    // the next batch's check is done with workspace k's segments: that batch's ev_res (the end of
    // its half X, recorded anyway, and not re-recorded before workspace k's next user records)
    hipEvent_t xfree_ev[kNumWork] = {};
    bool prev_segs = false;             // the last batch's segments are not merged when the next check runs
    int prev_wp = 0;
    int64_t prev_now = 0;
    int last_wp = -1, prev2_wp = -1;    // workspaces of the last two batches submitted (their Y events)
    bool xfree_rec[kNumWork] = {};      // xfree_ev[k] set since workspace k's last use
    // The batches behind ws ev_b[k] (workspace k's last user) and xfree_ev[k] (the batch whose check
    // reads workspace k's segments), or null once destroyed: while a batch lives its completion
    // flag tells whether its stages are done, one load from host-mapped memory instead of an event
    // query (a runtime call) per dependency per batch.
    fdbcs_batch* ws_user[kNumWork] = {};
    fdbcs_batch* xfree_user[kNumWork] = {};
    bool y_async[kNumWork] = {};        // Y of workspace k's last batch ran on ystream (not in `stream` order)
    bool wused[kNumWork] = {};
    int wpar = 0;                   // workspace of the next batch
    int timing = 0;       // 0: no events; 1: the copy kernels; 2: every phase (fdbcs_set_timing)
    uint32_t seq = 0;     // batches submitted (completion flag values)
    int64_t oldest = 0;          // ConflictSet::oldestVersion (SkipList.cpp:736)
    int64_t header_version = 0;  // SkipList(Version) header (SkipList.cpp:398-404)
    int64_t max_written = 0;     // highest version present in the history
    int gc_interval = 0;          // compaction (and GC) at least every this many batches; 0: by size only
    int batches_since_compact = 0;
    int compactions_since_gc = 0;
    int64_t gc_applied = 0;
    int64_t delta_limit = 0;      // compaction once the delta may exceed this; 0: automatic

    // base tier: two buffer sets (ping-pong) + range-max levels
    DBuf hkey[2], hlt[2], hver[2];
    DBuf lvl[kMaxLevels];  // lvl[0]: sampled key index (the level-0 versions are hver[cur])
    DBuf dir;              // radix directory over the base tier's level-0 samples (k_directory)
    DBuf edir[2];          // each delta buffer's directory (epoch-tagged entries, filled by k_epilogue)
    uint32_t ddir_epoch[2] = {0, 0};  // epoch of each delta buffer's directory (0: none)
    uint32_t ddir_counter = 0;  // last epoch handed out
    int cur = 0;
    int64_t hist_cap = 0;  // elements per buffer set
    int64_t n_ub = 0;      // upper bound of live base boundaries (exact after a wait)
    int64_t lvl3_n = 0;
    int64_t lvl2_n = 0;
    // delta tier: the same layout, small
    DBuf dkey[2], dlt[2], dver[2];
    DBuf dlvl[2][kMaxLevels];  // per delta buffer: the next batch's check reads one while the epilogue builds the other
    int dcur = 0;
    int64_t delta_cap = 0;
    int64_t nd_ub = 0;
    int64_t dlvl3_n = 0;
    int64_t dlvl2_n = 0;
    DBuf cws[6];  // compaction arrays (per delta boundary)
    DBuf htail[2];  // tail arenas (bytes [16, len) of long keys): append-only between GCs; each GC
    int tcur = 0;   // repacks the live tails into the other one, reclaiming the rest
    int64_t tail_ub = 0;
    int64_t tail_cap = 0;
    DBuf scal;  // Scalars
    int64_t route_timeout_ms = 60000;  // FDBCS_ROUTE_TIMEOUT_MS: bound of a routed batch's wait for its shares
    DBuf route_btail;                  // device routing: tails of this resolver's key-range bounds
    std::vector<uint8_t> route_bounds; // the bounds route_btail holds (lo | hi bytes), to skip re-uploads
    // batch workspaces (rotating)
    DBuf ws[kNumWork][56];  // [0, kWsScanSlot): TAKE slots of ensure_workspace
    DBuf wbtail[kNumWork];  // Work::btail of each workspace (ensure_btail)
    int64_t ws_T = -1, ws_R = -1, ws_W = -1;
    Work work[kNumWork]{};
    int64_t edge_cap = 0;

    int inflight = 0;
    bool validate = false;  // FDBCS_VALIDATE=1: device-side invariant checks (tests)
    int bucket_target = 0;  // FDBCS_SORT_BUCKET: endpoints per sort bucket on average (0 = kSortTarget)
    bool sort_cold = false; // FDBCS_SORT_COLD=1: splitters from every batch's own samples (tests)
    DBuf quant;             // the sort's splitter source, two tables: quantiles of the last batch of
    int qcur = 0;           // >= kQuantMinE endpoints in table qcur; the next such batch writes the other
    bool quant_valid = false;
    // the stream of the last stage A (its sort read one splitter table and wrote the other): a batch
    // whose stage A runs on another stream (a timing-level change) waits for ev_quant recorded there
    hipStream_t quant_sa = nullptr;
    hipEvent_t ev_quant = nullptr;
    int64_t sort_big_buckets = 0;  // buckets past kSlab so far (host view, from the published scalars)
    bool trace = false;     // FDBCS_TRACE=1: device timestamps of kernel sections printed per batch
    bool serial = false;    // FDBCS_SERIAL=1: both stages on one stream (no cross-batch overlap)
    bool no_prepass = false;  // FDBCS_RESOLVE_PREPASS=0: k_resolve without its pre-pass (tests)
    int64_t tail_reclaim = kTailReclaimDefault;  // FDBCS_TAIL_RECLAIM: tail bytes that force the GC repack
    bool write_groups = true;  // FDBCS_WRITE_GROUPS=0: one candidate edge per (read, writer) pair (A/B)
    bool directory = true;  // FDBCS_DIRECTORY=0: base-tier lookups descend the whole sample tree (A/B)
    // Directory code (MaxLevels::dir_p .. dir_w; set_dir_map): the loaded keys' common prefix
    // (capped at 15) and the value range of each byte position after it, as many positions as fit
    // the slot budget (dir_bits).  Keys written later outside the loaded values take neighbouring
    // codes, so the mapping stays monotone.  (Round 4's directory on the first two key bytes, and
    // its prefix-only variant, are the special cases this code replaced: DESIGN.md §5.)
    uint32_t dir_p = 0;
    uint64_t dir_phi = 0, dir_plo = 0;
    uint32_t dir_e = 0, dir_top = 0;
    uint32_t dir_pos[kDirPos] = {}, dir_w[kDirPos] = {};
    // FDBCS_DIR_BITS: slot budget 2^bits.  0 (default): 2^16, doubled while the base has over
    // eight level-0 samples per slot (C4: 2^17; a slot of up to 16 samples is counted directly).
    // A directory is read cold by every batch's check, so a larger one costs cache misses: C2's
    // isolated check 11.0 us at 2^16, 16.4 at 2^18; C4's 57.3 at 2^17, 62 at 2^19 and 2^20, 64 on
    // the first two bytes.
    int dir_bits = 0;
    DBuf trace_buf;
    // Per-kernel device time (fdbcs_kernel_profile): launches and milliseconds by kernel, from the
    // events of timing level 3 (every kernel) or of the timed kernel at level 1.
    struct KProf {
        const void* func;
        int64_t launches;
        double ms;
    };
    std::vector<KProf> kprof;
    const void* timed_func = nullptr;  // fdbcs_set_timed_kernel
    HBuf hold;                         // fdbcs_debug_hold: host-mapped release word of the hold kernels
    HBuf hedge;                        // per workspace {batch seq, any candidate edge} (Work::hedge)
    bool skip_edges = true;            // FDBCS_SKIP_EDGES=0: always issue the kGroupEdges launches
    fdbcs_stats stats{};
    std::vector<BatchSlot*> pool;  // staging slots of destroyed batches, reused by new ones
    // Two submitting threads (the default since round 4: C2 +3-10 % over five same-box A/Bs, C3 and
    // C4 unchanged; FDBCS_SUBMIT_THREAD=0 keeps one).  A helper thread issues stage A of batch i
    // (and its base-tier check) while the calling thread issues stage B's X half of batch i-1,
    // which waited for this call; the helper then issues that batch's Y half once X is out:
    // kernel launches on two streams from two threads take about half the wall time of one
    // thread's (tools/threadbench.hip: 3.4 -> 1.85 us per launch).  The
    // check of batch i waits (host side) until stage B of batch i-1 is issued, because it may wait
    // on that stage's compaction event; stage B of batch i waits for the helper to go idle.
    bool submit_thread = true;
    // addTransaction threads (FDBCS_ADD_THREADS, workers besides the calling thread; 0 = serial)
    int add_threads = 5;
    AddPool* add_pool = nullptr;
    int wait_query_ms = 2;  // FDBCS_WAIT_QUERY_MS: stream error checks while a wait spins (0: every 4096 spins)
    // FDBCS_HOST_TRACE: spans of the calling thread [0] and of the helper [1]
    bool htrace = false;
    std::vector<HSpan> htr[2];
    uint32_t work_a_seq = 0, work_y_seq = 0;
    double add_prof[4] = {0, 0, 0, 0};  // FDBCS_ADD_PROFILE: ms in add's serial pass, slot, count, fill
    int64_t add_prof_n = 0;
    std::thread worker;
    std::mutex wmu;
    std::condition_variable wcv;
    std::atomic<int> wjob{0};           // 0 idle, 1 job queued or running, 2 exit
    std::atomic<uint32_t> b_issued{0};  // stage-B lists issued (their Y halves: helper or flush)
    uint32_t b_recorded = 0;            // stage-B lists recorded
    std::atomic<int> werr{0};           // first HIP error of the helper
    LaunchList work_a, work_c;          // the helper's lists
    hipStream_t work_sa = nullptr;
    uint32_t work_need_b = 0;           // the check goes out once b_issued >= this
    // Stage B's Y half of the previous batch, issued by the helper once the calling thread has
    // issued its X half.  The calling thread issues record + X, the helper stage A + Y + base
    // check: their runtime calls split about evenly instead of ~2:1.
    LaunchList work_y;
    hipStream_t work_ys = nullptr;
    uint32_t work_need_x = 0;            // Y goes out once x_issued >= this
    std::atomic<uint32_t> x_issued{0};   // stage-B X lists issued (calling thread)
    fdbcs_batch* work_y_batch = nullptr; // whose Y the helper holds (calling thread's view)
    LaunchList rec_a, rec_b, rec_c, rec_y, pending_b, pending_y;
    hipStream_t pending_ys = nullptr;  // the stream of pending_y
    fdbcs_batch* pending_batch = nullptr;
    std::unordered_set<fdbcs_batch*> live;  // batches not yet destroyed (detached if the set goes first)
};

// Host/device staging of one batch.  Batches are short-lived (one per commit batch, as the
// reference's ConflictBatch), so their pinned and device buffers come from a per-set pool instead
// of fresh hipHostMalloc / hipMalloc calls.  A slot goes back to the pool only when its batch is
// destroyed, after its completion flag was seen (the epilogue's last store) or, for a batch still
// in flight, after its streams were synchronized: the next user's upload needs no event.
struct BatchSlot {
    DBuf dev;
    HBuf pin_in;
    HBuf pin_out;
    DBuf dverdict;
    hipEvent_t ev[kPhCount] = {};
    bool events_made = false;
    hipEvent_t ev_up = nullptr;    // upload done (recorded on stage A's stream)
    HBuf pin_inv;  // fdbcs_batch_set_conflict_output: global -> batch transaction map (host-mapped)
    // device routing (fdbcs_batch_add_routed): scan state, global -> batch map, read ids, totals
    DBuf rt_scan, rt_inv, rt_rids, rt_dres, rt_info, rt_txpre;
    HBuf rt_res;
    hipEvent_t ev_rt0 = nullptr, ev_rt1 = nullptr;  // around the routing kernels
    bool rt_timed = false;
    // per-kernel events of the batch (timing level 3, or the timed kernel at level 1)
    std::vector<hipEvent_t> prof_pool;
    size_t prof_next = 0;
    std::vector<std::pair<const void*, std::pair<hipEvent_t, hipEvent_t>>> prof_spans;
    LaunchList::Profile prof{&prof_pool, &prof_next, &prof_spans};
};

struct fdbcs_batch {
    fdbcs_conflict_set* cs = nullptr;
    BatchSlot* slot = nullptr;
    int report_enabled = 0;
    int state = 0;  // 0 adding, 1 uploaded, 2 submitted, 3 done
    // host staging (pageable); in `direct` mode (one fdbcs_batch_add_packed) the endpoint keys,
    // owners and tails were normalized straight into slot->pin_in at add time
    std::vector<int64_t> snap;
    std::vector<uint8_t> flags;
    std::vector<int32_t> roff{0}, woff{0};
    std::vector<int32_t> rowner, wowner;
    std::vector<DKey> rkeys, wkeys;
    std::vector<uint8_t> tail;
    bool direct = false;
    size_t d_keys = 0, d_rown = 0, d_wown = 0, d_tail = 0, d_small = 0;  // pin_in offsets (direct mode)
    size_t d_tail_bytes = 0;
    // device copy
    BatchDev bd{};
    size_t tail_bytes = 0;
    // results
    uint8_t* h_verdict = nullptr;
    Scalars* h_scal = nullptr;
    uint8_t* h_rconf = nullptr;
    uint8_t* h_hist = nullptr;
    int32_t* h_first = nullptr;
    bool gc_ran = false;
    bool compacted = false;
    uint32_t seq = 0;
    volatile uint32_t* h_flag = nullptr;
    int64_t n_report = 0;  // transactions added with report_conflicting_keys (and reports enabled)
    uint32_t recorded = 0;  // phases whose events were recorded (bit per Phase)
    bool any_report = false;
    int64_t check_hist = 0;  // boundaries (both tiers, upper bound) the read check searched
    std::vector<int32_t> out_ids;  // fdbcs_batch_set_conflict_output: global index per transaction
    int64_t out_n = 0;
    uint8_t* out_dev = nullptr;
    int wp = 0;           // the workspace this batch's detect used
    int32_t max_len = 0;  // longest key added (the sort stages tail windows only past kSortNxLen)
    int64_t wtail = 0;       // history tail bytes the batch's write endpoints could add (8-byte padded)
    std::vector<int32_t> conf_off, conf_idx;
    int32_t n_committed = 0, n_too_old = 0;

    // device-routed batch (fdbcs_batch_add_routed): sizes known once the route kernels finished
    bool routed = false, route_pending = false;
    int32_t rT = 0, rR = 0, rW = 0;
    size_t r_tail = 0;

    int32_t T() const { return routed ? rT : (int32_t)snap.size(); }
    int32_t R() const { return routed ? rR : roff.back(); }
    int32_t W() const { return routed ? rW : woff.back(); }
    size_t tail_size() const { return routed ? r_tail : direct ? d_tail_bytes : tail.size(); }
};

namespace {

void add_key(fdbcs_batch* b, std::vector<DKey>& out, const uint8_t* p, int32_t len) {
    DKey k;
    dkey_prefix(p, (uint32_t)len, &k.hi, &k.lo);
    k.len = (uint32_t)len;
    k.tail = 0;
    if (len > b->max_len) b->max_len = len;
    if (len > 16) {
        k.tail = (uint32_t)b->tail.size();
        b->tail.insert(b->tail.end(), p + 16, p + len);
    }
    out.push_back(k);
}

int cmp_bytes(const uint8_t* a, int32_t al, const uint8_t* b, int32_t bl) {
    int c = memcmp(a, b, (size_t)std::min(al, bl));
    if (c) return c;
    return (al > bl) - (al < bl);
}

// Scan arena for the current workspace shape and history capacity (zeroed per batch by k_prepare).
int ensure_scan_arena(fdbcs_conflict_set* cs) {
    if (cs->ws_T < 0 || cs->hist_cap <= 0) return FDBCS_OK;
    if (cs->delta_cap <= 0) return FDBCS_OK;
    const int64_t words = scan_arena_words(cs->ws_T, cs->ws_R, cs->ws_W, cs->hist_cap, cs->delta_cap);
    for (int k = 0; k < kNumWork; k++) {
        Work& w = cs->work[k];
        int rc = cs->ws[k][kWsArenaSlot].ensure(8 * words + 64);
        if (rc) return rc;
        w.scan_arena = (uint64_t*)cs->ws[k][kWsArenaSlot].p;
        if ((rc = cs->ws[k][kWsTileSlot].ensure(4 * (std::max(cs->hist_cap, cs->delta_cap) / 256 + 8)))) return rc;
        w.tile_first = (int32_t*)cs->ws[k][kWsTileSlot].p;
        carve_scans(w, cs->ws_T, cs->ws_R, cs->ws_W, cs->hist_cap, cs->delta_cap);
        HIPOK(hipMemsetAsync(w.scan_arena, 0, 8 * w.scan_words, cs->stream));
        for (int q = 0; q < kNumScans; q++) w.scan[q].error = &w.bsc->debug_error;
    }
    HIPOK(hipStreamSynchronize(cs->stream));
    return FDBCS_OK;
}

int flush_pending(fdbcs_conflict_set* cs);

// Both streams idle (before reallocating anything either stage uses).
int sync_all(fdbcs_conflict_set* cs) {
    if (int rc = flush_pending(cs)) return rc;
    HIPOK(hipStreamSynchronize(cs->ustream));
    HIPOK(hipStreamSynchronize(cs->cstream));
    HIPOK(hipStreamSynchronize(cs->astream));
    HIPOK(hipStreamSynchronize(cs->stream));
    HIPOK(hipStreamSynchronize(cs->ystream));
    cs->prev_segs = false;  // everything submitted is merged: the next check reads the current delta
    return FDBCS_OK;
}

// Each workspace's copy of a batch tail region (Work::btail) for `bytes`.
int ensure_btail(fdbcs_conflict_set* cs, int64_t bytes) {
    const size_t need = (size_t)bytes + 64;
    if (cs->wbtail[0].p && need <= cs->wbtail[0].cap) return FDBCS_OK;
    if (int rc = sync_all(cs)) return rc;
    for (int k = 0; k < kNumWork; k++) {
        if (int rc = cs->wbtail[k].ensure(std::max<size_t>(need, 1 << 16))) return rc;
        cs->work[k].btail = (uint8_t*)cs->wbtail[k].p;
    }
    return FDBCS_OK;
}

// Workspace sized for (T, R, W); edge capacity grows with R.
int ensure_workspace(fdbcs_conflict_set* cs, int64_t T, int64_t R, int64_t W) {
    if (T <= cs->ws_T && R <= cs->ws_R && W <= cs->ws_W) return FDBCS_OK;
    T = std::max<int64_t>(T, std::max<int64_t>(cs->ws_T, 1024));
    R = std::max<int64_t>(R, std::max<int64_t>(cs->ws_R, 4096));
    W = std::max<int64_t>(W, std::max<int64_t>(cs->ws_W, 4096));
    if (int rc = sync_all(cs)) return rc;
    const int64_t E = 2 * (R + W);
    int64_t edge_cap = std::max<int64_t>(16 * R, 1 << 22);
    if (const char* env = getenv("FDBCS_EDGE_CAP")) edge_cap = std::max<int64_t>(1, atoll(env));  // testing knob
    for (int k = 0; k < kNumWork; k++) {
    Work& w = cs->work[k];
    // One arena per workspace (slot 0), its size a multiple of 2 MiB: the ~50 scratch arrays of a
    // batch share a few large pages instead of one small allocation each (every kernel touches a
    // dozen of them; a single-workgroup kernel's first loads otherwise wait on address
    // translation misses).  Two passes: sizes, then the carve.
    size_t off = 0;
    char* arena = nullptr;
    auto take = [&](size_t bytes, void** ptr) -> int {
        off = align_up(off, 256);
        if (arena) *ptr = arena + off;
        off += bytes + 64;
        return FDBCS_OK;
    };
    for (int pass = 0; pass < 2; pass++) {
    if (pass == 1) {
        if (int rc = cs->ws[k][0].ensure(align_up(off, (size_t)2 << 20))) return rc;
        arena = (char*)cs->ws[k][0].p;
        off = 0;
    }
#define TAKE(field, bytes) \
    if (int rc = take((bytes), (void**)&w.field)) return rc
    TAKE(hist_conf, T);
    TAKE(rconf, R);
    TAKE(status, T);
    TAKE(first_conf, 4 * T);
    // the sort's slab holds kSlab endpoints per bucket for the buckets a batch of E endpoints
    // takes at the default target (sort_bucket_count clamps smaller targets to it)
    const int64_t slab_buckets = std::min<int64_t>(kSortMaxBuckets, (E + kSortTarget - 1) / kSortTarget + 1);
    TAKE(items, sizeof(SortItem) * E);
    TAKE(scnt, 8 * kCntStride * (size_t)kSortMaxBuckets);
    TAKE(slab, sizeof(SortItem) * kSlab * slab_buckets);
    TAKE(ovf, sizeof(SortItem) * E);
    TAKE(ovf_b, 4 * E);
    TAKE(big, sizeof(SortItem) * E);
    TAKE(big_p, 4 * E);
    TAKE(samples, sizeof(SortItem) * kMaxSample);
    TAKE(srank, 4 * (kMaxSample + 64));
    w.slab_buckets = (int32_t)slab_buckets;
    TAKE(pos, 4 * E);
    TAKE(pmeta, 4 * E);
    TAKE(cwb, 4 * (E + 1));
    TAKE(crb, 4 * (E + 1));
    TAKE(cwe, 4 * (E + 1));
    TAKE(wends, 8 * (2 * W + 1));
    TAKE(wkeys, sizeof(DKey) * (2 * W + 1));
    TAKE(segk, sizeof(DKey) * (2 * W + 2));
    TAKE(cflag, 2 * W + 2);
    TAKE(wbrange, 4 * W);
    TAKE(wlead, 4 * (W + 1));
    TAKE(wtxn, 4 * (W + 1));
    TAKE(gminc, 4 * (W + 1));
    TAKE(rbrange, 4 * R);
    TAKE(eoff, 4 * (R + 1));
    TAKE(poff, 4 * (R + W + 1));
    TAKE(pcg, 4 * (R + W + 1));
    TAKE(pcoff, 4 * (R + W + 1));
    TAKE(pcbase, 4 * (R + W + 1));
    TAKE(pca, 4 * (R + W + 1));
    TAKE(ecur, 4 * R);
    TAKE(edges, 4 * edge_cap);
    TAKE(eptr, 4 * T);
    TAKE(pre_st, T);
    TAKE(pre_ep, 4 * T);
    TAKE(pre_end, 4 * T);
    TAKE(ulist, 32 * T);
    TAKE(wpk, 4 * (W + 1));
    TAKE(tedges, 4 * edge_cap);
    TAKE(mcs_bits, 8 * (E / 64 + 2));
    TAKE(seg_b, 4 * (W + 1));
    TAKE(seg_e, 4 * (W + 1));
    TAKE(seg_lo, 8 * (W + 1));
    TAKE(seg_hi, 8 * (W + 1));
    TAKE(seg_rem, 8 * (W + 1));
    TAKE(seg_ins, 8 * (W + 1));
    TAKE(seg_tlen, 8 * (W + 1));
    TAKE(seg_endins, W + 1);
    TAKE(seg_vend, 8 * (W + 1));
    TAKE(verdict, T);
    TAKE(bsc, sizeof(BatchScalars));
    }
#undef TAKE
    w.edge_cap = edge_cap;
    w.cap_T = T;
    w.cap_R = R;
    // the epilogue of every batch re-zeroes these for the batch after next; start them zeroed
    HIPOK(hipMemsetAsync(w.hist_conf, 0, T, cs->stream));
    HIPOK(hipMemsetAsync(w.rconf, 0, R, cs->stream));
    HIPOK(hipMemsetAsync(w.ecur, 0, 4 * R, cs->stream));
    HIPOK(hipMemsetAsync(w.scnt, 0, 8 * kCntStride * (size_t)kSortMaxBuckets, cs->stream));
    HIPOK(hipMemsetAsync(w.srank, 0, 4 * (kMaxSample + 64), cs->stream));
    HIPOK(hipMemsetAsync(w.bsc, 0, sizeof(BatchScalars), cs->stream));
    // compaction arrays are shared (stage B only)
    if (k >= 1) {
        Work& w0 = cs->work[0];
        w.c_lo = w0.c_lo, w.c_hi = w0.c_hi, w.c_rem = w0.c_rem, w.c_ins = w0.c_ins, w.c_val = w0.c_val;
        w.c_exact = w0.c_exact;
    }
    }
    cs->edge_cap = edge_cap;
    cs->prev_segs = false;  // the last batch's segments were in the old arrays (and are merged: synced)
    cs->ws_T = T;
    cs->ws_R = R;
    cs->ws_W = W;
    return ensure_scan_arena(cs);
}

// Automatic delta bound: about 1/16 of the base, so a batch's merge touches a small tier and a
// compaction (a full rewrite of the base) is amortised over many batches.
// The delta tier's bound: N/16, raised towards N/4 up to kDeltaFloor boundaries.  A compaction
// rewrites the whole base on Y and the next check waits for it, so on a 5M-boundary base fewer,
// larger deltas pay although every merge copies more: C2 54.6 -> 56.7M, C3 45.9 -> 50.4M, C2 at
// 32768-txn batches 91.1 -> 92.9M over 150-400-batch windows with a 1.25M bound
// (scripts/gpu_r05_dl*.sh); a 50M base (C4) keeps N/16 = 3.1M.
constexpr int64_t kDeltaFloor = 1250000;
constexpr int kTimingEvery = 4;  // timing level 1 times the hot kernels of 1 batch in kTimingEvery
int64_t delta_limit_for(const fdbcs_conflict_set* cs, int64_t n_base) {
    if (cs->delta_limit > 0) return cs->delta_limit;
    return std::max<int64_t>({(int64_t)1 << 16, n_base / 16, std::min<int64_t>(n_base / 4, kDeltaFloor)});
}


Hist hist_of(fdbcs_conflict_set* cs, int k) {
    Hist h;
    h.key = (ulonglong2*)cs->hkey[k].p;
    h.lt = (uint2*)cs->hlt[k].p;
    h.ver = (int64_t*)cs->hver[k].p;
    return h;
}

// Search-tree levels laid out back to back in one allocation sized for `cap` boundaries.
void carve_index(MaxLevels& m, ulonglong2* base, int64_t cap) {
    for (int L = 0; L < kIdxLevels; L++) {
        m.skey[L] = base;
        base += idx_level_cap(cap, L);
    }
    m.skey8 = base;  // cap / 8 + 2 entries
    m.idx_cap = cap;
}

int64_t index_bytes(int64_t cap) {
    int64_t n = 0;
    for (int L = 0; L < kIdxLevels; L++) n += idx_level_cap(cap, L);
    return 16 * (n + cap / 8 + 2);
}

static void set_dir_fields(const fdbcs_conflict_set* cs, MaxLevels& m) {
    m.dir_p = cs->dir_p;
    m.dir_phi = cs->dir_phi;
    m.dir_plo = cs->dir_plo;
    m.dir_e = cs->dir_e;
    m.dir_top = cs->dir_top;
    for (int i = 0; i < kDirPos; i++) m.dir_pos[i] = cs->dir_pos[i], m.dir_w[i] = cs->dir_w[i];
}

// The directory code of the keys k[0..n) (sorted): their common prefix and, after it, the range
// of byte values at each position while the product of the ranges fits the slot budget (the last
// position coarsened by a shift).  See MaxLevels::dir_p.  Large loads are sampled (at most ~2M
// keys); values outside a position's range get the range's end codes.
static int set_dir_map(fdbcs_conflict_set* cs, const ulonglong2* k, int64_t n) {
    auto byte_at = [](const ulonglong2& x, int i) -> uint32_t {
        return i < 8 ? (uint32_t)(x.x >> (56 - 8 * i)) & 255u : (uint32_t)(x.y >> (56 - 8 * (i - 8))) & 255u;
    };
    const bool rank = n >= 2;
    uint32_t p = 0;
    if (rank) {
        const uint64_t xh = k[0].x ^ k[n - 1].x, xl = k[0].y ^ k[n - 1].y;
        const uint32_t lcp = xh ? (uint32_t)__builtin_clzll(xh) / 8 : (xl ? 8 + (uint32_t)__builtin_clzll(xl) / 8 : 16);
        p = std::min<uint32_t>(lcp, 15);
    }
    const uint64_t mh = p >= 8 ? ~0ull : (p ? ~0ull << (64 - 8 * p) : 0ull);
    const uint64_t ml = p <= 8 ? 0ull : ~0ull << (128 - 8 * p);
    cs->dir_p = p;
    cs->dir_phi = n ? k[0].x & mh : 0;
    cs->dir_plo = n ? k[0].y & ml : 0;
    const int npos = std::min<int>(kDirPos, 16 - (int)p);
    uint32_t lo[kDirPos], hi[kDirPos];
    for (int i = 0; i < kDirPos; i++) lo[i] = rank ? 255 : 0, hi[i] = 255;
    if (rank) {
        for (int i = 0; i < kDirPos; i++) hi[i] = 0;
        const int64_t stride = std::max<int64_t>(1, n / (1 << 21));
        auto mark = [&](const ulonglong2& x) {
            for (int i = 0; i < npos; i++) {
                const uint32_t b = byte_at(x, (int)p + i);
                lo[i] = std::min(lo[i], b);
                hi[i] = std::max(hi[i], b);
            }
        };
        for (int64_t j = 0; j < n; j += stride) mark(k[j]);
        mark(k[n - 1]);
    }
    const int64_t samples = (n + kFan - 1) / kFan;
    uint64_t budget = 1ull << 16;
    if (cs->dir_bits)
        budget = 1ull << cs->dir_bits;
    else
        while (budget < (1ull << kDirMaxBits) && 8 * budget < (uint64_t)samples) budget <<= 1;
    uint32_t radix[kDirPos], shift[kDirPos];
    uint64_t prod = 1;
    int e = 0;
    for (int i = 0; i < npos; i++) {
        const uint32_t d = hi[i] - lo[i] + 1;
        shift[i] = 0;
        if (prod * d <= budget) {
            radix[i] = d;
            prod *= d;
            if (d > 1) e = i + 1;  // trailing single-value positions add nothing
            continue;
        }
        uint32_t s = 0;  // coarsen: digit >> s, radix ((d - 1) >> s) + 1
        while (prod * (((d - 1) >> s) + 1) > budget) s++;
        if (((d - 1) >> s) + 1 > 1) {
            radix[i] = ((d - 1) >> s) + 1;
            shift[i] = s;
            e = i + 1;
        }
        break;
    }
    prod = 1;
    for (int i = 0; i < e; i++) prod *= radix[i];
    uint64_t w = 1;
    for (int i = kDirPos - 1; i >= 0; i--) {
        if (i >= e) {
            cs->dir_pos[i] = cs->dir_w[i] = 0;
            continue;
        }
        cs->dir_pos[i] = lo[i] | (hi[i] - lo[i] + 1) << 8 | shift[i] << 17;
        cs->dir_w[i] = (uint32_t)w;
        w *= radix[i];
    }
    cs->dir_e = (uint32_t)e;
    // codes run over [0, prod] (prod: above the range at the first position), slots are code + 1,
    // 0 below the common prefix and prod + 2 above it
    cs->dir_top = (uint32_t)prod + 2;
    return FDBCS_OK;
}

MaxLevels levels_of(fdbcs_conflict_set* cs, int k) {
    MaxLevels m;
    m.lvl[0] = (int64_t*)cs->hver[k].p;
    for (int L = 1; L < kMaxLevels; L++) m.lvl[L] = (int64_t*)cs->lvl[L].p;
    m.keys = (const ulonglong2*)cs->hkey[k].p;
    carve_index(m, (ulonglong2*)cs->lvl[0].p, cs->hist_cap);
    m.dir = cs->directory ? (const int32_t*)cs->dir.p : nullptr;
    set_dir_fields(cs, m);
    return m;
}

Hist delta_of(fdbcs_conflict_set* cs, int k) {
    Hist h;
    h.key = (ulonglong2*)cs->dkey[k].p;
    h.lt = (uint2*)cs->dlt[k].p;
    h.ver = (int64_t*)cs->dver[k].p;
    return h;
}

MaxLevels dlevels_of(fdbcs_conflict_set* cs, int k) {
    MaxLevels m;
    m.lvl[0] = (int64_t*)cs->dver[k].p;
    for (int L = 1; L < kMaxLevels; L++) m.lvl[L] = (int64_t*)cs->dlvl[k][L].p;
    m.keys = (const ulonglong2*)cs->dkey[k].p;
    carve_index(m, (ulonglong2*)cs->dlvl[k][0].p, cs->delta_cap);
    m.edir = (uint64_t*)cs->edir[k].p;
    m.edir_epoch = cs->edir[k].p ? cs->ddir_epoch[k] : 0;
    set_dir_fields(cs, m);  // the delta's directory slots too (the epilogue's fill)
    return m;
}

// Read the exact history size/tail usage back (synchronizes the stream).
int sync_sizes(fdbcs_conflict_set* cs) {
    if (int rc = sync_all(cs)) return rc;  // both halves of stage B
    Scalars s;
    HIPOK(hipMemcpyAsync(&s, cs->scal.p, sizeof(s), hipMemcpyDeviceToHost, cs->stream));
    HIPOK(hipStreamSynchronize(cs->stream));
    cs->n_ub = s.n;
    cs->nd_ub = s.nd;
    cs->tail_ub = s.tail_used;
    return FDBCS_OK;
}

// Range-max hierarchy buffers (and the sampled key index in lv[0]) for `cap` elements; returns the
// top level's length.
int alloc_levels(DBuf* lv, int64_t cap, int64_t* top_n, int64_t* l2_n) {
    lv[0].release();
    if (int rc = lv[0].ensure(index_bytes(cap))) return rc;
    int64_t m = cap;
    for (int L = 1; L < kMaxLevels; L++) {
        m = (m + kFan - 1) / kFan + 1;
        lv[L].release();
        if (int rc = lv[L].ensure(8 * (L == kMaxLevels - 1 ? l3_words(m) : m))) return rc;
        if (L == 2) *l2_n = m;
    }
    *top_n = m;
    return FDBCS_OK;
}

// Grow one ping-pong buffer set pair to `cap` elements, keeping the live `n` of set `live`.
int grow_sets(fdbcs_conflict_set* cs, DBuf* key, DBuf* lt, DBuf* ver, int live, int64_t n, int64_t cap) {
    int rc;
    for (int k = 0; k < 2; k++) {
        DBuf nk, nl, nv;
        if ((rc = nk.ensure(16 * cap)) || (rc = nl.ensure(8 * cap)) || (rc = nv.ensure(8 * cap))) return rc;
        if (k == live && n) {
            HIPOK(hipMemcpyAsync(nk.p, key[k].p, 16 * n, hipMemcpyDeviceToDevice, cs->stream));
            HIPOK(hipMemcpyAsync(nl.p, lt[k].p, 8 * n, hipMemcpyDeviceToDevice, cs->stream));
            HIPOK(hipMemcpyAsync(nv.p, ver[k].p, 8 * n, hipMemcpyDeviceToDevice, cs->stream));
        }
        HIPOK(hipStreamSynchronize(cs->stream));
        key[k].release();
        lt[k].release();
        ver[k].release();
        key[k] = nk;
        lt[k] = nl;
        ver[k] = nv;
    }
    return FDBCS_OK;
}

// Delta-tier capacity for `need` boundaries (plus the compaction arrays sized to match).
int ensure_delta(fdbcs_conflict_set* cs, int64_t need) {
    if (need <= cs->delta_cap) return FDBCS_OK;
    int rc = sync_sizes(cs);
    if (rc) return rc;
    int64_t cap = std::max<int64_t>(need, cs->delta_cap);
    cap = std::max<int64_t>(cap + cap / 2, 1 << 14);
    if ((rc = grow_sets(cs, cs->dkey, cs->dlt, cs->dver, cs->dcur, cs->nd_ub, cap))) return rc;
    for (int k = 0; k < 5; k++) {
        cs->cws[k].release();
        if ((rc = cs->cws[k].ensure(8 * (cap + 2)))) return rc;
    }
    cs->cws[5].release();
    if ((rc = cs->cws[5].ensure(cap + 2))) return rc;
    for (Work& w : cs->work) {  // compaction runs on stage B only: both workspaces share the arrays
        int64_t** c64[5] = {&w.c_lo, &w.c_hi, &w.c_rem, &w.c_ins, &w.c_val};
        for (int k = 0; k < 5; k++) *c64[k] = (int64_t*)cs->cws[k].p;
        w.c_exact = (uint8_t*)cs->cws[5].p;
    }
    for (int k = 0; k < 2; k++)
        if ((rc = alloc_levels(cs->dlvl[k], cap, &cs->dlvl3_n, &cs->dlvl2_n))) return rc;
    cs->delta_cap = cap;
    cs->ddir_epoch[0] = cs->ddir_epoch[1] = 0;  // the current delta's levels are rebuilt, its directory not
    cs->prev_segs = false;                      // (sync_sizes drained every stream)
    launch_rangemax(cs->stream, dlevels_of(cs, cs->dcur), (Scalars*)cs->scal.p, &((Scalars*)cs->scal.p)->ndb[cs->dcur],
                    cs->dlvl3_n, cs->dlvl2_n, std::max<int64_t>(cs->nd_ub, 1));
    HIPOK(take_launch_error());
    HIPOK(hipStreamSynchronize(cs->stream));
    return ensure_scan_arena(cs);
}

// Base-tier capacity for `need` boundaries (copies the live history when growing).
int ensure_history(fdbcs_conflict_set* cs, int64_t need, int64_t tail_need) {
    if (need <= cs->hist_cap && tail_need <= cs->tail_cap) return FDBCS_OK;
    int rc = sync_sizes(cs);
    if (rc) return rc;
    const int64_t tail_used = cs->tail_ub;
    if (need > cs->hist_cap) {
        int64_t cap = std::max<int64_t>(need, cs->hist_cap);
        cap = std::max<int64_t>(cap + cap / 4, 1 << 16);
        if ((rc = grow_sets(cs, cs->hkey, cs->hlt, cs->hver, cs->cur, cs->n_ub, cap))) return rc;
        if ((rc = alloc_levels(cs->lvl, cap, &cs->lvl3_n, &cs->lvl2_n))) return rc;
        if (cs->directory && (rc = cs->dir.ensure(4 * (size_t)kDirAlloc))) return rc;
        cs->hist_cap = cap;
        launch_rangemax(cs->stream, levels_of(cs, cs->cur), (Scalars*)cs->scal.p, &((Scalars*)cs->scal.p)->n,
                        cs->lvl3_n, cs->lvl2_n, std::max<int64_t>(cs->n_ub, 1));
        HIPOK(take_launch_error());
    }
    if (tail_need > cs->tail_cap) {
        int64_t tcap = std::max<int64_t>(tail_need, cs->tail_cap);
        tcap = std::max<int64_t>(tcap + tcap / 2, 1 << 16);
        DBuf nt, spare;
        if ((rc = nt.ensure(tcap + kTailSlack)) || (rc = spare.ensure(tcap + kTailSlack))) return rc;
        if (tail_used)
            HIPOK(hipMemcpyAsync(nt.p, cs->htail[cs->tcur].p, tail_used, hipMemcpyDeviceToDevice, cs->stream));
        HIPOK(hipStreamSynchronize(cs->stream));
        cs->htail[cs->tcur].release();
        cs->htail[cs->tcur ^ 1].release();
        cs->htail[cs->tcur] = nt;
        cs->htail[cs->tcur ^ 1] = spare;
        cs->tail_cap = tcap;
    }
    HIPOK(hipStreamSynchronize(cs->stream));
    return ensure_scan_arena(cs);
}

int ensure_events(fdbcs_batch* b) {
    BatchSlot* sl = b->slot;
    if (sl->events_made) return FDBCS_OK;
    for (int i = 0; i < kPhCount; i++) HIPOK(hipEventCreate(&sl->ev[i]));
    sl->events_made = true;
    return FDBCS_OK;
}

void release_slot(BatchSlot* sl) {
    if (!sl) return;
    if (sl->events_made)
        for (int i = 0; i < kPhCount; i++) (void)hipEventDestroy(sl->ev[i]);
    if (sl->ev_up) (void)hipEventDestroy(sl->ev_up);
    if (sl->ev_rt0) (void)hipEventDestroy(sl->ev_rt0);
    if (sl->ev_rt1) (void)hipEventDestroy(sl->ev_rt1);
    sl->rt_scan.release();
    sl->rt_inv.release();
    sl->rt_rids.release();
    sl->rt_dres.release();
    sl->rt_info.release();
    sl->rt_txpre.release();
    sl->rt_res.release();
    for (hipEvent_t e : sl->prof_pool) (void)hipEventDestroy(e);
    sl->dev.release();
    sl->dverdict.release();
    sl->pin_in.release();
    sl->pin_out.release();
    delete sl;
}

// Layout of a batch in pin_in / dev: [keys | rowner | wowner | snap | roff | woff | flags | tail].
// add_packed normalizes keys, owners and tails in place; the tail region is last so a capacity
// sized for an upper bound of the tail bytes costs no upload.
struct UploadLayout {
    size_t keys, rown, wown, snap, roff, woff, flags, tail, total;
};
UploadLayout upload_layout(size_t T, size_t R, size_t W, size_t tail_bytes) {
    UploadLayout L;
    size_t off = 0;
    L.keys = off;
    off = align_up(off + sizeof(DKey) * 2 * (R + W), 64);
    L.rown = off;
    off = align_up(off + 4 * R, 64);
    L.wown = off;
    off = align_up(off + 4 * W, 64);
    L.snap = off;
    off = align_up(off + 8 * T, 64);
    L.roff = off;
    off = align_up(off + 4 * (T + 1), 64);
    L.woff = off;
    off = align_up(off + 4 * (T + 1), 64);
    L.flags = off;
    off = align_up(off + T, 64);
    L.tail = off;
    off = align_up(off + tail_bytes + 48, 64);  // slack for dkey.h tail_word
    L.total = off;
    return L;
}

// History tail bytes a key of this length takes when inserted (8-byte aligned, kernels.hip tail_units).
inline int64_t padded_tail(int32_t len) { return len > 16 ? ((int64_t)len - 16 + 7) / 8 * 8 : 0; }

// Prefix words of a key (dkey_prefix), two big-endian loads when the key has 16 bytes or more.
inline void fast_prefix(const uint8_t* p, uint32_t len, uint64_t* hi, uint64_t* lo) {
    if (len >= 16) {
        uint64_t h, l;
        memcpy(&h, p, 8);
        memcpy(&l, p + 8, 8);
        *hi = __builtin_bswap64(h);
        *lo = __builtin_bswap64(l);
    } else {
        dkey_prefix(p, len, hi, lo);
    }
}

// Result buffer of a batch (host-mapped, written by the kernels): verdicts | scalars | completion
// flag, then the report copies rconf | hist | first_conf.
struct ResultLayout {
    size_t sc, fl, rc, hc, fc, total;
};
ResultLayout result_layout(size_t T, size_t R) {
    ResultLayout L;
    L.sc = (size_t)verdict_scalars_offset((int64_t)T);
    L.fl = align_up(L.sc + sizeof(Scalars), 64);
    L.rc = L.fl + 64;
    L.hc = align_up(L.rc + R + 1, 64);
    L.fc = align_up(L.hc + T + 1, 64);
    L.total = L.fc + 4 * (T + 1);
    return L;
}

// Every allocation a batch of this shape needs, made at add time so that detect (the timed,
// latency-critical call) never allocates: device copy, pinned result buffer, device verdicts.
int ensure_slot(BatchSlot* sl, size_t upload_bytes, size_t T, size_t R) {
    int rc;
    if ((rc = sl->dev.ensure(upload_bytes))) return rc;
    if ((rc = sl->pin_out.ensure(result_layout(T, R).total, true))) return rc;
    return sl->dverdict.ensure(T + 64);
}

int make_slot_events(BatchSlot* sl) {
    if (!sl->events_made) {
        for (int i = 0; i < kPhCount; i++) HIPOK(hipEventCreate(&sl->ev[i]));
        sl->events_made = true;
    }
    if (!sl->ev_up) HIPOK(hipEventCreateWithFlags(&sl->ev_up, hipEventDisableTiming));
    return FDBCS_OK;
}

// A direct-mode batch back into the pageable vectors (a second add call after add_packed).
void materialize(fdbcs_batch* b) {
    if (!b->direct) return;
    const char* h = (const char*)b->slot->pin_in.p;
    const size_t R = b->R(), W = b->W();
    const DKey* k = (const DKey*)(h + b->d_keys);
    b->rkeys.assign(k, k + 2 * R);
    b->wkeys.assign(k + 2 * R, k + 2 * (R + W));
    const int32_t* ro = (const int32_t*)(h + b->d_rown);
    const int32_t* wo = (const int32_t*)(h + b->d_wown);
    b->rowner.assign(ro, ro + R);
    b->wowner.assign(wo, wo + W);
    const uint8_t* t = (const uint8_t*)(h + b->d_tail);
    b->tail.assign(t, t + b->d_tail_bytes);
    b->direct = false;
}

// Has batch x's epilogue published its completion flag (null: destroyed, so done)?  The flag
// says the batch's results are final; workgroups of the epilogue other than the publishing one may
// still be writing the delta index and zeroing workspace scratch, so it never stands alone for
// "the launch is over" (stage_b_done).
inline bool batch_done(const fdbcs_batch* x) { return !x || (x->h_flag && *x->h_flag == x->seq && x->seq != 0); }

// May a dependency on workspace k's last stage B be skipped?  Only once that batch's flag was seen
// (so its stage B was issued: ev_b[k]'s last record is its own) AND ev_b[k] has completed, i.e. the
// whole epilogue launch is over.
inline bool stage_b_done(fdbcs_conflict_set* cs, int k) {
    return batch_done(cs->ws_user[k]) && hipEventQuery(cs->ev_b[k]) == hipSuccess;
}

// H2D of the packed batch by the DMA engine, issued now on `us` (the upload stream, or stage A's
// stream when the phases are timed one after another); ev_up marks its completion.
int do_upload(fdbcs_batch* b, hipStream_t us) {
    fdbcs_conflict_set* cs = b->cs;
    BatchSlot* sl = b->slot;
    const size_t T = b->T(), R = b->R(), W = b->W();
    const UploadLayout L = upload_layout(T, R, W, b->tail_size());
    int rc;
    if (!b->direct && (rc = sl->pin_in.ensure(L.total, true))) return rc;
    if ((rc = ensure_slot(sl, L.total, T, R))) return rc;
    char* h = (char*)sl->pin_in.p;
    if (!b->direct) {  // add_transaction path: normalized keys are in the pageable vectors
        if (R) memcpy(h + L.keys, b->rkeys.data(), sizeof(DKey) * 2 * R);
        if (W) memcpy(h + L.keys + sizeof(DKey) * 2 * R, b->wkeys.data(), sizeof(DKey) * 2 * W);
        if (R) memcpy(h + L.rown, b->rowner.data(), 4 * R);
        if (W) memcpy(h + L.wown, b->wowner.data(), 4 * W);
        if (!b->tail.empty()) memcpy(h + L.tail, b->tail.data(), b->tail.size());
    }
    memcpy(h + L.snap, b->snap.data(), 8 * T);
    memcpy(h + L.roff, b->roff.data(), 4 * (T + 1));
    memcpy(h + L.woff, b->woff.data(), 4 * (T + 1));
    if (T) memcpy(h + L.flags, b->flags.data(), T);
    // Both stages wait for ev_up.  A reused slot's device copy may still be read by the epilogue
    // of the batch that used it last.
    if (!sl->ev_up) HIPOK(hipEventCreateWithFlags(&sl->ev_up, hipEventDisableTiming));
    (void)cs;
    HIPOK(hipMemcpyAsync(sl->dev.p, h, L.total, hipMemcpyHostToDevice, us));
    HIPOK(hipEventRecord(sl->ev_up, us));
    char* d = (char*)sl->dev.p;
    b->bd.T = (int32_t)T;
    b->bd.R = (int32_t)R;
    b->bd.W = (int32_t)W;
    b->bd.snap = (int64_t*)(d + L.snap);
    b->bd.roff = (int32_t*)(d + L.roff);
    b->bd.woff = (int32_t*)(d + L.woff);
    b->bd.rowner = (int32_t*)(d + L.rown);
    b->bd.wowner = (int32_t*)(d + L.wown);
    b->bd.keys = (DKey*)(d + L.keys);
    b->bd.flags = (uint8_t*)(d + L.flags);
    b->bd.tail = (uint8_t*)(d + L.tail);
    b->tail_bytes = b->tail_size();
    b->bd.tail_n = (int64_t)b->tail_bytes;
    b->state = 1;
    return FDBCS_OK;
}

// ---- two submitting threads (FDBCS_SUBMIT_THREAD=1)
void worker_main(fdbcs_conflict_set* cs) {
    (void)hipSetDevice(cs->device);
    for (;;) {
        int j = 0;
        for (int spin = 0; spin < 20000 && (j = cs->wjob.load(std::memory_order_acquire)) == 0; spin++)
            std::this_thread::yield();
        if (j == 0) {
            std::unique_lock<std::mutex> lk(cs->wmu);
            cs->wcv.wait(lk, [&] { return (j = cs->wjob.load(std::memory_order_acquire)) != 0; });
        }
        if (j == 2) return;
        const int64_t ta = cs->htrace ? mono_ns() : 0;
        hipError_t e = cs->work_a.replay(cs->work_sa);
        if (cs->htrace) cs->htr[1].push_back({cs->work_a_seq, 'A', ta, mono_ns()});
        if (!cs->work_y.recs.empty()) {
            while (cs->x_issued.load(std::memory_order_acquire) < cs->work_need_x) std::this_thread::yield();
            const int64_t ty = cs->htrace ? mono_ns() : 0;
            const hipError_t e3 = cs->work_y.replay(cs->work_ys);
            if (cs->htrace) cs->htr[1].push_back({cs->work_y_seq, 'Y', ty, mono_ns()});
            if (e == hipSuccess) e = e3;
            cs->work_y.clear();
            cs->b_issued.fetch_add(1, std::memory_order_release);
        }
        if (!cs->work_c.recs.empty()) {
            while (cs->b_issued.load(std::memory_order_acquire) < cs->work_need_b) std::this_thread::yield();
            const hipError_t e2 = cs->work_c.replay(cs->cstream);
            if (e == hipSuccess) e = e2;
        }
        if (e != hipSuccess) {
            int expected = 0;
            cs->werr.compare_exchange_strong(expected, (int)e);
        }
        cs->wjob.store(0, std::memory_order_release);
    }
}

// Wait until the helper has issued its job; its first error, if any.
int worker_wait(fdbcs_conflict_set* cs) {
    if (!cs->worker.joinable()) return FDBCS_OK;
    while (cs->wjob.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    cs->work_y_batch = nullptr;  // any Y it held is issued
    return cs->werr.exchange(0) ? FDBCS_E_DEVICE : FDBCS_OK;
}

void worker_start_job(fdbcs_conflict_set* cs) {
    if (!cs->worker.joinable()) cs->worker = std::thread(worker_main, cs);
    {
        std::lock_guard<std::mutex> lk(cs->wmu);
        cs->wjob.store(1, std::memory_order_release);
    }
    cs->wcv.notify_one();
}

void worker_stop(fdbcs_conflict_set* cs) {
    if (!cs->worker.joinable()) return;
    (void)worker_wait(cs);
    {
        std::lock_guard<std::mutex> lk(cs->wmu);
        cs->wjob.store(2, std::memory_order_release);
    }
    cs->wcv.notify_one();
    cs->worker.join();
}

// The skip groups of batch b's X half at its replay: the kGroupEdges launches are left out once
// b's stage A has completed (ev_a) and its edge scan told the host (Work::hedge) that b has no
// candidate edge; otherwise (stage A still running, or not tracked) everything is issued.
uint8_t x_skip(fdbcs_conflict_set* cs, const fdbcs_batch* b) {
    if (!b || !cs->skip_edges || !cs->hedge.p) return 0;
    const volatile uint32_t* h = (const volatile uint32_t*)((char*)cs->hedge.p + 64 * b->wp);
    if (h[0] != b->seq) return 0;  // (cheap test first: no runtime call when the scan is not done)
    if (hipEventQuery(cs->ev_a[b->wp]) != hipSuccess) return 0;
    std::atomic_thread_fence(std::memory_order_acquire);
    return h[1] == 0u ? kGroupEdges : 0;
}

int flush_pending(fdbcs_conflict_set* cs) {
    if (int rc = worker_wait(cs)) return rc;  // stage A / check of the pending batch issued
    if (!cs->pending_batch) return FDBCS_OK;
    const uint8_t skip = x_skip(cs, cs->pending_batch);
    const uint32_t pseq = cs->pending_batch->seq;
    cs->pending_batch = nullptr;
    int rc = FDBCS_OK;
    const int64_t tx = cs->htrace ? mono_ns() : 0;
    if (cs->pending_b.replay(cs->stream, skip, &cs->stats.x_launches_skipped) != hipSuccess) rc = FDBCS_E_DEVICE;
    const int64_t ty = cs->htrace ? mono_ns() : 0;
    cs->x_issued.fetch_add(1, std::memory_order_release);
    if (cs->pending_y.replay(cs->pending_ys) != hipSuccess) rc = FDBCS_E_DEVICE;
    if (cs->htrace) {
        cs->htr[0].push_back({pseq, 'X', tx, ty});
        cs->htr[0].push_back({pseq, 'Y', ty, mono_ns()});
    }
    cs->b_issued.fetch_add(1, std::memory_order_release);
    cs->pending_b.clear();
    cs->pending_y.clear();
    return rc;
}

double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.0;
    return (double)ms;
}

}  // namespace

extern "C" {

const char* fdbcs_strerror(int s) {
    switch (s) {
        case FDBCS_OK: return "ok";
        case FDBCS_E_INVALID: return "invalid argument";
        case FDBCS_E_DEVICE: return "HIP device error";
        case FDBCS_E_NOMEM: return "out of memory";
        case FDBCS_E_VERSION: return "version below the history's newest version";
        case FDBCS_E_STATE: return "call out of order";
        case FDBCS_E_NODEVICE: return "no HIP device";
        case FDBCS_E_TIMEOUT: return "routed batch: the shares were never ready";
        default: return "unknown status";
    }
}

int fdbcs_new_conflict_set(int device, fdbcs_conflict_set** out) {
    if (!out) return FDBCS_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FDBCS_E_NODEVICE;
    if (device < 0 || device >= ndev) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(device));
    fdbcs_conflict_set* cs = new (std::nothrow) fdbcs_conflict_set();
    if (!cs) return FDBCS_E_NOMEM;
    cs->device = device;
    if (const char* v = getenv("FDBCS_VALIDATE")) cs->validate = v[0] == '1';
    if (const char* v = getenv("FDBCS_SORT_BUCKET")) cs->bucket_target = atoi(v);
    if (const char* v = getenv("FDBCS_SORT_COLD")) cs->sort_cold = v[0] == '1';
    if (const char* v = getenv("FDBCS_TRACE")) cs->trace = v[0] == '1';
    if (const char* v = getenv("FDBCS_SERIAL")) cs->serial = v[0] == '1';
    if (const char* v = getenv("FDBCS_RESOLVE_PREPASS")) cs->no_prepass = v[0] == '0';
    if (const char* v = getenv("FDBCS_SUBMIT_THREAD")) cs->submit_thread = v[0] != '0';
    if (const char* v = getenv("FDBCS_ADD_THREADS")) cs->add_threads = std::max(0, std::min(64, atoi(v)));
    if (const char* v = getenv("FDBCS_SKIP_EDGES")) cs->skip_edges = v[0] != '0';
    if (const char* v = getenv("FDBCS_WAIT_QUERY_MS")) cs->wait_query_ms = std::max(0, atoi(v));
    if (getenv("FDBCS_HOST_TRACE")) {
        cs->htrace = true;
        cs->htr[0].reserve(1 << 16);
        cs->htr[1].reserve(1 << 16);
    }
    if (const char* v = getenv("FDBCS_SPLIT_CHECK")) cs->split_check = atoi(v);
    if (const char* v = getenv("FDBCS_WRITE_GROUPS")) cs->write_groups = v[0] != '0';
    if (const char* v = getenv("FDBCS_DIRECTORY")) cs->directory = v[0] != '0';
    if (const char* v = getenv("FDBCS_DIR_BITS")) cs->dir_bits = std::max(0, std::min(kDirMaxBits, atoi(v)));
    if (const char* v = getenv("FDBCS_TAIL_RECLAIM")) cs->tail_reclaim = std::max<long long>(1, atoll(v));
    if (const char* v = getenv("FDBCS_ROUTE_TIMEOUT_MS")) cs->route_timeout_ms = std::max<long long>(1, atoll(v));
    static std::once_flag attr_once;
    std::call_once(attr_once, init_kernel_attributes);
    // Five streams at the default priority, every CU: stream priorities and CU partitions between
    // the chains measured slower (extra hardware queues; the chains slow each other
    // through the memory system, not by competing for CU slots).
    auto mk = [](hipStream_t* st) { return hipStreamCreateWithFlags(st, hipStreamNonBlocking) == hipSuccess; };
    bool ok = mk(&cs->stream) && mk(&cs->ystream) && mk(&cs->astream) && mk(&cs->ustream) && mk(&cs->cstream) &&
              hipEventCreateWithFlags(&cs->ev_cmp, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&cs->ev_quant, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; k < kNumWork && ok; k++)
        ok = hipEventCreateWithFlags(&cs->ev_a[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&cs->ev_c[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&cs->ev_b[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&cs->ev_res[k], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        fdbcs_destroy_conflict_set(cs);
        return FDBCS_E_DEVICE;
    }

    int rc = cs->scal.ensure(sizeof(Scalars));
    if (!rc) rc = cs->quant.ensure(2 * sizeof(SplitKey) * kQuant);
    if (!rc) rc = (hipMemsetAsync(cs->scal.p, 0, sizeof(Scalars), cs->stream) == hipSuccess) ? 0 : FDBCS_E_DEVICE;
    for (int k = 0; k < 2 && !rc && cs->directory; k++) {  // zeroed: epoch 0 entries are never trusted
        rc = cs->edir[k].ensure(8 * (size_t)kDirAlloc);
        if (!rc && hipMemsetAsync(cs->edir[k].p, 0, 8 * (size_t)kDirAlloc, cs->stream) != hipSuccess)
            rc = FDBCS_E_DEVICE;
    }
    if (!rc) rc = set_dir_map(cs, nullptr, 0);
    if (!rc) rc = ensure_history(cs, 1 << 16, 1 << 16);
    if (!rc) rc = ensure_delta(cs, 1 << 14);
    if (!rc) rc = ensure_workspace(cs, 1024, 4096, 4096);
    if (!rc) rc = ensure_btail(cs, 0);
    if (!rc && cs->trace) rc = cs->trace_buf.ensure(8 * kTrSlots);
    if (!rc && cs->skip_edges) rc = cs->hedge.ensure(64 * kNumWork, true);
    if (!rc && cs->skip_edges) {
        memset(cs->hedge.p, 0, 64 * kNumWork);
        for (int k = 0; k < kNumWork; k++) cs->work[k].hedge = (uint32_t*)((char*)cs->hedge.dp + 64 * k);
    }
    if (rc) {
        fdbcs_destroy_conflict_set(cs);
        return rc;
    }
    *out = cs;
    return FDBCS_OK;
}

void fdbcs_destroy_conflict_set(fdbcs_conflict_set* cs) {
    if (!cs) return;
    (void)hipSetDevice(cs->device);
    (void)flush_pending(cs);
    worker_stop(cs);
    if (cs->htrace) {
        char path[512];
        snprintf(path, sizeof(path), "%s.%d.csv", getenv("FDBCS_HOST_TRACE"), (int)getpid());
        if (FILE* f = fopen(path, "w")) {
            fprintf(f, "thread,seq,kind,t0,t1\n");
            for (int k = 0; k < 2; k++)
                for (const HSpan& h : cs->htr[k])
                    fprintf(f, "%d,%u,%c,%lld,%lld\n", k, h.seq, h.kind, (long long)h.t0, (long long)h.t1);
            fclose(f);
        }
    }
    if (getenv("FDBCS_ADD_PROFILE") && cs->add_prof_n)
        fprintf(stderr, "fdbcs add profile (%d threads, ms per batch over %lld): serial %.4f slot %.4f count %.4f fill %.4f\n",
                cs->add_threads, (long long)cs->add_prof_n, cs->add_prof[0] / cs->add_prof_n,
                cs->add_prof[1] / cs->add_prof_n, cs->add_prof[2] / cs->add_prof_n, cs->add_prof[3] / cs->add_prof_n);
    delete cs->add_pool;
    cs->add_pool = nullptr;
    if (cs->ustream) (void)hipStreamSynchronize(cs->ustream);
    if (cs->cstream) (void)hipStreamSynchronize(cs->cstream);
    if (cs->astream) (void)hipStreamSynchronize(cs->astream);
    if (cs->stream) (void)hipStreamSynchronize(cs->stream);
    if (cs->ystream) (void)hipStreamSynchronize(cs->ystream);
    for (int k = 0; k < 2; k++) {
        cs->hkey[k].release();
        cs->hlt[k].release();
        cs->hver[k].release();
        cs->dkey[k].release();
        cs->dlt[k].release();
        cs->dver[k].release();
    }
    cs->htail[0].release();
    cs->htail[1].release();
    for (auto& l : cs->lvl) l.release();
    cs->dir.release();
    for (auto& e : cs->edir) e.release();
    for (auto& set : cs->dlvl)
        for (auto& l : set) l.release();
    for (auto& x : cs->cws) x.release();
    for (auto& set : cs->ws)
        for (auto& x : set) x.release();
    for (auto& x : cs->wbtail) x.release();
    cs->scal.release();
    cs->quant.release();
    cs->trace_buf.release();
    cs->hold.release();
    cs->hedge.release();
    for (BatchSlot* sl : cs->pool) release_slot(sl);
    cs->pool.clear();
    // batches that outlive their set (e.g. garbage-collection order in a binding) keep their own
    // slot and refuse every further call
    for (fdbcs_batch* b : cs->live) b->cs = nullptr;
    cs->live.clear();
    for (int k = 0; k < kNumWork; k++) {
        if (cs->ev_a[k]) (void)hipEventDestroy(cs->ev_a[k]);
        if (cs->ev_c[k]) (void)hipEventDestroy(cs->ev_c[k]);
        if (cs->ev_b[k]) (void)hipEventDestroy(cs->ev_b[k]);
        if (cs->ev_res[k]) (void)hipEventDestroy(cs->ev_res[k]);
    }
    if (cs->ustream) (void)hipStreamDestroy(cs->ustream);
    if (cs->cstream) (void)hipStreamDestroy(cs->cstream);
    if (cs->ev_cmp) (void)hipEventDestroy(cs->ev_cmp);
    if (cs->ev_quant) (void)hipEventDestroy(cs->ev_quant);
    if (cs->astream) (void)hipStreamDestroy(cs->astream);
    if (cs->stream) (void)hipStreamDestroy(cs->stream);
    if (cs->ystream) (void)hipStreamDestroy(cs->ystream);
    delete cs;
}

int fdbcs_clear_conflict_set(fdbcs_conflict_set* cs, int64_t version) {
    if (!cs) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    if (int rc = flush_pending(cs)) return rc;
    if (int rc = sync_all(cs)) return rc;
    HIPOK(hipMemsetAsync(cs->scal.p, 0, sizeof(Scalars), cs->stream));
    HIPOK(hipStreamSynchronize(cs->stream));
    cs->header_version = version;
    cs->max_written = version;
    cs->ddir_epoch[0] = cs->ddir_epoch[1] = 0;
    if (int rc = set_dir_map(cs, nullptr, 0)) return rc;
    cs->prev_segs = false;
    cs->n_ub = 0;
    cs->nd_ub = 0;
    cs->tail_ub = 0;
    return FDBCS_OK;
}

int fdbcs_set_oldest_version(fdbcs_conflict_set* cs, int64_t v) {
    if (!cs) return FDBCS_E_INVALID;
    if (v > cs->oldest) cs->oldest = v;
    return FDBCS_OK;
}

int fdbcs_get_oldest_version(const fdbcs_conflict_set* cs, int64_t* out) {
    if (!cs || !out) return FDBCS_E_INVALID;
    *out = cs->oldest;
    return FDBCS_OK;
}

int fdbcs_reserve(fdbcs_conflict_set* cs, int64_t boundaries, int64_t tail_bytes, int32_t max_txns,
                  int32_t max_reads, int32_t max_writes) {
    if (!cs || boundaries < 0 || tail_bytes < 0 || max_txns < 0 || max_reads < 0 || max_writes < 0)
        return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    int rc = ensure_workspace(cs, max_txns, max_reads, max_writes);
    if (rc) return rc;
    const int64_t dneed = delta_limit_for(cs, boundaries) + 2 * (int64_t)max_writes + 2;
    if ((rc = ensure_delta(cs, dneed))) return rc;
    return ensure_history(cs, std::max<int64_t>(boundaries + dneed, cs->hist_cap),
                          std::max<int64_t>(tail_bytes, cs->tail_cap));
}

int fdbcs_set_gc_interval(fdbcs_conflict_set* cs, int32_t every) {
    if (!cs || every < 0) return FDBCS_E_INVALID;
    cs->gc_interval = every;
    return FDBCS_OK;
}

int fdbcs_set_timing(fdbcs_conflict_set* cs, int32_t level) {
    if (!cs || level < 0 || level > 3) return FDBCS_E_INVALID;
    cs->timing = level;
    return FDBCS_OK;
}

int fdbcs_set_delta_limit(fdbcs_conflict_set* cs, int64_t boundaries) {
    if (!cs || boundaries < 0) return FDBCS_E_INVALID;
    cs->delta_limit = boundaries;
    return FDBCS_OK;
}

int fdbcs_history_size(fdbcs_conflict_set* cs, int64_t* out) {
    if (!cs || !out) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    int rc = sync_sizes(cs);
    if (rc) return rc;
    *out = cs->n_ub + cs->nd_ub;
    return FDBCS_OK;
}

int fdbcs_load_history(fdbcs_conflict_set* cs, int64_t n, const uint8_t* key_bytes, const int64_t* key_offsets,
                       const int64_t* versions, int64_t header_version) {
    if (!cs || n < 0 || (n > 0 && (!key_bytes || !key_offsets || !versions))) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    if (int rc = sync_all(cs)) return rc;
    std::vector<ulonglong2> k(n);
    std::vector<uint2> lt(n);
    std::vector<uint8_t> tail;
    int64_t maxv = header_version;
    for (int64_t i = 0; i < n; i++) {
        const uint8_t* p = key_bytes + key_offsets[i];
        const int32_t len = (int32_t)(key_offsets[i + 1] - key_offsets[i]);
        if (len < 0) return FDBCS_E_INVALID;
        if (i > 0) {
            const uint8_t* q = key_bytes + key_offsets[i - 1];
            const int32_t ql = (int32_t)(key_offsets[i] - key_offsets[i - 1]);
            if (cmp_bytes(q, ql, p, len) >= 0) return FDBCS_E_INVALID;  // strictly ascending
        }
        uint64_t hi, lo;
        dkey_prefix(p, (uint32_t)len, &hi, &lo);
        k[i] = make_ulonglong2(hi, lo);
        uint32_t toff = 0;
        if (len > 16) {  // 8-byte aligned, offset in 8-byte units
            if ((int64_t)tail.size() + len >= kTailLimit) return FDBCS_E_NOMEM;
            toff = (uint32_t)(tail.size() / 8);
            tail.insert(tail.end(), p + 16, p + len);
            tail.resize((tail.size() + 7) / 8 * 8, 0);
        }
        lt[i] = make_uint2((uint32_t)len, toff);
        maxv = std::max(maxv, versions[i]);
    }
    int rc = ensure_history(cs, n + 1, (int64_t)tail.size() + 1);
    if (rc) return rc;
    if (n) {
        HIPOK(hipMemcpyAsync(cs->hkey[cs->cur].p, k.data(), 16 * n, hipMemcpyHostToDevice, cs->stream));
        HIPOK(hipMemcpyAsync(cs->hlt[cs->cur].p, lt.data(), 8 * n, hipMemcpyHostToDevice, cs->stream));
        HIPOK(hipMemcpyAsync(cs->hver[cs->cur].p, versions, 8 * n, hipMemcpyHostToDevice, cs->stream));
    }
    if (!tail.empty())
        HIPOK(hipMemcpyAsync(cs->htail[cs->tcur].p, tail.data(), tail.size(), hipMemcpyHostToDevice, cs->stream));
    Scalars s{};
    s.n = n;
    s.tail_used = (int64_t)tail.size();
    HIPOK(hipMemcpyAsync(cs->scal.p, &s, sizeof(s), hipMemcpyHostToDevice, cs->stream));
    // the directory code of the loaded keys (k_directory below builds on it)
    if (int rc = set_dir_map(cs, k.data(), n)) return rc;
    launch_rangemax(cs->stream, levels_of(cs, cs->cur), (Scalars*)cs->scal.p, &((Scalars*)cs->scal.p)->n, cs->lvl3_n,
                    cs->lvl2_n, std::max<int64_t>(n, 1));
    HIPOK(take_launch_error());
    HIPOK(hipStreamSynchronize(cs->stream));
    cs->header_version = header_version;
    cs->max_written = maxv;
    cs->ddir_epoch[0] = cs->ddir_epoch[1] = 0;  // no delta directory entry of the old slot mapping is trusted
    cs->prev_segs = false;
    cs->n_ub = n;
    cs->nd_ub = 0;
    cs->tail_ub = (int64_t)tail.size();
    return FDBCS_OK;
}

int fdbcs_get_stats(fdbcs_conflict_set* cs, fdbcs_stats* out) {
    if (!cs || !out) return FDBCS_E_INVALID;
    *out = cs->stats;
    return FDBCS_OK;
}

int fdbcs_reset_stats(fdbcs_conflict_set* cs) {
    if (!cs) return FDBCS_E_INVALID;
    memset(&cs->stats, 0, sizeof(cs->stats));
    cs->kprof.clear();
    return FDBCS_OK;
}

// Demangled kernel name without its namespace and argument list ("k_scan<3, fdbcs::PosScan>").
static std::string kernel_name(const void* func, hipStream_t s) {
    const char* m = hipKernelNameRefByPtr(func, s);
    if (!m) return "?";
    int st = 0;
    char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
    std::string n = (st == 0 && d) ? d : m;
    free(d);
    // drop the return type, namespace prefix and parameter list
    if (n.rfind("void ", 0) == 0) n = n.substr(5);
    int depth = 0;
    for (size_t i = 0; i < n.size(); i++) {
        if (n[i] == '<') depth++;
        if (n[i] == '>') depth--;
        if (n[i] == '(' && depth == 0) {
            n = n.substr(0, i);
            break;
        }
    }
    if (n.rfind("fdbcs::", 0) == 0) n = n.substr(7);
    return n;
}

int fdbcs_kernel_profile(fdbcs_conflict_set* cs, int32_t index, char* name, int32_t cap, int64_t* launches,
                         double* ms) {
    if (!cs || index < 0 || index >= (int32_t)cs->kprof.size()) return FDBCS_E_INVALID;
    const auto& k = cs->kprof[index];
    if (name && cap > 0) {
        const std::string n = kernel_name(k.func, cs->stream);
        snprintf(name, (size_t)cap, "%s", n.c_str());
    }
    if (launches) *launches = k.launches;
    if (ms) *ms = k.ms;
    return FDBCS_OK;
}

int fdbcs_debug_hold(fdbcs_conflict_set* cs, int32_t on) {
    if (!cs) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    if (int rc = cs->hold.ensure(64, true)) return rc;
    volatile uint32_t* word = (volatile uint32_t*)cs->hold.p;
    if (!on) {
        __atomic_store_n((uint32_t*)word, 1u, __ATOMIC_SEQ_CST);
        return FDBCS_OK;
    }
    if (int rc = sync_all(cs)) return rc;
    *word = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    for (hipStream_t st : {cs->ustream, cs->astream, cs->cstream, cs->stream}) launch_hold(st, (const uint32_t*)cs->hold.dp);
    HIPOK(take_launch_error());
    return FDBCS_OK;
}

int fdbcs_set_timed_kernel(fdbcs_conflict_set* cs, const char* name) {
    if (!cs) return FDBCS_E_INVALID;
    cs->timed_func = nullptr;
    if (!name || !name[0]) return FDBCS_OK;
    for (const auto& k : cs->kprof)
        if (kernel_name(k.func, cs->stream) == name) {
            cs->timed_func = k.func;
            return FDBCS_OK;
        }
    return FDBCS_E_INVALID;  // only kernels seen by a profiled batch can be named
}

int fdbcs_batch_new(fdbcs_conflict_set* cs, int report_keys, fdbcs_batch** out) {
    if (!cs || !out) return FDBCS_E_INVALID;
    fdbcs_batch* b = new (std::nothrow) fdbcs_batch();
    if (!b) return FDBCS_E_NOMEM;
    b->cs = cs;
    if (!cs->pool.empty()) {
        b->slot = cs->pool.back();
        cs->pool.pop_back();
    } else {
        b->slot = new (std::nothrow) BatchSlot();
        if (!b->slot) {
            delete b;
            return FDBCS_E_NOMEM;
        }
        if (int rc = make_slot_events(b->slot)) {
            release_slot(b->slot);
            delete b;
            return rc;
        }
    }
    cs->live.insert(b);
    b->report_enabled = report_keys ? 1 : 0;
    *out = b;
    return FDBCS_OK;
}

void fdbcs_batch_destroy(fdbcs_batch* b) {
    if (!b) return;
    if (!b->cs) {  // its set was destroyed first (and synchronized its streams)
        release_slot(b->slot);
        delete b;
        return;
    }
    if (b->state == 2) {  // still in flight: its set (which must outlive it) owns the stream
        (void)hipSetDevice(b->cs->device);
        (void)flush_pending(b->cs);
        (void)hipStreamSynchronize(b->cs->ustream);
        (void)hipStreamSynchronize(b->cs->cstream);
        (void)hipStreamSynchronize(b->cs->astream);
        (void)hipStreamSynchronize(b->cs->stream);
        (void)hipStreamSynchronize(b->cs->ystream);
        b->cs->inflight--;
    } else if (b->state == 1) {  // uploaded, never submitted: the copy may still be in flight
        (void)hipSetDevice(b->cs->device);
        (void)hipStreamSynchronize(b->cs->ustream);
        (void)hipStreamSynchronize(b->cs->astream);
    }
    // done (waited or synchronized): dependencies on it need no wait any more
    for (int k = 0; k < kNumWork; k++) {
        if (b->cs->ws_user[k] == b) b->cs->ws_user[k] = nullptr;
        if (b->cs->xfree_user[k] == b) b->cs->xfree_user[k] = nullptr;
    }
    // the slot goes back to the set's pool (its buffers and events are reused by the next batch)
    if (b->slot) b->cs->pool.push_back(b->slot);
    b->cs->live.erase(b);
    delete b;
}

int fdbcs_batch_add_transaction(fdbcs_batch* b, int64_t read_snapshot, int report_conflicting_keys, int32_t n_reads,
                                const uint8_t* const* read_begin, const int32_t* read_begin_len,
                                const uint8_t* const* read_end, const int32_t* read_end_len, int32_t n_writes,
                                const uint8_t* const* write_begin, const int32_t* write_begin_len,
                                const uint8_t* const* write_end, const int32_t* write_end_len) {
    if (!b || n_reads < 0 || n_writes < 0) return FDBCS_E_INVALID;
    if (b->state != 0 || !b->cs) return FDBCS_E_STATE;
    if ((n_reads && (!read_begin || !read_end || !read_begin_len || !read_end_len)) ||
        (n_writes && (!write_begin || !write_end || !write_begin_len || !write_end_len)))
        return FDBCS_E_INVALID;
    // KeyRangeRef rejects begin > end (FDBTypes.h:288-291): validate before mutating anything.
    for (int32_t i = 0; i < n_reads; i++)
        if (read_begin_len[i] < 0 || read_end_len[i] < 0 ||
            cmp_bytes(read_begin[i], read_begin_len[i], read_end[i], read_end_len[i]) > 0)
            return FDBCS_E_INVALID;
    for (int32_t i = 0; i < n_writes; i++)
        if (write_begin_len[i] < 0 || write_end_len[i] < 0 ||
            cmp_bytes(write_begin[i], write_begin_len[i], write_end[i], write_end_len[i]) > 0)
            return FDBCS_E_INVALID;
    materialize(b);
    const int32_t t = b->T();
    uint8_t fl = (report_conflicting_keys && b->report_enabled) ? kFlagReport : 0;
    b->n_report += fl ? 1 : 0;
    const bool too_old = read_snapshot < b->cs->oldest && n_reads > 0;  // SkipList.cpp:770
    if (too_old) fl |= kFlagTooOld;
    b->snap.push_back(read_snapshot);
    b->flags.push_back(fl);
    if (!too_old) {
        for (int32_t i = 0; i < n_reads; i++) {
            add_key(b, b->rkeys, read_begin[i], read_begin_len[i]);
            add_key(b, b->rkeys, read_end[i], read_end_len[i]);
            b->rowner.push_back(t);
        }
        for (int32_t i = 0; i < n_writes; i++) {
            add_key(b, b->wkeys, write_begin[i], write_begin_len[i]);
            add_key(b, b->wkeys, write_end[i], write_end_len[i]);
            b->wtail += padded_tail(write_begin_len[i]) + padded_tail(write_end_len[i]);
            b->wowner.push_back(t);
        }
    }
    b->roff.push_back(b->roff.back() + (too_old ? 0 : n_reads));
    b->woff.push_back(b->woff.back() + (too_old ? 0 : n_writes));
    return FDBCS_OK;
}

// begin <= end of one range (KeyRangeRef, FDBTypes.h:288-291) from the normalized prefixes, the
// tails only when both prefixes tie and both keys run past 16 bytes (SkipList.cpp:53-60 order).
static inline bool range_inverted(const DKey& a, const DKey& b, const uint8_t* ka, const uint8_t* kb) {
    if (a.hi != b.hi) return a.hi > b.hi;
    if (a.lo != b.lo) return a.lo > b.lo;
    if (a.len <= 16 || b.len <= 16) return a.len > b.len;  // the shorter is a prefix of the longer
    return cmp_bytes(ka + 16, (int32_t)a.len - 16, kb + 16, (int32_t)b.len - 16) > 0;
}

static inline void normalize_key(const uint8_t* p, uint32_t len, DKey* out) {
    fast_prefix(p, len, &out->hi, &out->lo);
    out->len = len;
    out->tail = 0;
}

// addTransaction of a whole packed batch into an empty batch (offsets already checked monotone):
// the endpoint keys are validated and normalized straight into the batch's pinned staging, in
// chunks of transactions over the conflict set's add threads (AddPool), with no per-range
// vectors and no copy at upload.  All-or-nothing: an inverted range leaves the batch empty.
static int add_packed_direct(fdbcs_batch* b, const fdbcs_packed_batch* pb) {
    fdbcs_conflict_set* cs = b->cs;
    const int32_t T = pb->n_txn;
    const int64_t oldest = cs->oldest;
    using clk = std::chrono::steady_clock;
    const auto tp0 = clk::now();
    b->snap.assign(pb->read_snapshot, pb->read_snapshot + T);
    b->flags.resize(T);
    b->roff.resize(T + 1);
    b->woff.resize(T + 1);
    int32_t Ra = 0, Wa = 0, n_report = 0;
    for (int32_t t = 0; t < T; t++) {
        const int32_t nr = pb->read_offsets[t + 1] - pb->read_offsets[t];
        const int32_t nw = pb->write_offsets[t + 1] - pb->write_offsets[t];
        uint8_t fl = (pb->report_conflicting_keys && pb->report_conflicting_keys[t] && b->report_enabled)
                         ? kFlagReport
                         : 0;
        n_report += fl ? 1 : 0;
        const bool too_old = pb->read_snapshot[t] < oldest && nr > 0;  // SkipList.cpp:770
        if (too_old) fl |= kFlagTooOld;
        b->flags[t] = fl;
        b->roff[t] = Ra;
        b->woff[t] = Wa;
        if (!too_old) {
            Ra += nr;
            Wa += nw;
        }
    }
    b->roff[T] = Ra;
    b->woff[T] = Wa;
    const int32_t R = pb->read_offsets[T];
    const int64_t nk = 2 * ((int64_t)R + pb->write_offsets[T]);
    const size_t tail_bound = nk ? (size_t)(pb->key_offsets[nk] - pb->key_offsets[0]) : 0;
    const UploadLayout L = upload_layout(T, Ra, Wa, tail_bound);
    auto fail = [&](int rc) {
        b->snap.clear();
        b->flags.clear();
        b->roff.assign(1, 0);
        b->woff.assign(1, 0);
        return rc;
    };
    const auto tp1 = clk::now();
    if (int rc = b->slot->pin_in.ensure(L.total, true)) return fail(rc);
    if (int rc = ensure_slot(b->slot, L.total, T, Ra)) return fail(rc);
    const auto tp2 = clk::now();
    char* h = (char*)b->slot->pin_in.p;
    DKey* keys = (DKey*)(h + L.keys);
    DKey* wk = keys + 2 * (size_t)Ra;
    int32_t* rown = (int32_t*)(h + L.rown);
    int32_t* wown = (int32_t*)(h + L.wown);
    uint8_t* tail = (uint8_t*)(h + L.tail);
    const uint8_t* kb = pb->key_bytes;
    const int64_t* ko = pb->key_offsets;
    // chunks of ~512 ranges; one chunk (no pool) for small batches
    const int64_t G = (int64_t)R + pb->write_offsets[T];
    const int nchunk = (int)std::max<int64_t>(1, std::min<int64_t>(256, G / 512));
    struct Chunk {
        int32_t t0, t1;
        int64_t tails, wtail;
        int32_t max_len;
        bool bad;
    };
    std::vector<Chunk> ch(nchunk);
    for (int c = 0; c < nchunk; c++) {
        ch[c] = Chunk{(int32_t)((int64_t)T * c / nchunk), (int32_t)((int64_t)T * (c + 1) / nchunk), 0, 0, 0, false};
    }
    const bool pooled = nchunk > 1 && cs->add_threads > 0;
    if (pooled && !cs->add_pool) {
        try {
            cs->add_pool = new AddPool(cs->add_threads);
        } catch (...) {  // no memory or no threads left: this call and later ones run serially
            cs->add_pool = nullptr;
            cs->add_threads = 0;
        }
    }
    // pass 1 (tickets [0, nchunk)): tail bytes of each chunk's admitted keys (key offsets only), so
    // the tails pack exactly in transaction order; pass 2 (tickets [nchunk, 2 nchunk)) waits for
    // every count (tickets go out in order, so every count is held by a running thread)
    std::atomic<int> counted{0};
    const std::function<void(int)> count = [&](int c) {
        Chunk& k = ch[c];
        int64_t tb = 0;
        for (int32_t t = k.t0; t < k.t1; t++) {
            if (b->flags[t] & kFlagTooOld) continue;
            const int64_t r0 = 2 * (int64_t)pb->read_offsets[t], r1 = 2 * (int64_t)pb->read_offsets[t + 1];
            const int64_t w0 = 2 * ((int64_t)R + pb->write_offsets[t]), w1 = 2 * ((int64_t)R + pb->write_offsets[t + 1]);
            for (int64_t q = r0; q < r1; q++) tb += std::max<int64_t>(0, ko[q + 1] - ko[q] - 16);
            for (int64_t q = w0; q < w1; q++) tb += std::max<int64_t>(0, ko[q + 1] - ko[q] - 16);
        }
        k.tails = tb;
        counted.fetch_add(1, std::memory_order_release);
    };
    const auto tp3 = clk::now();
    // pass 2: every range validated (TooOld transactions' too: KeyRangeRef asserts begin <= end
    // whatever the batch does with it), admitted ones normalized with their owners and tails
    const std::function<void(int)> fill = [&](int c) {
        Chunk& k = ch[c];
        while (counted.load(std::memory_order_acquire) < nchunk) __builtin_ia32_pause();
        int64_t tb = 0, wt = 0;
        for (int q = 0; q < c; q++) tb += ch[q].tails;
        int32_t ml = 0;
        bool bad = false;
        auto put = [&](DKey* out, int64_t q) {
            const uint8_t* p = kb + ko[q];
            const uint32_t len = (uint32_t)(ko[q + 1] - ko[q]);
            normalize_key(p, len, out);
            if ((int32_t)len > ml) ml = (int32_t)len;
            if (len > 16) {
                out->tail = (uint32_t)tb;
                memcpy(tail + tb, p + 16, len - 16);
                tb += len - 16;
            }
        };
        for (int32_t t = k.t0; t < k.t1 && !bad; t++) {
            const int32_t r0 = pb->read_offsets[t], r1 = pb->read_offsets[t + 1];
            const int32_t w0 = pb->write_offsets[t], w1 = pb->write_offsets[t + 1];
            if (b->flags[t] & kFlagTooOld) {
                auto check = [&](int64_t q) {
                    DKey x, y;
                    normalize_key(kb + ko[q], (uint32_t)(ko[q + 1] - ko[q]), &x);
                    normalize_key(kb + ko[q + 1], (uint32_t)(ko[q + 2] - ko[q + 1]), &y);
                    bad |= range_inverted(x, y, kb + ko[q], kb + ko[q + 1]);
                };
                for (int32_t r = r0; r < r1; r++) check(2 * (int64_t)r);
                for (int32_t w = w0; w < w1; w++) check(2 * ((int64_t)R + w));
                continue;
            }
            const int32_t ra = b->roff[t], wa = b->woff[t];
            for (int32_t r = r0, i = 0; r < r1; r++, i++) {
                DKey* o = keys + 2 * (size_t)(ra + i);
                put(o, 2 * (int64_t)r);
                put(o + 1, 2 * (int64_t)r + 1);
                bad |= range_inverted(o[0], o[1], kb + ko[2 * (int64_t)r], kb + ko[2 * (int64_t)r + 1]);
                rown[ra + i] = t;
            }
            for (int32_t w = w0, i = 0; w < w1; w++, i++) {
                DKey* o = wk + 2 * (size_t)(wa + i);
                const int64_t q = 2 * ((int64_t)R + w);
                put(o, q);
                put(o + 1, q + 1);
                bad |= range_inverted(o[0], o[1], kb + ko[q], kb + ko[q + 1]);
                wt += padded_tail((int32_t)(ko[q + 1] - ko[q])) + padded_tail((int32_t)(ko[q + 2] - ko[q + 1]));
                wown[wa + i] = t;
            }
        }
        k.wtail = wt;
        k.max_len = ml;
        k.bad = bad;
    };
    const std::function<void(int)> both = [&](int q) { q < nchunk ? count(q) : fill(q - nchunk); };
    if (pooled && cs->add_pool)
        cs->add_pool->parallel_for(2 * nchunk, both);
    else
        for (int q = 0; q < 2 * nchunk; q++) both(q);
    int64_t tb_total = 0;
    for (int c = 0; c < nchunk; c++) tb_total += ch[c].tails;
    const auto tp4 = clk::now();
    {
        auto ms = [](clk::time_point a, clk::time_point b_) { return std::chrono::duration<double, std::milli>(b_ - a).count(); };
        cs->add_prof[0] += ms(tp0, tp1);
        cs->add_prof[1] += ms(tp1, tp2);
        cs->add_prof[2] += ms(tp2, tp3);  // (nothing: count and fill run as one job)
        cs->add_prof[3] += ms(tp3, tp4);
        cs->add_prof_n++;
    }
    int64_t wtail = 0;
    int32_t max_len = b->max_len;
    for (const Chunk& k : ch) {
        if (k.bad) return fail(FDBCS_E_INVALID);
        wtail += k.wtail;
        max_len = std::max(max_len, k.max_len);
    }
    b->wtail += wtail;
    b->max_len = max_len;
    b->n_report += n_report;
    b->direct = true;
    b->d_keys = L.keys;
    b->d_rown = L.rown;
    b->d_wown = L.wown;
    b->d_tail = L.tail;
    b->d_tail_bytes = (size_t)tb_total;
    return FDBCS_OK;
}

static inline double host_ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

static int add_packed_impl(fdbcs_batch* b, const fdbcs_packed_batch* pb);

int fdbcs_batch_add_packed(fdbcs_batch* b, const fdbcs_packed_batch* pb) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = add_packed_impl(b, pb);
    if (rc == FDBCS_OK && b->cs) {
        b->cs->stats.host_ms_add += host_ms_since(t0);
        b->cs->stats.added_txns += pb->n_txn;
    }
    return rc;
}

static int add_packed_impl(fdbcs_batch* b, const fdbcs_packed_batch* pb) {
    if (!b || !pb || pb->n_txn < 0) return FDBCS_E_INVALID;
    if (b->state != 0 || !b->cs) return FDBCS_E_STATE;
    const int32_t T = pb->n_txn;
    if (T == 0) return FDBCS_OK;
    if (!pb->read_snapshot || !pb->read_offsets || !pb->write_offsets || !pb->key_offsets) return FDBCS_E_INVALID;
    const int32_t R = pb->read_offsets[T];
    const int64_t nk = 2 * ((int64_t)R + pb->write_offsets[T]);
    if (nk && !pb->key_bytes) return FDBCS_E_INVALID;
    // validate everything first (all-or-nothing): offsets here, ranges below (fused with the
    // normalization on the direct path)
    for (int32_t t = 0; t < T; t++)
        if (pb->read_offsets[t + 1] < pb->read_offsets[t] || pb->write_offsets[t + 1] < pb->write_offsets[t])
            return FDBCS_E_INVALID;
    for (int64_t k = 0; k < nk; k++)
        if (pb->key_offsets[k + 1] < pb->key_offsets[k]) return FDBCS_E_INVALID;
    if (b->T() == 0 && !b->direct) return add_packed_direct(b, pb);
    for (int64_t k = 0; k < nk; k += 2) {
        const int64_t a0 = pb->key_offsets[k], a1 = pb->key_offsets[k + 1], a2 = pb->key_offsets[k + 2];
        if (cmp_bytes(pb->key_bytes + a0, (int32_t)(a1 - a0), pb->key_bytes + a1, (int32_t)(a2 - a1)) > 0)
            return FDBCS_E_INVALID;
    }
    const int64_t oldest = b->cs->oldest;
    materialize(b);
    b->snap.reserve(b->snap.size() + T);
    for (int32_t t = 0; t < T; t++) {
        const int32_t tt = b->T();
        const int32_t r0 = pb->read_offsets[t], r1 = pb->read_offsets[t + 1];
        const int32_t w0 = pb->write_offsets[t], w1 = pb->write_offsets[t + 1];
        uint8_t fl = (pb->report_conflicting_keys && pb->report_conflicting_keys[t] && b->report_enabled)
                         ? kFlagReport
                         : 0;
        b->n_report += fl ? 1 : 0;
        const bool too_old = pb->read_snapshot[t] < oldest && r1 > r0;
        if (too_old) fl |= kFlagTooOld;
        b->snap.push_back(pb->read_snapshot[t]);
        b->flags.push_back(fl);
        if (!too_old) {
            for (int32_t r = r0; r < r1; r++) {
                for (int e = 0; e < 2; e++) {
                    const int64_t k = 2 * (int64_t)r + e;
                    add_key(b, b->rkeys, pb->key_bytes + pb->key_offsets[k],
                            (int32_t)(pb->key_offsets[k + 1] - pb->key_offsets[k]));
                }
                b->rowner.push_back(tt);
            }
            for (int32_t w = w0; w < w1; w++) {
                for (int e = 0; e < 2; e++) {
                    const int64_t k = 2 * ((int64_t)R + w) + e;
                    b->wtail += padded_tail((int32_t)(pb->key_offsets[k + 1] - pb->key_offsets[k]));
                    add_key(b, b->wkeys, pb->key_bytes + pb->key_offsets[k],
                            (int32_t)(pb->key_offsets[k + 1] - pb->key_offsets[k]));
                }
                b->wowner.push_back(tt);
            }
        }
        b->roff.push_back(b->roff.back() + (too_old ? 0 : r1 - r0));
        b->woff.push_back(b->woff.back() + (too_old ? 0 : w1 - w0));
    }
    return FDBCS_OK;
}

// ---- multi-resolver routing: proxy shares (engine.h ShareHeader) and the device split

static size_t share_layout(int32_t T, int64_t R, int64_t W, int64_t tail, ShareHeader* h) {
    size_t off = sizeof(ShareHeader);
    h->T = T;
    h->R = (int32_t)R;
    h->W = (int32_t)W;
    h->off_keys = (int64_t)off;
    off = align_up(off + sizeof(DKey) * 2 * (size_t)(R + W), 64);
    h->off_snap = (int64_t)off;
    off = align_up(off + 8 * (size_t)T, 64);
    h->off_roff = (int64_t)off;
    off = align_up(off + 4 * ((size_t)T + 1), 64);
    h->off_woff = (int64_t)off;
    off = align_up(off + 4 * ((size_t)T + 1), 64);
    h->off_report = (int64_t)off;
    off = align_up(off + (size_t)T, 64);
    h->off_owner = (int64_t)off;
    off = align_up(off + 4 * (size_t)(R + W), 64);
    h->off_tail = (int64_t)off;
    h->tail_bytes = tail;
    off = align_up(off + (size_t)tail + 64, 64);  // slack for dkey.h tail_word
    h->bytes = (int64_t)off;
    return off;
}

static int64_t packed_tail_bytes(const fdbcs_packed_batch* pb) {
    const int32_t T = pb->n_txn;
    const int64_t nk = T > 0 ? 2 * ((int64_t)pb->read_offsets[T] + pb->write_offsets[T]) : 0;
    int64_t tail = 0;
    for (int64_t k = 0; k < nk; k++) {
        const int64_t len = pb->key_offsets[k + 1] - pb->key_offsets[k];
        if (len > 16) tail += len - 16;
    }
    return tail;
}

int fdbcs_share_bytes(const fdbcs_packed_batch* pb, int64_t* out) {
    if (!pb || !out || pb->n_txn < 0) return FDBCS_E_INVALID;
    if (pb->n_txn > 0 && (!pb->read_offsets || !pb->write_offsets || !pb->key_offsets)) return FDBCS_E_INVALID;
    const int32_t T = pb->n_txn;
    ShareHeader h{};
    *out = (int64_t)share_layout(T, T ? pb->read_offsets[T] : 0, T ? pb->write_offsets[T] : 0, packed_tail_bytes(pb), &h);
    return FDBCS_OK;
}

int fdbcs_share_pack(const fdbcs_packed_batch* pb, void* out, int64_t cap, int64_t* used) {
    if (!pb || !out || pb->n_txn < 0) return FDBCS_E_INVALID;
    const int32_t T = pb->n_txn;
    if (T > 0 && (!pb->read_snapshot || !pb->read_offsets || !pb->write_offsets || !pb->key_offsets))
        return FDBCS_E_INVALID;
    const int64_t R = T ? pb->read_offsets[T] : 0, W = T ? pb->write_offsets[T] : 0;
    const int64_t nk = 2 * (R + W);
    if (nk && !pb->key_bytes) return FDBCS_E_INVALID;
    for (int32_t t = 0; t < T; t++)
        if (pb->read_offsets[t + 1] < pb->read_offsets[t] || pb->write_offsets[t + 1] < pb->write_offsets[t])
            return FDBCS_E_INVALID;
    for (int64_t k = 0; k < nk; k += 2) {  // KeyRangeRef: begin <= end (FDBTypes.h:288-291)
        const int64_t a0 = pb->key_offsets[k], a1 = pb->key_offsets[k + 1], a2 = pb->key_offsets[k + 2];
        if (a1 < a0 || a2 < a1) return FDBCS_E_INVALID;
        if (cmp_bytes(pb->key_bytes + a0, (int32_t)(a1 - a0), pb->key_bytes + a1, (int32_t)(a2 - a1)) > 0)
            return FDBCS_E_INVALID;
    }
    ShareHeader h{};
    const size_t bytes = share_layout(T, R, W, packed_tail_bytes(pb), &h);
    if ((int64_t)bytes > cap) return FDBCS_E_NOMEM;
    char* o = (char*)out;
    memcpy(o, &h, sizeof(h));
    DKey* keys = (DKey*)(o + h.off_keys);
    uint8_t* tail = (uint8_t*)(o + h.off_tail);
    uint32_t tb = 0;
    for (int64_t k = 0; k < nk; k++) {
        const uint8_t* p = pb->key_bytes + pb->key_offsets[k];
        const uint32_t len = (uint32_t)(pb->key_offsets[k + 1] - pb->key_offsets[k]);
        DKey d;
        fast_prefix(p, len, &d.hi, &d.lo);
        d.len = len;
        d.tail = 0;
        if (len > 16) {
            d.tail = tb;
            memcpy(tail + tb, p + 16, len - 16);
            tb += len - 16;
        }
        keys[k] = d;
    }
    memset(tail + tb, 0, 64);
    if (T) {
        memcpy(o + h.off_snap, pb->read_snapshot, 8 * (size_t)T);
        memcpy(o + h.off_roff, pb->read_offsets, 4 * ((size_t)T + 1));
        memcpy(o + h.off_woff, pb->write_offsets, 4 * ((size_t)T + 1));
        if (pb->report_conflicting_keys)
            memcpy(o + h.off_report, pb->report_conflicting_keys, (size_t)T);
        else
            memset(o + h.off_report, 0, (size_t)T);
        int32_t* owner = (int32_t*)(o + h.off_owner);
        for (int32_t t = 0; t < T; t++) {
            for (int32_t r = pb->read_offsets[t]; r < pb->read_offsets[t + 1]; r++) owner[r] = t;
            for (int32_t w = pb->write_offsets[t]; w < pb->write_offsets[t + 1]; w++) owner[R + w] = t;
        }
    }
    if (used) *used = (int64_t)bytes;
    return FDBCS_OK;
}

int fdbcs_batch_add_routed(fdbcs_batch* b, const void* shares, int64_t stride, int32_t n_shares, int32_t max_share_txns,
                           const uint8_t* lo_key, int32_t lo_len, const uint8_t* hi_key, int32_t hi_len, int32_t cap_txns,
                           int32_t cap_reads, int32_t cap_writes, int64_t cap_tail, uint8_t* conflict_out,
                           int64_t n_global, const uint32_t* ready_flag, uint32_t ready_value) {
    if (!b || !shares || stride <= (int64_t)sizeof(ShareHeader) || n_shares <= 0 || max_share_txns < 0 || cap_txns < 0 ||
        cap_reads < 0 || cap_writes < 0 || cap_tail < 0 || (lo_len > 0 && !lo_key) || (hi_len > 0 && !hi_key) ||
        n_global < 0 || (conflict_out && n_global > (int64_t)n_shares * max_share_txns))
        return FDBCS_E_INVALID;
    if (!b->cs || b->state != 0 || b->T() != 0 || b->direct) return FDBCS_E_STATE;
    if ((int64_t)cap_txns > kMaxTxnLds) return FDBCS_E_INVALID;
    if (lo_len >= 0 && hi_len >= 0 && cmp_bytes(lo_key, lo_len, hi_key, hi_len) >= 0) return FDBCS_E_INVALID;
    fdbcs_conflict_set* cs = b->cs;
    HIPOK(hipSetDevice(cs->device));
    BatchSlot* sl = b->slot;
    int rc;
    // bounds of this resolver's key range: prefixes by value, tails in a small device arena
    std::vector<uint8_t> want;
    auto put_len = [&](int32_t n) {
        for (int i = 0; i < 4; i++) want.push_back((uint8_t)((uint32_t)n >> (8 * i)));
    };
    put_len(lo_len);
    if (lo_len > 0) want.insert(want.end(), lo_key, lo_key + lo_len);
    put_len(hi_len);
    if (hi_len > 0) want.insert(want.end(), hi_key, hi_key + hi_len);
    RouteArgs a{};
    std::vector<uint8_t> btail;
    auto bound = [&](const uint8_t* k, int32_t len, DKey* d) {
        fast_prefix(k, (uint32_t)len, &d->hi, &d->lo);
        d->len = (uint32_t)len;
        d->tail = 0;
        if (len > 16) {
            d->tail = (uint32_t)btail.size();
            btail.insert(btail.end(), k + 16, k + len);
            while (btail.size() % 8) btail.push_back(0);
        }
    };
    a.has_lo = lo_len >= 0;
    a.has_hi = hi_len >= 0;
    if (a.has_lo) bound(lo_key, lo_len, &a.lo);
    if (a.has_hi) bound(hi_key, hi_len, &a.hi);
    btail.resize(btail.size() + 64, 0);
    if (want != cs->route_bounds) {
        if ((rc = sync_all(cs))) return rc;
        if ((rc = cs->route_btail.ensure(btail.size()))) return rc;
        HIPOK(hipMemcpy(cs->route_btail.p, btail.data(), btail.size(), hipMemcpyHostToDevice));
        cs->route_bounds = want;
    }
    a.btail = (const uint8_t*)cs->route_btail.p;
    // the routed batch's layout at capacity offsets (upload layout)
    const UploadLayout L = upload_layout((size_t)cap_txns, (size_t)cap_reads, (size_t)cap_writes, (size_t)cap_tail);
    if ((rc = ensure_slot(sl, L.total, (size_t)cap_txns, (size_t)cap_reads))) return rc;
    const int64_t n_elems = (int64_t)n_shares * max_share_txns;
    // ranges of one share: each takes 48 bytes of endpoint records, so the stride bounds them
    const int64_t rstride = std::max<int64_t>(1, (stride - (int64_t)sizeof(ShareHeader)) / (2 * (int64_t)sizeof(DKey)));
    if ((rc = sl->rt_scan.ensure(8 * (size_t)route_scan_words(n_elems)))) return rc;
    if ((rc = sl->rt_info.ensure(4 * (size_t)(n_shares * rstride)))) return rc;
    if ((rc = sl->rt_txpre.ensure(16 * (size_t)std::max<int64_t>(n_elems, 1)))) return rc;
    if ((rc = sl->rt_inv.ensure(4 * (size_t)std::max<int64_t>(n_elems, 1)))) return rc;
    if ((rc = sl->rt_rids.ensure(4 * ((size_t)cap_reads + 1)))) return rc;
    if ((rc = sl->rt_dres.ensure(sizeof(RouteResult)))) return rc;
    if ((rc = sl->rt_res.ensure(sizeof(RouteResult), true))) return rc;
    if ((rc = make_slot_events(sl))) return rc;
    if (!sl->ev_rt0) HIPOK(hipEventCreate(&sl->ev_rt0));
    if (!sl->ev_rt1) HIPOK(hipEventCreate(&sl->ev_rt1));
    const auto t_host = std::chrono::steady_clock::now();
    char* d = (char*)sl->dev.p;
    a.shares = (const uint8_t*)shares;
    a.stride = stride;
    a.n_shares = n_shares;
    a.tcap = std::max(1, max_share_txns);
    a.report_enabled = 0;  // conflicting-key reports go through the host-routed path (sharding.py)
    a.cap_T = cap_txns;
    a.cap_R = cap_reads;
    a.cap_W = cap_writes;
    a.cap_tail = cap_tail;
    a.keys = (DKey*)(d + L.keys);
    a.info = (uint32_t*)sl->rt_info.p;
    a.rstride = rstride;
    a.txpre = (int4*)sl->rt_txpre.p;
    a.rown = (int32_t*)(d + L.rown);
    a.wown = (int32_t*)(d + L.wown);
    a.snap = (int64_t*)(d + L.snap);
    a.roff = (int32_t*)(d + L.roff);
    a.woff = (int32_t*)(d + L.woff);
    a.flags = (uint8_t*)(d + L.flags);
    a.tail = (uint8_t*)(d + L.tail);
    a.inv = (int32_t*)sl->rt_inv.p;
    a.inv_n = std::max<int64_t>(n_elems, 1);
    a.read_ids = (int32_t*)sl->rt_rids.p;
    a.out_zero = conflict_out;
    a.out_n = n_global;
    a.res = (RouteResult*)sl->rt_res.dp;
    a.dres = (RouteResult*)sl->rt_dres.p;
    ((RouteResult*)sl->rt_res.p)->error = -1;  // not written yet
    hipStream_t us = cs->ustream;
    // the shares are complete once *ready_flag == ready_value (k_route_wait); the slot's previous
    // batch may still read its device buffer
    a.ready = ready_flag;
    a.ready_value = ready_value;
    a.wait_ticks = (uint64_t)cs->route_timeout_ms * 100000ull;  // 100 MHz wall clock
    a.wait_err = (uint32_t*)((uint64_t*)sl->rt_scan.p + 2);
    HIPOK(hipMemsetAsync(sl->rt_scan.p, 0, 8 * (size_t)route_scan_words(n_elems), us));
    // global indices past the shares' transactions stay "not routed here"
    HIPOK(hipMemsetAsync(sl->rt_inv.p, 0xFF, 4 * (size_t)a.inv_n, us));
    uint64_t* sw = (uint64_t*)sl->rt_scan.p;
    ScanState st{sw + 8, (int*)sw, (int*)(sw + 1)};
    t_record = nullptr;
    HIPOK(hipEventRecord(sl->ev_rt0, us));
    launch_route(us, a, st);
    HIPOK(take_launch_error());
    HIPOK(hipEventRecord(sl->ev_rt1, us));
    sl->rt_timed = true;
    HIPOK(hipEventRecord(sl->ev_up, us));
    cs->stats.host_ms_route += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host).count();
    b->bd.keys = a.keys;
    b->bd.rowner = a.rown;
    b->bd.wowner = a.wown;
    b->bd.snap = a.snap;
    b->bd.roff = a.roff;
    b->bd.woff = a.woff;
    b->bd.flags = a.flags;
    b->bd.tail = a.tail;
    b->routed = true;
    b->route_pending = true;
    b->rT = b->rR = b->rW = 0;
    b->out_dev = conflict_out;
    b->out_n = n_global;
    b->out_ids.clear();
    b->state = 1;
    return FDBCS_OK;
}

// Sizes of a routed batch, once its route kernels are done (blocks until then).
static int finish_route(fdbcs_batch* b) {
    if (!b->route_pending) return FDBCS_OK;
    BatchSlot* sl = b->slot;
    HIPOK(hipEventSynchronize(sl->ev_up));
    std::atomic_thread_fence(std::memory_order_acquire);
    RouteResult r;
    memcpy(&r, (const void*)sl->rt_res.p, sizeof(r));
    if (r.error != 0) {
        // 2: the shares never arrived; 1: the routed part exceeds the capacities given; 3: n_global
        // differs from the shares' transaction count.  Whatever the routing kernels placed is
        // unusable either way: the batch goes back to the empty state, so it can be routed again
        // (with corrected arguments) or destroyed, never detected half-routed.
        if (r.error == 2) fprintf(stderr, "fdbcs: routed batch: the shares' ready flag was never set\n");
        b->routed = b->route_pending = false;
        b->out_dev = nullptr;
        b->out_n = 0;
        b->state = 0;
        return r.error == 2 ? FDBCS_E_TIMEOUT
                            : r.error == 1 ? FDBCS_E_NOMEM : r.error == 3 ? FDBCS_E_INVALID : FDBCS_E_DEVICE;
    }
    b->rT = r.T;
    b->rR = r.R;
    b->rW = r.W;
    b->r_tail = (size_t)r.tail_bytes;
    b->tail_bytes = b->r_tail;
    b->bd.tail_n = r.tail_bytes;
    b->bd.T = r.T;
    b->bd.R = r.R;
    b->bd.W = r.W;
    // history tail bytes the batch's write endpoints can add, each tail padded to 8 (a bound: the
    // kept tails plus 7 bytes of padding per write endpoint)
    b->wtail = r.tail_bytes + 14 * (int64_t)r.W;
    b->max_len = r.n_gt24 ? 25 : (r.n_gt19 ? 20 : 16);
    b->any_report = r.reports > 0;
    b->route_pending = false;
    return FDBCS_OK;
}

int fdbcs_batch_routed_info(fdbcs_batch* b, int32_t* T, int32_t* R, int32_t* W, void** inv_dev, void** read_ids_dev) {
    if (!b) return FDBCS_E_INVALID;
    if (!b->routed) return FDBCS_E_STATE;
    if (int rc = finish_route(b)) return rc;
    if (T) *T = b->rT;
    if (R) *R = b->rR;
    if (W) *W = b->rW;
    if (inv_dev) *inv_dev = b->slot->rt_inv.p;
    if (read_ids_dev) *read_ids_dev = b->slot->rt_rids.p;
    return FDBCS_OK;
}

int fdbcs_sync(fdbcs_conflict_set* cs) {
    if (!cs) return FDBCS_E_INVALID;
    HIPOK(hipSetDevice(cs->device));
    return sync_all(cs);
}

int fdbcs_batch_upload(fdbcs_batch* b) {
    if (!b) return FDBCS_E_INVALID;
    if (!b->cs) return FDBCS_E_STATE;
    if (b->state != 0) return b->state == 1 ? FDBCS_OK : FDBCS_E_STATE;
    HIPOK(hipSetDevice(b->cs->device));
    return do_upload(b, b->cs->ustream);
}


int fdbcs_batch_detect_async(fdbcs_batch* b, int64_t now, int64_t new_oldest_version) {
    if (!b) return FDBCS_E_INVALID;
    if (!b->cs) return FDBCS_E_STATE;
    if (b->state > 1) return FDBCS_E_STATE;
    fdbcs_conflict_set* cs = b->cs;
    const auto t_begin = std::chrono::steady_clock::now();
    HIPOK(hipSetDevice(cs->device));
    if (now < cs->max_written) return FDBCS_E_VERSION;
    if (int rc0 = finish_route(b)) return rc0;  // a routed batch's sizes (its route ran ahead)
    if (b->T() > kMaxTxnLds) return FDBCS_E_INVALID;
    // tail offsets are 32-bit: refuse a batch that could overflow the arena (GC repacks it long before)
    // history tail bytes this batch can append (each inserted tail padded to 8 bytes)
    // only write endpoints ever enter the history (merge inserts segment begins and ends)
    const int64_t tail_add = b->wtail;
    if (cs->tail_ub + tail_add + 1 >= kTailLimit) return FDBCS_E_NOMEM;
    const int64_t T = b->T(), R = b->R(), W = b->W();
    int rc;
    if ((rc = ensure_workspace(cs, T, R, W))) return rc;
    if ((rc = ensure_btail(cs, (int64_t)b->tail_size()))) return rc;
    if ((rc = ensure_delta(cs, cs->nd_ub + 2 * W + 1))) return rc;
    if ((rc = ensure_history(cs, cs->n_ub + cs->nd_ub + 2 * W + 1, cs->tail_ub + tail_add + 1)))
        return rc;
    if ((rc = ensure_events(b))) return rc;
    if (cs->ddir_counter == UINT32_MAX && cs->edir[0].p) {
        // the delta directory's 32-bit epoch tag is about to wrap: clear every entry (once per 2^32
        // batches) so that no entry left by an old fill can carry the reused epoch value
        if ((rc = sync_all(cs))) return rc;
        for (int k = 0; k < 2; k++) HIPOK(hipMemsetAsync(cs->edir[k].p, 0, 8 * (size_t)kDirAlloc, cs->stream));
        HIPOK(hipStreamSynchronize(cs->stream));
        cs->ddir_counter = 0;
    }
    // results (host-mapped; verdicts written by k_resolve, scalars and flag by the epilogue):
    // verdicts | scalars | completion flag, then the
    // report copies rconf | hist | first_conf
    const ResultLayout RL = result_layout(T, R);
    const size_t o_sc = RL.sc, o_fl = RL.fl, o_rc = RL.rc, o_hc = RL.hc, o_fc = RL.fc, out_bytes = RL.total;
    BatchSlot* sl = b->slot;
    if ((rc = sl->pin_out.ensure(out_bytes, true))) return rc;
    char* ho = (char*)sl->pin_out.p;
    b->h_verdict = (uint8_t*)ho;
    b->h_scal = (Scalars*)(ho + o_sc);
    b->h_flag = (volatile uint32_t*)(ho + o_fl);
    b->h_rconf = (uint8_t*)(ho + o_rc);
    b->h_hist = (uint8_t*)(ho + o_hc);
    b->h_first = (int32_t*)(ho + o_fc);
    if ((rc = sl->dverdict.ensure(T + 64))) return rc;
    if (b->out_dev && b->out_n > 0 && !b->routed) {
        // global -> batch transaction map, read by k_conflict_output straight from host-mapped
        // memory (n_global * 4 bytes; the slot's previous batch finished with it: its flag was seen)
        if ((int64_t)b->out_ids.size() != T) return FDBCS_E_STATE;  // transactions added after the call
        if ((rc = sl->pin_inv.ensure(4 * (size_t)b->out_n + 64, true))) return rc;
        int32_t* inv = (int32_t*)sl->pin_inv.p;
        std::fill(inv, inv + b->out_n, -1);
        for (int32_t t = 0; t < (int32_t)T; t++) inv[b->out_ids[t]] = t;
    }
    if (!b->routed) {  // (a routed batch's count came with its sizes)
        b->any_report = b->n_report > 0;  // (counted as the transactions were added)
    }
    b->seq = ++cs->seq;
    if (b->seq == 0) b->seq = ++cs->seq;  // 0 means "not done"
    *b->h_flag = 0;
    b->recorded = 0;

    hipStream_t s = cs->stream;
    const int timing = cs->timing;
    // Stage A (sort, positions, candidate edges) depends only on this batch: it runs on its own
    // stream and overlaps stage B of the previous batch.  Phase timing (level 2) runs both stages on
    // one stream so the phases are measured one after another.
    hipStream_t sa = (timing == 2 || cs->serial) ? s : cs->astream;  // level 3 keeps the timed layout
    const int wp = cs->wpar;
    cs->wpar = (wp + 1) % kNumWork;
    b->wp = wp;
    Work& w = cs->work[wp];
    // write groups need the group minima in the resolver's LDS beside the status bytes
    w.groups = cs->write_groups && W > 0 && W <= kMaxGroupWrites && T <= kMaxTxnLds ? 1 : 0;
    // phase events: level 2 records every phase, level 1 only the hot kernels (roofline)
    // level-1 (roofline) events on one batch in timing_every: each event record is a runtime call
    // on the submitting thread, and the per-launch averages need only a sample of the batches
    const bool sampled = timing >= 2 || b->seq % (uint32_t)kTimingEvery == 0;
    // level 3 (per-kernel profile) records only the events around every kernel
    // level 1 with a timed kernel (fdbcs_set_timed_kernel) records only that kernel's events
    auto rec = [&](int ph, int level) -> hipEvent_t {
        if (timing == 3 || timing < level || (level == 1 && (!sampled || cs->timed_func))) return nullptr;
        b->recorded |= 1u << ph;
        return sl->ev[ph];
    };
    auto mark = [&](int ph) -> int {
        if (hipEvent_t e = rec(ph, 2)) fdb_event(LaunchList::kTimingRecord, e, s);
        return FDBCS_OK;
    };
    const bool was_uploaded = b->state == 1;
    LaunchList& la = cs->rec_a;
    LaunchList& lb = cs->rec_b;
    LaunchList& lc = cs->rec_c;
    LaunchList& ly = cs->rec_y;
    la.clear();
    lb.clear();
    lc.clear();
    ly.clear();
    // per-kernel events: every kernel at level 3, the kernel fdbcs_set_timed_kernel named at level 1
    // (sampled batches)
    sl->prof_next = 0;
    sl->prof_spans.clear();
    const bool kprof = timing == 3 || (timing == 1 && sampled && cs->timed_func);
    for (LaunchList* L : {&la, &lb, &lc, &ly}) {
        L->prof = kprof ? &sl->prof : nullptr;
        L->timed_func = timing == 3 ? nullptr : cs->timed_func;
    }
    // Split read check: the base tier changes only at compactions, so unless one is still pending
    // on the stream its half of D.CheckRead runs beside stage A on its own stream; stage B keeps the
    // delta half.
    const bool split = (cs->split_check == 1 || (cs->split_check == 2 && cs->n_ub >= kSplitCheckMinBase)) &&
                       !cs->serial && timing != 2;
    // two submitting threads: this batch's stage A and check go out from the helper, stage B on the
    // next call.  The previous batch's stage B is recorded but maybe not issued yet, so an event it
    // records cannot be queried here: waits on its events are kept unconditionally.
    const bool threaded = cs->submit_thread && timing < 2 && !cs->trace && sa != s;
    cs->stats.host_ms_prepare += host_ms_since(t_begin);
    const auto t_rec = std::chrono::steady_clock::now();
    // ---- upload (issued now) and record stage A: D.Sort and the candidate edges of D.CheckIntraBatch
    // The upload runs on its own stream unless the phases are timed one after another (then on
    // stage A's stream, bracketed by the upload phase's events).
    const bool own_upload = timing != 2 && !cs->serial;
    if (hipEvent_t e = rec(kPhStart, 2)) HIPOK(hipEventRecord(e, sa));
    if (b->state == 0 && (rc = do_upload(b, own_upload ? cs->ustream : sa))) return rc;
    if (hipEvent_t e = rec(kPhUpload, 2)) HIPOK(hipEventRecord(e, sa));
    t_record = &la;
    // workspace wp was last used by the batch before the previous one: its epilogue re-zeroed it.
    // ev_b[wp] is recorded by every batch's stage B, whatever its stream layout, so the query is
    // never answered by a stale or never-recorded event (a timing-level change with batches in
    // flight included).
    const bool ws_busy = cs->wused[wp] && (threaded || !stage_b_done(cs, wp));
    if (ws_busy && (sa != s || cs->y_async[wp])) fdb_event(LaunchList::kSyncWait, cs->ev_b[wp], sa);
    // and the check after that batch may still read its union segments and their tails
    if (cs->xfree_rec[wp] && sa != s && (threaded || !batch_done(cs->xfree_user[wp])))
        fdb_event(LaunchList::kSyncWait, cs->xfree_ev[wp], sa);
    cs->xfree_rec[wp] = false;
    cs->wused[wp] = true;
    cs->ws_user[wp] = b;
    // stage A reads the batch: wait for the upload stream
    if (own_upload || (was_uploaded && hipEventQuery(sl->ev_up) != hipSuccess))
        fdb_event(LaunchList::kSyncWait, sl->ev_up, sa);
    const BatchDev& bd = b->bd;
    // a routed batch's TooOld test (SkipList.cpp:770) against the oldest version every earlier
    // detect left (its routing may have run before the previous batch's detect): stage A, ahead
    // of every kernel that reads the flags (stage B)
    if (b->routed) launch_route_too_old(sa, bd, cs->oldest);
    // long-key probes pay off once tails run past a word (a 17-byte end key k\0 of a 16-byte key
    // ties on the prefix with k only, and the length decides)
    const bool long_keys = b->max_len > 24;
    Scalars* sc = (Scalars*)cs->scal.p;
    const int bsrc = cs->cur, dsrc = cs->dcur;
    // Stage B in two halves (fdbcs_conflict_set::ystream): X = check, resolution, D.Combine on
    // `stream`; Y = merge, compaction / GC, epilogue on `ystream`.  Unless the previous batch
    // compacted, this batch's check reads the delta before the previous batch's merge (buffer
    // dsrc ^ 1, complete once the batch before it finished Y) plus the previous batch's union
    // segments at its `now` (PrevSegs): the same history, so the check need not wait for that merge.
    const bool pipe = !(timing == 2 || cs->serial);
    hipStream_t ys = pipe ? cs->ystream : s;
    const bool use_prev = pipe && cs->prev_segs;
    const int dchk = use_prev ? dsrc ^ 1 : dsrc;
    const Tier base{hist_of(cs, bsrc), levels_of(cs, bsrc), &sc->n, cs->header_version};
    const Tier delta{delta_of(cs, dsrc), dlevels_of(cs, dsrc), &sc->ndb[dsrc], kHole};
    const Tier cdelta{delta_of(cs, dchk), dlevels_of(cs, dchk), &sc->ndb[dchk], kHole};  // what the check reads
    PrevSegs ps{};
    if (use_prev) {
        const Work& pw = cs->work[cs->prev_wp];
        ps = PrevSegs{pw.segk, pw.btail, &pw.bsc->n_segments, cs->prev_now};
    }
    uint8_t* htail = (uint8_t*)cs->htail[cs->tcur].p;

    w.trace = cs->trace ? (unsigned long long*)cs->trace_buf.p : nullptr;
    w.no_prepass = cs->no_prepass ? 1 : 0;
    if (w.trace) {
        HIPOK(hipStreamSynchronize(cs->astream));
        HIPOK(hipStreamSynchronize(s));
        unsigned long long init[kTrSlots];
        for (int i = 0; i < kTrSlots; i++)
            init[i] = (i == kTrSampleBegin || i == kTrCheckBegin || i == kTrEpiBegin || i == kTrResBegin || i == kTrResW0min ||
                       i == kTrPartBegin || i == kTrBktBegin)
                          ? ~0ull
                          : 0ull;
        HIPOK(hipMemcpy(w.trace, init, sizeof(init), hipMemcpyHostToDevice));
    }
    // D.Sort and the sorted positions.  Splitters: the quantiles the last batch of >= kQuantMinE
    // endpoints left (stage A runs in batch order on one stream), or this batch's ranked samples
    // when there are none yet (cold start)
    int sort_nb = 0, sort_samples = 0;  // what the epilogue re-zeroes of the sort's scratch
    {
        const int64_t E = 2 * (R + W);
        const int nbk = sort_bucket_count(E, cs->bucket_target, w.slab_buckets);
        const bool cold = nbk > 1 && (cs->sort_cold || !cs->quant_valid);
        sort_nb = E > 0 ? nbk : 0;
        sort_samples = E > 0 && cold ? sort_cold_samples(E, nbk) : 0;
        const bool write_quant = E >= kQuantMinE;
        SplitKey* qt = (SplitKey*)cs->quant.p;
        if (cs->quant_sa && cs->quant_sa != sa) {
            // the splitter tables were last read and written by a sort on another stream: order
            // this sort after it (every stage A before this one has been issued: flush the helper)
            if ((rc = flush_pending(cs))) return rc;
            HIPOK(hipEventRecord(cs->ev_quant, cs->quant_sa));
            fdb_event(LaunchList::kSyncWait, cs->ev_quant, sa);
        }
        cs->quant_sa = sa;
        launch_sort(sa, bd, w, qt + cs->qcur * kQuant, write_quant ? qt + (cs->qcur ^ 1) * kQuant : nullptr, cold,
                    cs->bucket_target, b->max_len > (int32_t)kSortNxLen, cs->validate, rec(kPhSortBegin, 1),
                    rec(kPhSortEnd, 1));
        if (write_quant) {
            cs->qcur ^= 1;
            cs->quant_valid = true;
        }
    }
    mark(kPhSort);
    if (cs->validate) launch_validate_sort(sa, bd, w);
    w.hseq = b->seq;  // (Work is passed by value: the edge scan's finish tags its host word)
    launch_edges(sa, bd, w);
    if (sa != s) fdb_event(LaunchList::kSyncRecord, cs->ev_a[wp], sa);
    mark(kPhEdges);
    if (split) {  // ---- record the base-tier check (its own stream)
        t_record = &lc;
        hipStream_t sc_ = cs->cstream;
        fdb_event(LaunchList::kSyncWait, sl->ev_up, sc_);
        if (ws_busy) fdb_event(LaunchList::kSyncWait, cs->ev_b[wp], sc_);
        if (cs->cmp_recorded && (threaded || hipEventQuery(cs->ev_cmp) != hipSuccess))
            fdb_event(LaunchList::kSyncWait, cs->ev_cmp, sc_);
        fdb_event(LaunchList::kTimingRecord, rec(kPhCheckBegin, 1), sc_);
        launch_check_tier(sc_, bd, w, base, true, htail, long_keys, PrevSegs{});
        fdb_event(LaunchList::kTimingRecord, rec(kPhCheckEnd, 1), sc_);
        fdb_event(LaunchList::kSyncRecord, cs->ev_c[wp], sc_);
    }
    // ---- record stage B, half X: D.CheckRead, then batch order
    t_record = &lb;
    if (sa == s || !was_uploaded || hipEventQuery(sl->ev_up) != hipSuccess) fdb_event(LaunchList::kSyncWait, sl->ev_up, s);
    {
        // the delta the check reads is complete: Y of the batch before the previous one (with the
        // previous batch's segments), or of the previous batch (it compacted, or nothing pending).
        // Only a Y on ystream needs the event (a timing-level change may switch layouts mid-flight).
        const int wy = use_prev ? cs->prev2_wp : cs->last_wp;
        if (wy >= 0 && cs->y_async[wy] && (threaded || !stage_b_done(cs, wy)))
            fdb_event(LaunchList::kSyncWait, cs->ev_b[wy], s);
    }
    if (split) {
        b->check_hist = cs->n_ub;  // the timed (base-tier) check
        launch_check_tier(s, bd, w, cdelta, false, htail, long_keys, ps);
    } else {
        b->check_hist = cs->n_ub + cs->nd_ub;
        fdb_event(LaunchList::kTimingRecord, rec(kPhCheckBegin, 1), s);
        launch_check(s, bd, w, base, cdelta, htail, long_keys, ps);
        fdb_event(LaunchList::kTimingRecord, rec(kPhCheckEnd, 1), s);
    }
    if (use_prev) {  // the previous batch's workspace may be reused once this check is done with it
        cs->xfree_ev[cs->prev_wp] = cs->ev_res[wp];  // recorded at the end of this half X
        cs->xfree_user[cs->prev_wp] = b;
        cs->xfree_rec[cs->prev_wp] = true;
    }
    mark(kPhCheck);
    if (sa != s) fdb_event(LaunchList::kSyncWait, cs->ev_a[wp], s);
    if (split) fdb_event(LaunchList::kSyncWait, cs->ev_c[wp], s);
    w.vdev = (uint8_t*)sl->dverdict.p;  // (Work by value: the resolution's launches carry it)
    launch_resolve(s, bd, w, b->any_report, (uint8_t*)sl->pin_out.dp, sc);
    w.vdev = nullptr;
    if (b->out_dev && b->out_n > 0)  // multi-resolver combine input, final before the completion flag
        launch_conflict_output(s, bd, w, b->routed ? (const int32_t*)sl->rt_inv.p : (const int32_t*)sl->pin_inv.dp,
                               b->out_n, b->out_dev);
    if (b->any_report) {  // before the epilogue re-zeroes hist_conf (into the host-mapped results)
        char* hdv = (char*)sl->pin_out.dp;
        if (R) launch_copy_bytes(s, hdv + o_rc, w.rconf, R);
        launch_copy_bytes(s, hdv + o_hc, w.hist_conf, T);
        launch_copy_bytes(s, hdv + o_fc, w.first_conf, 4 * T);
    }
    mark(kPhIntra);
    mark(kPhCombine);
    // ---- half Y: D.MergeWrite, compaction / GC, epilogue, after X
    fdb_event(LaunchList::kSyncRecord, cs->ev_res[wp], s);
    t_record = &ly;
    if (ys != s) fdb_event(LaunchList::kSyncWait, cs->ev_res[wp], ys);
    const int dnew = dsrc ^ 1;
    const int64_t nd_after = cs->nd_ub + 2 * W;
    const int64_t new_oldest = std::max(cs->oldest, new_oldest_version);
    // Compaction when the delta may outgrow its bound (or on the forced cadence); removeBefore
    // (SkipList.cpp:880-889) runs with it whenever the oldest version moved.
    bool compact = nd_after > delta_limit_for(cs, cs->n_ub);
    if (cs->gc_interval > 0 && ++cs->batches_since_compact >= cs->gc_interval) compact = true;
    if (cs->tail_ub > cs->tail_reclaim) compact = true;
    // D.MergeWrite into the delta tier
    char* hd = (char*)sl->pin_out.dp;
    launch_merge(ys, bd, w, delta.h, delta.m, delta_of(cs, dnew), dlevels_of(cs, dnew), &sc->ndb[dsrc], htail, sc, now,
                 cs->dlvl3_n, cs->dlvl2_n, cs->nd_ub + 1, rec(kPhCopyBegin, 1), rec(kPhCopyEnd, 1), long_keys);
    mark(kPhMerge);
    bool gc = false;
    int final_base = bsrc;
    const int64_t base_hint = cs->n_ub + nd_after + 1;
    if (compact) {
        launch_compact(ys, w, base.h, base.m, delta_of(cs, dnew), hist_of(cs, bsrc ^ 1), htail, sc,
                       cs->header_version, cs->lvl3_n, cs->lvl2_n, nd_after + 1, cs->n_ub + 1, rec(kPhCompBegin, 1),
                       rec(kPhCompEnd, 1), long_keys ? 2 : 1, cs->n_ub <= (16 << 20) ? 1024 : 4096,
                       cs->n_ub > (16 << 20));
        final_base = bsrc ^ 1;
        cs->batches_since_compact = 0;
        // Size-triggered compactions (gc_interval 0) run removeBefore on every kGcEveryCompactions-th
        // one: a full pass over the base costs ~10x the compaction copy at C2 while one
        // window-step of oldest-version movement makes few boundaries removable (a boundary goes
        // only when it and its predecessor are both older, SkipList.cpp:555-561). Verdict-neutral
        // either way; a forced cadence (gc_interval > 0) keeps GC at every compaction.  Past the
        // tail-reclaim threshold the GC also repacks the tail arena.
        const bool gc_turn = cs->gc_interval > 0 || ++cs->compactions_since_gc >= kGcEveryCompactions;
        gc = (new_oldest > cs->gc_applied && gc_turn) || cs->tail_ub > cs->tail_reclaim;
        if (gc) cs->compactions_since_gc = 0;
    }
    mark(kPhCompact);
    if (gc) {
        launch_gc(ys, w, hist_of(cs, final_base), hist_of(cs, final_base ^ 1), htail,
                  (uint8_t*)cs->htail[cs->tcur ^ 1].p, sc, std::max(new_oldest, cs->gc_applied), cs->header_version,
                  base_hint);
        cs->tcur ^= 1;
        final_base ^= 1;
        cs->gc_applied = new_oldest;
    }
    mark(kPhGc);
    b->gc_ran = gc;
    b->compacted = compact;
    // the epilogue that rebuilds the delta tier's index also fills its directory under a new epoch
    // (a compaction leaves none).  The epoch tag is 32 bits: before it wraps, every entry is
    // cleared (ensure_delta_directory), so a slot an old fill left behind is never trusted.
    if (compact || !cs->edir[dnew].p) {
        cs->ddir_epoch[dnew] = 0;
    } else {
        cs->ddir_epoch[dnew] = ++cs->ddir_counter;
    }
    launch_epilogue(ys, bd, w, compact ? levels_of(cs, final_base) : dlevels_of(cs, dnew), sc, compact ? 1 : 0,
                    gc ? 1 : 0, (uint8_t*)hd, (uint32_t*)(hd + o_fl), b->seq,
                    compact ? base_hint : nd_after + 1, &sc->ndb[dnew], sort_nb, sort_samples);
    fdb_event(LaunchList::kSyncRecord, cs->ev_b[wp], ys);
    // (no event marks the slot free: a slot returns to the pool only from fdbcs_batch_destroy,
    // after the batch's completion flag was seen or its streams were synchronized; every kernel
    // of the batch that reads or writes the slot precedes the epilogue, which touches none of it)
    if (compact || gc) {  // later base-tier checks wait for this rewrite of the base
        fdb_event(LaunchList::kSyncRecord, cs->ev_cmp, ys);
        cs->cmp_recorded = true;
    }
    mark(kPhEpilogue);
    mark(kPhEnd);
    t_record = nullptr;
    cs->stats.host_ms_record += host_ms_since(t_rec);
    const auto t_sub = std::chrono::steady_clock::now();
    // ---- submit
    if (threaded) {
        // the helper issues this batch's stage A and check while this thread issues the
        // previous batch's stage B; this batch's stage B waits for the next call (or a flush)
        if ((rc = worker_wait(cs))) return rc;
        std::swap(cs->work_a, la);
        std::swap(cs->work_c, lc);  // empty unless split
        cs->work_sa = sa;
        cs->work_a_seq = b->seq;
        const bool prev = cs->pending_batch != nullptr;
        if (prev) {  // the previous batch's Y to the helper, after the X this thread issues below
            cs->work_y_seq = cs->pending_batch->seq;
            std::swap(cs->work_y, cs->pending_y);
            cs->work_ys = cs->pending_ys;
            cs->work_need_x = cs->x_issued.load(std::memory_order_relaxed) + 1;
            cs->work_y_batch = cs->pending_batch;
        }
        cs->work_need_b = cs->b_recorded;  // every stage B recorded so far, batch i-1's included
        worker_start_job(cs);
        if (prev) {
            fdbcs_batch* pb_ = cs->pending_batch;
            cs->pending_batch = nullptr;
            const int64_t tx = cs->htrace ? mono_ns() : 0;
            const uint32_t pseq = pb_->seq;
            hipError_t e = cs->pending_b.replay(s, x_skip(cs, pb_), &cs->stats.x_launches_skipped);
            if (cs->htrace) cs->htr[0].push_back({pseq, 'X', tx, mono_ns()});
            cs->x_issued.fetch_add(1, std::memory_order_release);  // (the helper issues its Y)
            if (e != hipSuccess) return FDBCS_E_DEVICE;
        }
        std::swap(cs->pending_b, lb);
        std::swap(cs->pending_y, ly);
        cs->pending_ys = ys;
        cs->b_recorded++;
        cs->pending_batch = b;
    } else if (flush_pending(cs)) {
        return FDBCS_E_DEVICE;
    } else {
        HIPOK(la.replay(sa));
        if (split) HIPOK(lc.replay(cs->cstream));
        HIPOK(lb.replay(s));
        HIPOK(ly.replay(ys));
    }
    HIPOK(take_launch_error());
    cs->stats.host_ms_submit += host_ms_since(t_sub);
    cs->cur = final_base;
    cs->dcur = dnew;
    // the next batch's check: this batch's segments stand in for its merge unless it compacted
    cs->prev_segs = pipe && !compact;
    cs->prev2_wp = cs->last_wp;
    cs->last_wp = wp;
    cs->y_async[wp] = ys != s;
    cs->prev_wp = wp;
    cs->prev_now = now;
    cs->oldest = new_oldest;  // SkipList.cpp:880-882
    if (W) cs->max_written = std::max(cs->max_written, now);
    if (compact) {
        cs->n_ub += nd_after;
        cs->nd_ub = 0;
    } else {
        cs->nd_ub = nd_after;
    }
    cs->tail_ub += tail_add;
    cs->inflight++;
    b->state = 2;
    if (cs->htrace)
        cs->htr[0].push_back({b->seq, 'D',
                              (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_begin.time_since_epoch()).count(),
                              mono_ns()});
    return FDBCS_OK;
}

int fdbcs_batch_wait(fdbcs_batch* b, uint8_t* verdicts, int32_t* n_committed, int32_t* n_too_old) {
    if (!b) return FDBCS_E_INVALID;
    if (b->state == 2 && !b->cs) return FDBCS_E_STATE;
    fdbcs_conflict_set* cs = b->cs;
    if (b->state == 2) {
        const int64_t tw0 = cs->htrace ? mono_ns() : 0;
        HIPOK(hipSetDevice(cs->device));
        if (cs->pending_batch == b)  // its stage B still waits for the next detect: launch it now
            if (int rc = flush_pending(cs)) return rc;
        if (cs->work_y_batch == b)  // its Y is with the helper: issued (events and all) before reading them
            if (int rc = worker_wait(cs)) return rc;
        // the epilogue publishes b->seq; poll it, checking the streams for errors only every ~2 ms:
        // hipStreamQuery takes runtime locks the helper thread's launches need, so querying at
        // the spin rate slows the submission of the batches behind this one
        auto t_q = std::chrono::steady_clock::now();
        for (uint64_t spin = 0; *b->h_flag != b->seq; spin++) {
            __builtin_ia32_pause();
            if ((spin & 4095) != 4095) continue;
            if (std::chrono::steady_clock::now() - t_q < std::chrono::milliseconds(cs->wait_query_ms)) continue;
            t_q = std::chrono::steady_clock::now();
            {
                // the flag comes from the epilogue (stage B's Y half): done or failing once both
                // halves are idle
                hipError_t e = hipStreamQuery(cs->astream);
                if (e == hipSuccess || e == hipErrorNotReady) e = hipStreamQuery(cs->stream);
                if (e == hipSuccess) e = hipStreamQuery(cs->ystream);
                if (e != hipSuccess && e != hipErrorNotReady) {
                    fprintf(stderr, "fdbcs: stream error while waiting: %s\n", hipGetErrorString(e));
                    return FDBCS_E_DEVICE;
                }
                if (e == hipSuccess && *b->h_flag != b->seq) {
                    fprintf(stderr, "fdbcs: stream idle but batch %u not completed\n", b->seq);
                    return FDBCS_E_DEVICE;
                }
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (cs->htrace) cs->htr[0].push_back({b->seq, 'W', tw0, mono_ns()});
        if (cs->trace && cs->inflight == 1) {
            if (int rc = sync_all(cs)) return rc;
            unsigned long long tr[kTrSlots];
            HIPOK(hipMemcpy(tr, cs->trace_buf.p, sizeof(tr), hipMemcpyDeviceToHost));
            auto us = [&](int a, int z) { return (double)((long long)(tr[z] - tr[a])) / 100.0; };  // 100 MHz
            fprintf(stderr,
                    "fdbcs trace: sample %.2f us, check %.2f us (check starts %+.2f us after sample); epilogue "
                    "levels %.2f, zero %.2f, host %.2f, fence %.2f us\n",
                    us(kTrSampleBegin, kTrSampleEnd), us(kTrCheckBegin, kTrCheckEnd), us(kTrSampleBegin, kTrCheckBegin),
                    us(kTrEpiBegin, kTrEpiLevels), us(kTrEpiLevels, kTrEpiZero), us(kTrEpiZero, kTrEpiHost),
                    us(kTrEpiHost, kTrEpiFence));
            fprintf(stderr,
                    "fdbcs trace: sort partition fill %.2f, search %.2f, end %.2f us; bucket prologue %.2f, "
                    "sorted %.2f, ties %.2f, end %.2f us (partition start to bucket start %.2f us)\n",
                    us(kTrPartBegin, kTrPartFill), us(kTrPartBegin, kTrPartSearch), us(kTrPartBegin, kTrPartEnd),
                    us(kTrBktBegin, kTrBktPrologue), us(kTrBktBegin, kTrBktSorted), us(kTrBktBegin, kTrBktTies),
                    us(kTrBktBegin, kTrBktEnd),
                    us(kTrPartBegin, kTrBktBegin));
            {
                const double nw = tr[kTrBktWaves] ? (double)tr[kTrBktWaves] : 1.0;
                fprintf(stderr, "fdbcs trace: bucket tie runs: %llu lanes in runs, %llu ranked in registers, %llu serially, "
                        "longest run %llu\n", tr[kTrBktRuns], tr[kTrBktSimple], tr[kTrBktSlow], tr[kTrBktMaxRun]);
                fprintf(stderr,
                        "fdbcs trace: bucket per wave (%llu waves): load %.2f, sort %.2f, ties %.2f, put %.2f us\n",
                        tr[kTrBktWaves], tr[kTrBktSumLoad] / nw / 100.0, tr[kTrBktSumSort] / nw / 100.0,
                        tr[kTrBktSumTies] / nw / 100.0, tr[kTrBktSumPut] / nw / 100.0);
                const double np = tr[kTrPartWaves] ? (double)tr[kTrPartWaves] : 1.0;
                fprintf(stderr,
                        "fdbcs trace: partition per wave (%llu waves): fill %.2f, tail copy %.2f, search %.2f, "
                        "place %.2f us\n",
                        tr[kTrPartWaves], tr[kTrPartSumFill] / np / 100.0, tr[kTrPartSumCopy] / np / 100.0,
                        tr[kTrPartSumSearch] / np / 100.0, tr[kTrPartSumPlace] / np / 100.0);
            }
            fprintf(stderr, "fdbcs trace: resolve pre-pass %.2f us, wait %.2f us, rounds %.2f us (setup %.2f, first round "
                    "%.2f of which minima %.2f, %d rounds), finish %.2f us; waves start %.2f..%.2f us before the first kernarg use\n",
                    us(kTrResBegin, kTrResPre), us(kTrResPre, kTrResWait), us(kTrResWait, kTrResRounds),
                    us(kTrResWait, kTrResSetup), us(kTrResSetup, kTrResRound1), us(kTrResSetup, kTrResMin1),
                    (int)b->h_scal->intra_rounds,
                    us(kTrResRounds, kTrResEnd), us(kTrResW0min, kTrResWait), us(kTrResW0max, kTrResWait));
            fprintf(stderr, "fdbcs trace: combine chunk 0: loads %.2f, scan1 %.2f, scan2 %.2f, stores %.2f us\n",
                    us(kTrResRounds, kTrCmbLoad), us(kTrCmbLoad, kTrCmbScan1), us(kTrCmbScan1, kTrCmbScan2),
                    us(kTrCmbScan2, kTrCmbStore));


        }
        if (b->h_scal->debug_error) {
            fprintf(stderr, "fdbcs: device invariant check failed (debug_error=%d)\n", b->h_scal->debug_error);
            cs->inflight--;
            b->state = 3;
            return FDBCS_E_DEVICE;
        }
        const int32_t T = b->T();
        int32_t nc = 0, nt = 0;
        for (int32_t t = 0; t < T; t++) {
            nc += b->h_verdict[t] == FDBCS_TRANSACTION_COMMITTED;
            nt += b->h_verdict[t] == FDBCS_TRANSACTION_TOO_OLD;
        }
        b->n_committed = nc;
        b->n_too_old = nt;
        // conflictingKeyRangeMap: every conflicting read for history conflicts (SkipList.cpp:641-645),
        // the first for intra-batch conflicts (SkipList.cpp:821-828).
        b->conf_off.assign(T + 1, 0);
        b->conf_idx.clear();
        if (b->any_report) {
            for (int32_t t = 0; t < T; t++) {
                if ((b->flags[t] & kFlagReport) && b->h_verdict[t] == FDBCS_TRANSACTION_CONFLICT) {
                    if (b->h_hist[t]) {
                        for (int32_t r = b->roff[t]; r < b->roff[t + 1]; r++)
                            if (b->h_rconf[r]) b->conf_idx.push_back(r - b->roff[t]);
                    } else if (b->h_first[t] != INT_MAX) {
                        b->conf_idx.push_back(b->h_first[t]);
                    }
                }
                b->conf_off[t + 1] = (int32_t)b->conf_idx.size();
            }
        }
        // stats
        fdbcs_stats& st = cs->stats;
        st.batches++;
        st.transactions += T;
        st.read_ranges += b->R();
        st.write_ranges += b->W();
        // timing events may trail the completion flag: wait for the last one recorded
        for (int e : {(int)kPhEnd, (int)kPhCompEnd, (int)kPhCopyEnd, (int)kPhCheckEnd})
            if ((b->recorded >> e) & 1u) {
                HIPOK(hipEventSynchronize(b->slot->ev[e]));
                break;
            }
        for (const auto& sp : b->slot->prof_spans) {  // per-kernel events (levels 3 and 1)
            HIPOK(hipEventSynchronize(sp.second.second));
            const double ms = ev_ms(sp.second.first, sp.second.second);
            auto it = std::find_if(cs->kprof.begin(), cs->kprof.end(), [&](const auto& k) { return k.func == sp.first; });
            if (it == cs->kprof.end()) {
                cs->kprof.push_back({sp.first, 0, 0.0});
                it = cs->kprof.end() - 1;
            }
            it->launches += 1;
            it->ms += ms;
        }
        b->slot->prof_spans.clear();
        auto ph = [&](int a, int z) {
            return ((b->recorded >> a) & (b->recorded >> z) & 1u) ? ev_ms(b->slot->ev[a], b->slot->ev[z]) : 0.0;
        };
        st.ms_upload += ph(kPhStart, kPhUpload);
        st.ms_sort += ph(kPhUpload, kPhSort);
        st.ms_intra += ph(kPhSort, kPhEdges) + ph(kPhCheck, kPhIntra);
        st.ms_check_read += ph(kPhEdges, kPhCheck);
        st.ms_combine += ph(kPhIntra, kPhCombine);
        st.ms_merge += ph(kPhCombine, kPhMerge);
        st.ms_compact += ph(kPhMerge, kPhCompact);
        st.ms_gc += ph(kPhCompact, kPhGc);
        st.ms_epilogue += ph(kPhGc, kPhEpilogue);
        st.ms_total += ph(kPhUpload, kPhEnd);
        // roofline inputs: a kernel's launches, bytes and device time are counted together, on the
        // batches whose events were recorded (timing level 1 samples 1 batch in timing_every)
        if (b->h_scal->intra_edges < 0) {
            st.intra_fallbacks += 1;
        } else {
            st.intra_edges += b->h_scal->intra_edges;
            st.intra_rounds += b->h_scal->intra_rounds;
        }
        // algorithmic bytes of the copy kernels (roofline.py): read every kept old boundary and
        // every inserted one (its key from the batch), write every boundary of the result, 32 B
        // each (16 B key, 8 B length/tail, 8 B version); kept + inserted = the result's size
        {
            const int64_t kept = b->h_scal->d_before - b->h_scal->d_rem, out = b->h_scal->nd_next;
            const int64_t bytes = 32 * (kept + (out - kept) + out);
            st.merge_bytes_all += bytes;
            st.delta_sum += b->h_scal->d_before;
            st.base_sum += b->h_scal->n;
            st.segments_sum += b->h_scal->n_segments;
            if ((b->recorded >> kPhCopyEnd) & 1u) {
                st.ms_merge_kernel += ph(kPhCopyBegin, kPhCopyEnd);
                st.merge_launches += 1;
                st.merge_bytes += bytes;
            }
        }
        if ((b->recorded >> kPhCheckEnd) & 1u) {
            st.ms_check_kernel += ph(kPhCheckBegin, kPhCheckEnd);
            st.check_launches += b->R() > 0;
            st.check_reads += b->R();
            st.check_history += b->R() > 0 ? b->check_hist : 0;
        }
        if ((b->recorded >> kPhSortEnd) & 1u) {
            st.ms_sort_kernel += ph(kPhSortBegin, kPhSortEnd);
            st.sort_launches += 1;
            st.sort_items += 2 * (int64_t)(b->R() + b->W());
        }
        st.gc_runs += b->gc_ran ? 1 : 0;
        st.sort_big_buckets += b->h_scal->sort_big;
        if (b->routed && b->slot->rt_timed) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, b->slot->ev_rt0, b->slot->ev_rt1) == hipSuccess) st.ms_route_kernels += ms;
            st.routed_batches += 1;
            b->slot->rt_timed = false;
        }
        if (b->compacted) {
            st.compactions += 1;
            // kept base boundaries read, delta boundaries inserted read, result written
            const int64_t kept = b->h_scal->c_before - b->h_scal->c_rem;
            const int64_t bytes = 32 * (kept + (b->h_scal->n_next - kept) + b->h_scal->n_next);
            st.compact_bytes_all += bytes;
            if ((b->recorded >> kPhCompEnd) & 1u) {
                st.ms_compact_kernel += ph(kPhCompBegin, kPhCompEnd);
                st.compact_launches += 1;
                st.compact_bytes += bytes;
            }
        }
        cs->inflight--;
        if (cs->inflight == 0) {
            cs->n_ub = b->h_scal->n;
            cs->nd_ub = b->h_scal->nd;
            cs->tail_ub = b->h_scal->tail_used;
        }
        b->state = 3;
    }
    if (b->state != 3) return FDBCS_E_STATE;
    if (verdicts && b->T()) memcpy(verdicts, b->h_verdict, b->T());
    if (n_committed) *n_committed = b->n_committed;
    if (n_too_old) *n_too_old = b->n_too_old;
    return FDBCS_OK;
}

int fdbcs_batch_detect_conflicts(fdbcs_batch* b, int64_t now, int64_t new_oldest_version, uint8_t* verdicts,
                                 int32_t* n_committed, int32_t* n_too_old) {
    int rc = fdbcs_batch_detect_async(b, now, new_oldest_version);
    if (rc) return rc;
    return fdbcs_batch_wait(b, verdicts, n_committed, n_too_old);
}

int fdbcs_batch_conflicting_reads(fdbcs_batch* b, int32_t txn, int32_t* idx_out, int32_t cap, int32_t* n_out) {
    if (!b || !n_out) return FDBCS_E_INVALID;
    if (b->state != 3) return FDBCS_E_STATE;
    if (txn < 0 || txn >= b->T()) return FDBCS_E_INVALID;
    const int32_t a = b->conf_off[txn], e = b->conf_off[txn + 1];
    *n_out = e - a;
    if (idx_out)
        for (int32_t i = a; i < e && i - a < cap; i++) idx_out[i - a] = b->conf_idx[i];
    return FDBCS_OK;
}

int fdbcs_batch_too_old(fdbcs_batch* b, int32_t* idx_out, int32_t cap, int32_t* n_out) {
    if (!b || !n_out || cap < 0) return FDBCS_E_INVALID;
    if (b->routed) return FDBCS_E_STATE;  // decided at detect (k_route_too_old)
    int32_t n = 0;
    for (int32_t t = 0; t < (int32_t)b->flags.size(); t++) {
        if (!(b->flags[t] & kFlagTooOld)) continue;
        if (idx_out && n < cap) idx_out[n] = t;
        n++;
    }
    *n_out = n;
    return FDBCS_OK;
}

int fdbcs_batch_device_verdicts(fdbcs_batch* b, void** dptr) {
    if (!b || !dptr) return FDBCS_E_INVALID;
    if (b->state < 2) return FDBCS_E_STATE;
    *dptr = b->slot->dverdict.p;
    return FDBCS_OK;
}

int fdbcs_batch_set_conflict_output(fdbcs_batch* b, const int32_t* txn_ids, int32_t n_global, uint8_t* dev_out) {
    if (!b || n_global < 0 || (n_global > 0 && !dev_out)) return FDBCS_E_INVALID;
    if (!b->cs || b->state >= 2) return FDBCS_E_STATE;
    const int32_t T = b->T();
    if (T > 0 && !txn_ids) return FDBCS_E_INVALID;
    std::vector<uint8_t> seen((size_t)n_global, 0);
    for (int32_t t = 0; t < T; t++) {
        if (txn_ids[t] < 0 || txn_ids[t] >= n_global) return FDBCS_E_INVALID;
        if (seen[txn_ids[t]]++) return FDBCS_E_INVALID;  // one batch transaction per global index
    }
    b->out_ids.assign(txn_ids, txn_ids + T);
    b->out_n = n_global;
    b->out_dev = dev_out;
    return FDBCS_OK;
}

int fdbcs_debug_kernel_time(fdbcs_batch* b, int which, int reps, double* us_per_launch) {
    if (!b || !us_per_launch || reps <= 0 || which < 0 || which > 4) return FDBCS_E_INVALID;
    if (!b->cs) return FDBCS_E_STATE;
    fdbcs_conflict_set* cs = b->cs;
    HIPOK(hipSetDevice(cs->device));
    if (b->state == 0)
        if (int rc = fdbcs_batch_upload(b)) return rc;
    if (b->state != 1) return FDBCS_E_STATE;
    if (cs->inflight) return FDBCS_E_STATE;
    const int64_t T = b->T(), R = b->R(), W = b->W();
    if (int rc = ensure_workspace(cs, T, R, W)) return rc;
    if (int rc = sync_all(cs)) return rc;
    Work& w = cs->work[cs->wpar];
    Scalars* sc = (Scalars*)cs->scal.p;
    const Tier base{hist_of(cs, cs->cur), levels_of(cs, cs->cur), &sc->n, cs->header_version};
    const Tier delta{delta_of(cs, cs->dcur), dlevels_of(cs, cs->dcur), &sc->ndb[cs->dcur], kHole};
    if (which == 1 || which == 2) {  // the sort kernels
        if (!cs->quant_valid) return FDBCS_E_STATE;  // warm splitters only: detect a batch first
        HIPOK(debug_time_sort(cs->stream, b->bd, w, (SplitKey*)cs->quant.p + cs->qcur * kQuant, cs->bucket_target,
                              b->max_len > (int32_t)kSortNxLen, which, reps, us_per_launch));
        return FDBCS_OK;
    }
    hipEvent_t e0, e1;
    HIPOK(hipEventCreate(&e0));
    HIPOK(hipEventCreate(&e1));
    const bool dlong = b->max_len > 24;
    // 0: the whole check; 3 / 4: the split check's base / delta tier launch alone
    auto one = [&]() {
        uint8_t* ht = (uint8_t*)cs->htail[cs->tcur].p;
        if (which == 0)
            launch_check(cs->stream, b->bd, w, base, delta, ht, dlong);
        else
            launch_check_tier(cs->stream, b->bd, w, which == 3 ? base : delta, which == 3, ht, dlong, PrevSegs{});
    };
    one();
    HIPOK(hipEventRecord(e0, cs->stream));
    for (int i = 0; i < reps; i++) one();
    HIPOK(hipEventRecord(e1, cs->stream));
    HIPOK(hipEventSynchronize(e1));
    *us_per_launch = ev_ms(e0, e1) * 1000.0 / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // the check leaves per-transaction conflict flags the next batch on this workspace expects zeroed
    HIPOK(hipMemsetAsync(w.hist_conf, 0, w.cap_T, cs->stream));
    HIPOK(hipMemsetAsync(w.rconf, 0, w.cap_R, cs->stream));
    HIPOK(hipStreamSynchronize(cs->stream));
    return FDBCS_OK;
}

}  // extern "C"
