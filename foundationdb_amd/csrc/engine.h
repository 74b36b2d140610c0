// engine.h — internal interface between the host engine (engine.cpp) and the
// gfx950 kernels (kernels.hip).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>

#include "dkey.h"
#include "scan.h"

namespace fdbcs {

constexpr int kBlock = 256;        // default workgroup: 4 waves of 64
constexpr int kWG = 1024;          // single-workgroup kernels (scans, resolution)
constexpr int kSortTile = 4096;    // endpoints per LDS sort tile (128 KiB of LDS)
constexpr int kFan = 64;           // range-max fan-out per level (one wave per block)
constexpr int kMaxLevels = 4;      // hv, max1 (/64), max2 (/4096), max3 (/262144)
// Level 3 (the top, a few entries per tier) is built by atomicMax from every wave of the epilogue:
// each entry is kept as kL3Rep replicas, one 128-byte line apart, written by different workgroups
// and max-ed by the readers (one line took ~1000 atomics per entry: 89 of the 106 us of a 5M-base
// rebuild, scripts/gpu_r05_k.sh).
constexpr int kL3Rep = 8;
constexpr int kL3Pad = 16;  // 8-byte words per replica line
__host__ __device__ constexpr int64_t l3_words(int64_t n) { return n * kL3Rep * kL3Pad; }
constexpr int kGcTile = 4096;      // history elements per GC / merge tile
constexpr int kMaxGroupWrites = 12288;  // write groups: 8 bytes of resolver LDS per write
constexpr int kMaxTxnLds = 49152;  // transactions whose status bytes fit the resolver's LDS (> the
                                   // reference's 32768-transaction batch cap, fdbserver/Knobs.cpp:370)

// Transaction status during batch-order resolution.
enum : uint8_t { kUndecided = 0, kAborted = 1, kCommitted = 2 };
// Per-transaction input flags.
enum : uint8_t { kFlagTooOld = 1, kFlagReport = 2 };

// One history buffer set (structure of arrays; boundary i covers [key_i, key_{i+1})).
struct Hist {
    ulonglong2* key;  // (hi, lo) prefix words
    uint2* lt;        // (len, tail offset)
    int64_t* ver;     // segment version
};

// Range-max hierarchy over the current history's versions.
// Range-max hierarchy over a tier's versions, and its static kArity-ary search tree over sampled
// key prefixes: skey[L][j] = prefix of boundary 64 * A^L * j, so skey[L][j] == skey[L-1][A j].  A
// lookup descends the tree with kArity cooperating lanes, one node (one 128-byte line at A = 8) per
// level, and lands in one 64-boundary block.
constexpr int kArity = 8;
constexpr int kDirMaxBits = 20;     // radix directory: at most 2^20 code values (+3 end slots) per tier
constexpr int kDirAlloc = (1 << kDirMaxBits) + 4;  // directory entries allocated (dir, edir)
constexpr int kDirPos = 8;          // byte positions after the common prefix a directory code reads
constexpr int kDirRun = 128;        // delta directory: slots one sample fills at most (the rest stay stale)
constexpr int kIdxLevels = 12;  // A^11 * 64 * A boundaries under an A-entry top level
struct MaxLevels {
    int64_t* lvl[kMaxLevels];       // lvl[0] == current Hist::ver
    const ulonglong2* keys;         // the tier's keys (source of the samples)
    ulonglong2* skey[kIdxLevels];   // [ceil(n / (64 * A^L))]
    ulonglong2* skey8;              // [ceil(n / 8)] prefix of every 8th boundary: the level below skey[0]
    int64_t idx_cap;                // capacity the levels were carved for: skey[L] = skey[0] + sum of
                                    // idx_level_cap(idx_cap, l < L), computable without indexing skey[]
    const int32_t* dir = nullptr;   // [dir_top + 2] radix directory over skey[0] (base tier; k_directory)
    // Directory slots (kernels.hip dir_slot), an order-preserving code of the 16-byte prefix fixed
    // when the history is loaded (engine.cpp set_dir_map) and used by both tiers: keys outside the
    // dir_p bytes every loaded key shares (dir_phi, dir_plo: those bytes, the rest zero) take slot
    // 0 (below) or dir_top (above); inside, the next dir_e byte positions are read as a mixed-radix
    // number whose digit at position i is the byte's offset in the range [lo, lo + d) of values
    // the loaded keys hold there (dir_pos[i] = lo | d << 8 | s << 17, weight dir_w[i]; a byte
    // below the range counts 0 and one above it d, and either ends the code; the last position
    // may be coarsened by >> s to fit the slot budget), so C4's decimal user digits after a 9-byte
    // common prefix spread over 10^6 slots instead of 100.  Arithmetic only: no table loads on the
    // lookup's chain.
    uint32_t dir_p = 0;
    uint64_t dir_phi = 0, dir_plo = 0;
    uint32_t dir_e = 0;
    uint32_t dir_top = 0;
    uint32_t dir_pos[kDirPos] = {};
    uint32_t dir_w[kDirPos] = {};
    uint64_t* edir = nullptr;       // [dir_top + 2] delta tier's directory, entries (epoch << 32 | count),
    uint32_t edir_epoch = 0;        // filled by k_epilogue; lookups trust entries of this epoch (0: off)
};
__host__ __device__ inline int64_t idx_level_cap(int64_t cap, int L) {
    int64_t d = 64;
    for (int i = 0; i < L && d <= cap; i++) d *= kArity;
    return cap / d + 2;
}

// Device-side scalars of a conflict set (one allocation).  The history has two tiers: the base
// (sorted boundaries, rewritten only by compaction) and the delta (this window's merges, versions
// or kHole where the base shows through).
struct Scalars {
    int64_t n;             // base boundaries
    int64_t nd;            // delta boundaries
    int64_t n_next;        // base after this batch's compaction
    int64_t nd_next;       // delta after this batch's merge
    int64_t n_gc;          // base after GC
    int64_t tail_used;     // bytes used in the history tail arena
    int64_t tail_next;     // after this batch's merge appended its new boundaries' tails
    int64_t tail_gc;       // after GC repacked the live tails into the other arena
    int64_t n_segments;    // union segments of committed writes
    int64_t d_before;      // delta size at the start of the merge
    int64_t d_rem;         // delta boundaries removed by union segments
    int64_t c_before;      // base size at the start of a compaction
    int64_t c_rem;         // base boundaries removed (overwritten) by the compaction
    int32_t debug_error;   // copied from the batch's BatchScalars by the epilogue (host view only)
    int32_t intra_rounds;  // copied from BatchScalars::rounds by the epilogue (host view only)
    int64_t intra_edges;   // copied from BatchScalars::n_edges (host view only; overflow -> -1)
    int32_t sort_big;      // copied from BatchScalars::sort_big (host view only)
    int32_t sort_pad;
    int64_t ndb[2];        // delta boundaries held by delta buffer k (read checks and merges address
                           // the buffer they use: the next batch's check reads the buffer before
                           // this batch's merge while the merge writes the other one)
};

// Device scalars of one batch workspace (two workspaces alternate, so batch i+1's history-
// independent stage can run while batch i finishes).
struct BatchScalars {
    int64_t n_edges;       // candidate edges
    int32_t edge_overflow; // candidate edges exceeded capacity -> sequential fallback
    int32_t rounds;        // resolution rounds used
    int32_t debug_error;   // FDBCS_VALIDATE: invariant violated; bit 1: scan look-back timed out
    int32_t ovf_n;         // sort: endpoints past their bucket's slab (reset by the epilogue)
    int32_t sort_big;      // sort: buckets past the slab, sorted by the workgroup path (reset by the epilogue)
    int64_t n_segments;    // union segments of committed writes (D.Combine, k_resolve)
    int64_t n_pranges;     // ranges with candidate pairs (k_scan<EdgePairScan>)
    int32_t n_undec;       // transactions the resolution pre-pass left undecided (Work::ulist; reset by the epilogue)
    int32_t pad2;
};

// Delta-tier version meaning "not written in this window: the base tier's version applies".
constexpr int64_t kHole = INT64_MIN;

// Where a merge reads its source size and reports its result.
struct TierIO {
    const int64_t* n_in;   // source boundaries
    int64_t* n_out;        // boundaries after the merge
    int64_t* before;       // copy of *n_in (stats)
    int64_t* removed;      // boundaries removed (stats)
};

// Segments applied to a sorted boundary array by k_merge_copy: segment s removes [lo_s, hi_s) and
// inserts ins_s boundaries at lo_s.  rem/ins hold counts, then exclusive prefixes (sentinel at U).
struct Segs {
    int64_t *lo, *hi, *rem, *ins;
    int32_t* tile_first;   // first segment whose lo lies in copy tile t or later
};

// Scans of one batch (each owns a slice of the per-batch zeroed scan arena).
enum ScanKind { kScanEdges, kScanSegSum, kScanCompact, kScanGc, kScanCover, kScanSegNum, kScanFold, kNumScans };

// Device copy of one batch's packed input (tooOld transactions carry no ranges,
// as in addTransaction, SkipList.cpp:770-790).
struct BatchDev {
    int32_t T, R, W;
    int64_t* snap;       // [T]
    uint8_t* flags;      // [T]
    int32_t* roff;       // [T+1]
    int32_t* woff;       // [T+1]
    int32_t* rowner;     // [R]
    int32_t* wowner;     // [W]
    DKey* keys;          // [2(R+W)]
    uint8_t* tail;       // key bytes beyond 16
    int64_t tail_n;      // bytes of `tail` in use
};

// D.Sort geometry (kernels.hip): a bucket holds kSortTarget endpoints on average and is sorted in
// registers by one wave up to kSlab endpoints; splitters are projections of the quantiles of the
// last sorted batch (kQuant of them), or of this batch's ranked samples at a cold start.
#ifndef FDBCS_SORT_TARGET
#define FDBCS_SORT_TARGET 64
#endif
constexpr int kSortTarget = FDBCS_SORT_TARGET;
constexpr int kSlab = 256;
constexpr int kSortMaxBuckets = 4096;
constexpr int kQuant = 4096;
constexpr int kQuantMinE = 2048;  // batches with fewer endpoints leave the quantiles as they are
constexpr int kMaxSample = 8192;
#ifndef FDBCS_CNT_STRIDE
#define FDBCS_CNT_STRIDE 16
#endif
constexpr int kCntStride = FDBCS_CNT_STRIDE;  // u64 words per sort bucket counter line
// A splitter: the projection of an endpoint onto its first kSplitBytes key bytes (big-endian
// words, zero past the key), min(len, kSplitBytes + 1), and for keys no longer than kSplitBytes
// the class and id (meta).  Projections are monotone in the full order (keys tied on their first
// kSplitBytes bytes share one), so a bucket boundary never separates endpoints the order needs the
// bytes beyond the window for.
constexpr int kSplitWords = 8;
constexpr int kSplitBytes = 8 * kSplitWords;
struct SplitKey {
    uint64_t w[kSplitWords];
    uint32_t len, meta;
};

// Per-set scratch, sized for the largest batch seen.
struct Work {
    uint8_t* hist_conf;    // [T]
    uint8_t* rconf;        // [R]
    uint8_t* status;       // [T]
    int32_t* first_conf;   // [T]
    // D.Sort (k_sort_partition / k_sort_bucket): endpoints partitioned into buckets between
    // splitters, each bucket sorted by one wave (or its workgroup past kSlab endpoints)
    SortItem* items;       // [E] sorted endpoints (FDBCS_VALIDATE only)
    uint64_t* scnt;        // [kCntStride kSortMaxBuckets] per bucket, one 128-byte line: endpoints |
                           // write-begins << 32, read-begins | write-ends << 32 (zeroed per batch)
    SortItem* slab;        // [slab_buckets * kSlab] each bucket's first kSlab endpoints
    int32_t slab_buckets;  // buckets the slab holds
    SortItem* ovf;         // [E] endpoints past their bucket's slab
    int32_t* ovf_b;        // [E] their buckets
    SortItem* big;         // [E] a big bucket's endpoints, gathered (workgroup path)
    int32_t* big_p;        // [E] a big bucket's endpoint ids in sorted order (workgroup path)
    SortItem* samples;     // [kMaxSample] cold start: sample items (k_sample)
    int32_t* srank;        // [kMaxSample + 64] cold start: sample ranks (zeroed per batch)
    int32_t* pos;          // [2(R+W)] sorted position of each endpoint
    uint32_t* pmeta;       // [E] meta of the item at each position
    int32_t* cwb;          // [E+1] write-begins before each position
    int32_t* crb;          // [E+1] read-begins before each position
    int32_t* cwe;          // [E+1] write-ends before each position
    int2* wends;           // [2W] write endpoints in sorted order: (position, 2 owner + is-end; -1 empty write)
    DKey* wkeys;           // [2W] their keys (tails in the batch's tail region)
    DKey* segk;            // [2W] union segment j: begin key 2j, end key 2j + 1 (D.Combine)
    uint8_t* cflag;        // [2W] D.Combine across workgroups: write endpoint opens (1) / closes (2) a segment
    uint8_t* btail;        // [btail_cap] copy of the batch's tail region (k_sort_partition): the next
                           // batch's read check reads segk's tails here, after the batch is waited
    int32_t* wbrange;      // [W] range of each write-begin, in sorted order
    int32_t* rbrange;      // [R] range of each read-begin, in sorted order
    int32_t* eoff;         // [R+1] first edge slot of each read
    int32_t* poff;         // [R+W+1] first candidate pair of each range
    int32_t* pcg;          // [R+W+1] the ranges with candidate pairs, in order (then G)
    int32_t* pcoff;        // [R+W+1] their first pairs (then the pair count): k_edge_fill's index
    int32_t* pcbase;       // [R+W] their partner lists' bases (cwb / crb at the range's begin)
    int32_t* pca;          // [R+W] their side of the edge test (EdgePairScan::store)
    int32_t* ecur;         // [R] edges of each read (slots taken; zeroed by the epilogue)
    // write groups (groups != 0): consecutive write-begins (in sorted order) whose writes contain
    // exactly the same read-begins are one group; a read gets one edge T + j per group j (j = the
    // group's first write-begin index) instead of one per writer (C3: a hot key's writers)
    int32_t* wlead;        // [W] per write-begin index: 2 first of a group, 1 member, 0 none
    int32_t* wtxn;         // [W] transaction of the write with that write-begin
    int32_t* gminc;        // [W] per group: least committed member transaction (k_resolve)
    int32_t groups = 0;    // set per batch
    int32_t* edges;        // [edge_cap] writer transaction of each candidate edge
    int64_t edge_cap;
    int32_t* eptr;         // [T] resume pointer per transaction
    uint8_t* pre_st;       // [T] k_resolve pre-pass: status before the batch-order rounds
    int32_t* pre_ep;       // [T] k_resolve pre-pass: start of t's packed live writers in tedges
    int32_t* pre_end;      // [T] k_resolve pre-pass: end of t's packed live writers
    int4* ulist;           // [2T] k_resolve pre-pass: per undecided transaction {t, first live writer slot,
                           // end slot, 0} and its first four live writers (-1 past the end)
    uint32_t* wpk;         // [W] per write-begin index: group lead (bits 30-31: 2 first, 1 member, 0 none)
                           // | its transaction + 1 unless the pre-pass knows it aborted (k_resolve_pre)
    int32_t report = 0;    // the batch reports conflicting keys (k_resolve keeps gminc)
    int32_t* tedges;       // [edge_cap] per transaction, its writers not known aborted (packed)
    uint64_t* mcs_bits;    // [E/64+1] sequential-fallback MiniConflictSet
    // union segments (<= W)
    int32_t* seg_b;        // position of segment begin
    int32_t* seg_e;        // position of segment end
    int64_t* seg_lo;
    int64_t* seg_hi;
    int64_t* seg_rem;      // -> exclusive prefix after scan
    int64_t* seg_ins;
    int64_t* seg_tlen;
    uint8_t* seg_endins;
    int64_t* seg_vend;
    uint8_t* verdict;      // [T]
    BatchScalars* bsc;
    ScanState scan[kNumScans];
    int64_t scan_gran[kNumScans];  // granules each scan's slice of the arena holds
    uint64_t* scan_arena;  // zeroed by the previous batch's epilogue (and at allocation)
    int64_t scan_words;
    int64_t cap_T, cap_R;  // workspace capacity (what the epilogue zeroes)
    int32_t* tile_first;   // [max(hist_cap, delta_cap) / kGcTile + 4] first segment of each copy tile
    // compaction: one entry per delta boundary (sized by the delta capacity)
    int64_t *c_lo, *c_hi, *c_rem, *c_ins, *c_val;
    uint8_t* c_exact;
    unsigned long long* trace;  // [kTrSlots] or null
    int32_t no_prepass;         // FDBCS_RESOLVE_PREPASS=0: resolution rounds without the pre-pass (tests)
    // host-mapped {batch seq, any candidate edge} of the batch on this workspace, written by the
    // edge scan's finish (kGroupEdges launches left out when 0; null: not tracked)
    uint32_t* hedge;
    uint32_t hseq;
    // [T] device copy of the batch's verdicts (its slot's dverdict), written by the resolution next
    // to the host-mapped verdict bytes (fdbcs_batch_device_verdicts); set per batch, null: none
    uint8_t* vdev;
};

// FDBCS_TRACE: device timestamps (wall_clock64 ticks) of kernel sections, for tuning.
enum TraceSlot {
    kTrSampleBegin, kTrSampleEnd, kTrCheckBegin, kTrCheckEnd,
    kTrEpiBegin, kTrEpiLevels, kTrEpiZero, kTrEpiHost, kTrEpiFence, kTrEpiEnd,
    kTrResBegin, kTrResPre, kTrResWait, kTrResRounds, kTrResEnd,
    kTrPartBegin, kTrPartFill, kTrPartSearch, kTrPartEnd,
    kTrBktBegin, kTrBktPrologue, kTrBktSorted, kTrBktTies, kTrBktEnd,
    kTrBktWaves, kTrBktSumLoad, kTrBktSumSort, kTrBktSumTies, kTrBktSumPut,  // per-wave sums (ticks)
    kTrPartWaves, kTrPartSumFill, kTrPartSumCopy, kTrPartSumSearch, kTrPartSumPlace,
    kTrCmbLoad, kTrCmbScan1, kTrCmbScan2, kTrCmbStore,
    kTrResSetup, kTrResRound1,  // k_resolve: statuses and members staged; first round done
    kTrResMin1,  // k_resolve: the first round's group minima done
    kTrResW0min, kTrResW0max,  // k_resolve: first instruction of its first / last wave (before kernargs)
    kTrBktRuns, kTrBktSimple, kTrBktSlow, kTrBktMaxRun,  // k_sort_bucket tie runs: lanes in a run, ranked
                                                         // in registers, by the serial path; longest run
    kTrSlots
};
__device__ __forceinline__ void trace_min(unsigned long long* tr, int slot) {
    if (tr) atomicMin(&tr[slot], (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void trace_max(unsigned long long* tr, int slot) {
    if (tr) atomicMax(&tr[slot], (unsigned long long)wall_clock64());
}

// Byte offset of the Scalars copy that follows the verdicts in a batch's result buffer.
__host__ __device__ inline int64_t verdict_scalars_offset(int64_t T) { return (T + 64) / 64 * 64; }

// ---- multi-resolver routing on the device (the commit proxy's step, CommitProxyServer.actor.cpp:
// 118-187, for a static key-range split).  Every rank is the proxy of one share of the global
// batch: it packs its share in the wire layout below (fdbcs_share_pack), the shares are
// all-gathered over xGMI (RCCL), and each resolver keeps the ranges that meet its key range
// (k_route_mark, k_scan<RouteScan>, k_route_write) as a batch in the upload layout.
// Wire layout of a share: ShareHeader, then DKey keys[2(R+W)] (tail = byte offset in the share's
// tail region), int64 snap[T], int32 roff[T+1], int32 woff[T+1], uint8 report[T], int32 owner[R+W],
// tail bytes; every region 64-byte aligned, the whole share <= the all-gather stride.
struct ShareHeader {
    int32_t T, R, W, pad0;
    int64_t bytes;       // the share, header included
    int64_t off_keys, off_snap, off_roff, off_woff, off_report, off_tail;
    int64_t tail_bytes;
    int64_t off_owner;   // int32 owner[R+W]: the transaction of each read, then of each write
    int64_t pad[5];
};
static_assert(sizeof(ShareHeader) == 128, "ShareHeader is 128 bytes");
// Totals of a routed batch (host-mapped copy for the host, device copy for k_route_write).
struct RouteResult {
    int32_t T, R, W, reports;
    int32_t n_gt19, n_gt24;  // kept keys longer than 19 / 24 bytes (sort tail windows, long-key probes)
    int64_t tail_bytes;
    int32_t error;           // 1: a capacity bound was exceeded (nothing past it was written); 2: the
                             // shares' ready flag was never set; 3: conflict output size != global T
    int32_t pad;
    int64_t global_T;        // transactions of all shares
};
struct RouteArgs {
    const uint8_t* shares;  // n_shares shares, `stride` bytes apart
    int64_t stride;
    int32_t n_shares, tcap;  // tcap: bound on any share's T (global element i = share i / tcap)
    int32_t has_lo, has_hi;  // this resolver owns [lo, hi): lo absent for the first, hi for the last
    DKey lo, hi;
    const uint8_t* btail;    // tails of lo / hi
    int32_t report_enabled;
    int32_t cap_T, cap_R, cap_W;  // capacity of the output layout
    int64_t cap_tail;
    // outputs: the routed batch at capacity offsets of the upload layout
    DKey* keys;      // the routed endpoints: reads' [2R'], then writes'
    uint32_t* info;  // [n_shares * rstride] per range: kept, long-key bits, tail bytes (k_route_mark)
    int64_t rstride; // >= any share's R + W
    int4* txpre;     // [n_shares * tcap] per transaction: batch index, read / write / tail prefixes
    int32_t *rown, *wown, *roff, *woff;
    int64_t* snap;
    uint8_t* flags;
    uint8_t* tail;
    int32_t* inv;       // [inv_n] batch index of each global transaction, -1 if not routed here
    int64_t inv_n;      // n_shares * tcap (every global index fits)
    int32_t* read_ids;  // [R'] index of each kept read in its transaction (txReadConflictRangeIndexMap)
    uint8_t* out_zero;  // conflict output to zero for this batch (or null), out_n global transactions
    int64_t out_n;
    RouteResult* res;   // host-mapped
    RouteResult* dres;  // device copy
    const uint32_t* ready;  // device word the caller's stream sets to ready_value once the shares are
    uint32_t ready_value;   // gathered (null: already complete); k_route_wait spins on it
    uint32_t* wait_err;     // set when that wait timed out (the routed batch then reports an error)
    uint64_t wait_ticks;    // bound of that wait, in 100 MHz wall-clock ticks
};
// Route the all-gathered shares into this resolver's batch (two launches on `s`).  grid_n: bound
// on n_shares * tcap (global elements); the scan state's granules are zeroed by the caller.
void launch_route(hipStream_t s, const RouteArgs& a, ScanState st);
int64_t route_scan_words(int64_t n_elems);
// TooOld (SkipList.cpp:770) of a routed batch against the oldest version at detect time.
void launch_route_too_old(hipStream_t s, const BatchDev& b, int64_t oldest);

// ---- launchers (kernels.hip); all enqueue on `s` and never synchronize.
// A history tier as the read check sees it.
struct Tier {
    Hist h;
    MaxLevels m;
    const int64_t* n;  // device size
    int64_t hdr;       // version below the first boundary (kHole for the delta)
};
// The previous batch's union segments (its committed writes' union, at version `version`), for
// a read check that runs before that batch's merge into the delta tier (stage B's merge half runs
// on its own stream, beside the next batch's check).  n == nullptr: none.
struct PrevSegs {
    const DKey* segk;     // begin / end keys of segment j at 2j / 2j + 1
    const uint8_t* tail;  // their tails (the previous batch's workspace copy)
    const int64_t* n;     // segments
    int64_t version;      // the previous batch's `now`
};
// Per batch, two stages on two streams:
//   A (history-independent): launch_sort (D.Sort + positions), launch_edges;
//   B (reads/writes the history, in batch order): launch_check, launch_resolve (+ D.Combine),
//     launch_merge, launch_compact/gc, launch_epilogue.
// D.Sort and the sorted positions (replaces the sample sort + position scan): splitters from the
// quantile table `quant` (cold: written first from this batch's ranked samples, k_sample +
// k_quant_cold), then k_sort_partition and k_sort_bucket.  quant_out: the other table, which
// receives this batch's quantiles for the next batch (null: keep).  long_keys: the batch has keys
// longer than kSortNxLen (tail comparisons possible).
void launch_sort(hipStream_t s, const BatchDev& b, const Work& w, SplitKey* quant, SplitKey* quant_out, bool cold,
                 int bucket_target, bool long_keys, bool validate, hipEvent_t sort_begin, hipEvent_t sort_end);
// Buckets of a batch of E endpoints (target 0 = kSortTarget), within the workspace slab.
int sort_bucket_count(int64_t E, int target, int slab_buckets);
// D.CheckRead against the history the previous batch left: one lane per lookup, four lanes per
// read (begin and end in both tiers).  long_keys: the batch has keys over 24 bytes (the long-key
// lookup, lane_lower_bound_long).
void launch_check(hipStream_t s, const BatchDev& b, const Work& w, const Tier& base, const Tier& delta,
                  const uint8_t* htail, bool long_keys = false, const PrevSegs& ps = PrevSegs{});
// D.CheckRead over one tier (the split check: base tier in stage A when no compaction is pending,
// delta tier in stage B), two lanes per read; both OR into the workspace's pre-zeroed conflict flags.
void launch_check_tier(hipStream_t s, const BatchDev& b, const Work& w, const Tier& t, bool is_base,
                       const uint8_t* htail, bool long_keys = false, const PrevSegs& ps = PrevSegs{});
// Diagnostics (fdbcs_debug_kernel_time): isolated device time of the sort's launches (which 1 =
// k_sort_partition, 2 = k_sort_bucket) over `reps` runs on an idle stream.
hipError_t debug_time_sort(hipStream_t s, const BatchDev& b, const Work& w, SplitKey* quant, int bucket_target,
                           bool long_keys, int which, int reps, double* us);
// FDBCS_VALIDATE: the sorted endpoints are in order and the positions invert the permutation.
void launch_validate_sort(hipStream_t s, const BatchDev& b, const Work& w);
void launch_edges(hipStream_t s, const BatchDev& b, const Work& w);
// verdict_out: the batch's host-mapped verdict bytes (the epilogue publishes them with the flag).
void launch_resolve(hipStream_t s, const BatchDev& b, const Work& w, bool report, uint8_t* verdict_out, Scalars* sc);
// Union segments of the batch into the delta tier (src -> dst), new boundaries at `now`.
// `srcm` are the source tier's levels: its key index is searched, its top level reset for the
// epilogue's rebuild.
// nd_src: the source buffer's size; dstm: the destination's levels (top level reset for the epilogue).
void launch_merge(hipStream_t s, const BatchDev& b, const Work& w, const Hist& src, const MaxLevels& srcm,
                  const Hist& dst, const MaxLevels& dstm, const int64_t* nd_src, uint8_t* htail, Scalars* sc,
                  int64_t now, int64_t lvl3_n, int64_t lvl2_n, int64_t grid_hint_n, hipEvent_t copy_begin,
                  hipEvent_t copy_end, bool long_keys = false);
// Overlay the delta tier onto the base tier (src -> dst); the delta becomes empty.
void launch_compact(hipStream_t s, const Work& w, const Hist& base, const MaxLevels& basem, const Hist& delta,
                    const Hist& dst, const uint8_t* htail, Scalars* sc, int64_t header_version, int64_t lvl3_n,
                    int64_t lvl2_n, int64_t delta_hint_n, int64_t grid_hint_n, hipEvent_t copy_begin,
                    hipEvent_t copy_end, int mode, int base_tile, bool nt);
// removeBefore over the whole base (src -> dst); the live tails are repacked from arena tsrc into
// the empty arena tdst (reclaiming the bytes of removed and overwritten boundaries).
void launch_gc(hipStream_t s, const Work& w, const Hist& src, const Hist& dst, const uint8_t* tsrc, uint8_t* tdst,
               Scalars* sc, int64_t oldest, int64_t header_version, int64_t grid_hint_n);
// Hold `s` until *release != 0 (host-mapped word; bounded spin).
void launch_hold(hipStream_t s, const uint32_t* release);
// Kernel attributes set once per process (the resolver's dynamic LDS above 64 KiB).
void init_kernel_attributes();
// Byte copy (device -> host-mapped result buffer), as a kernel.
void launch_copy_bytes(hipStream_t s, void* dst, const void* src, int64_t n);
// Multi-resolver conflict bytes out[g] = 2 - verdict of batch transaction inv[g] (0 if inv[g] < 0).
void launch_conflict_output(hipStream_t s, const BatchDev& b, const Work& w, const int32_t* inv, int64_t n,
                            uint8_t* out);
int64_t scan_arena_words(int64_t T, int64_t R, int64_t W, int64_t hist_cap, int64_t delta_cap);
void carve_scans(Work& w, int64_t T, int64_t R, int64_t W, int64_t hist_cap, int64_t delta_cap);
// Range-max levels of a tier whose size is *n (lvl[2] and lvl[3] reset first).
void launch_rangemax(hipStream_t s, const MaxLevels& m, Scalars* sc, const int64_t* n, int64_t lvl3_n,
                     int64_t lvl2_n, int64_t grid_hint_n);
// Scalar roll-over, the device copy of the verdicts, scratch zeroing and the range-max levels of
// the tier that changed (the base after a compaction, else the delta).  k_resolve already wrote the
// verdict bytes into the host-mapped result; the epilogue publishes the scalars after them and
// then the completion flag (the host waits for *flag == seq instead of an event).
// nd_out: the size word of the delta buffer the batch leaves current (Scalars::ndb).
// sort_nb / sort_samples: the batch's sort buckets and cold-start samples (their counters and
// ranks are re-zeroed; 0 samples on a warm start).
void launch_epilogue(hipStream_t s, const BatchDev& b, const Work& w, const MaxLevels& m, Scalars* sc,
                     int compacted, int gc_ran, uint8_t* verdict_out, uint32_t* flag,
                     uint32_t seq, int64_t grid_hint_n, int64_t* nd_out, int sort_nb, int sort_samples);
// Cold-start samples of a sort over E endpoints in nb buckets (k_sample; ranks re-zeroed by the epilogue).
int sort_cold_samples(int64_t E, int nb);

}  // namespace fdbcs
