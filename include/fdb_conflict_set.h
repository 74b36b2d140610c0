/*
 * fdb_conflict_set.h — C-ABI of the MI355X-native MVCC conflict-resolution engine.
 *
 * Drop-in boundary for the FoundationDB resolver hot path.  Each entry point
 * replaces one member of the reference interface `fdbserver/ConflictSet.h`
 * (implemented by `fdbserver/SkipList.cpp`); the citation on every
 * declaration names the reference line it stands in for.  Plain C types only:
 * pointers, sizes, int64 versions.  No entry point throws; every fallible call
 * returns an `int` status (FDBCS_OK == 0, negative on error).
 *
 * Semantics are those of the reference:
 *   - keys are unsigned byte strings, compared memcmp-then-length
 *     (SkipList.cpp:53-60, flow/Arena.h:692-697);
 *   - a transaction is TooOld iff read_snapshot < oldestVersion and it has at
 *     least one read range (SkipList.cpp:770);
 *   - history conflict: some read range [b,e) overlaps history written at a
 *     version > read_snapshot (SkipList.cpp:619-706);
 *   - intra-batch conflict: in batch order, a read range overlaps a write range
 *     of an earlier committed transaction of the same batch (SkipList.cpp:812-834);
 *   - committed write ranges are recorded at version `now` (SkipList.cpp:899-939);
 *   - verdict bytes use the reference enum: 0 = TransactionConflict,
 *     1 = TransactionTooOld, 2 = TransactionCommitted (ConflictSet.h:40-44).
 *
 * Threading: like the reference (single flow thread, Resolver.actor.cpp:179-194)
 * a conflict set handle is not thread-safe; one handle per GPU.
 * Precondition the reference relies on implicitly (Resolver orders batches by
 * version, Resolver.actor.cpp:139-150): `now` never decreases below a version
 * already written; violating it returns FDBCS_E_VERSION.
 */
#ifndef FDB_CONFLICT_SET_H
#define FDB_CONFLICT_SET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes. */
#define FDBCS_OK 0
#define FDBCS_E_INVALID (-1)   /* bad argument: NULL handle, inverted range (KeyRangeRef throws inverted_range, FDBTypes.h:288-291), ... */
#define FDBCS_E_DEVICE (-2)    /* HIP runtime error */
#define FDBCS_E_NOMEM (-3)     /* host or device allocation failed / capacity exceeded */
#define FDBCS_E_VERSION (-4)   /* `now` below a version already present in the history */
#define FDBCS_E_STATE (-5)     /* call out of order (e.g. add after detect) */
#define FDBCS_E_NODEVICE (-6)  /* no HIP device / extension unusable: the product never falls back to the CPU */
#define FDBCS_E_TIMEOUT (-7)   /* a routed batch's shares never became ready (fdbcs_batch_add_routed) */

/* Verdict bytes: ConflictBatch::TransactionCommitResult (ConflictSet.h:40-44). */
#define FDBCS_TRANSACTION_CONFLICT 0
#define FDBCS_TRANSACTION_TOO_OLD 1
#define FDBCS_TRANSACTION_COMMITTED 2

typedef struct fdbcs_conflict_set fdbcs_conflict_set; /* ConflictSet (SkipList.cpp:730-737) */
typedef struct fdbcs_batch fdbcs_batch;               /* ConflictBatch (ConflictSet.h:35-69) */

/*
 * Packed, structure-of-arrays form of a commit batch: the CommitTransactionRef
 * fields the conflict set reads (CommitTransaction.h:184-188), flattened.
 * R = read_offsets[n_txn], W = write_offsets[n_txn].
 * Key k occupies key_bytes[key_offsets[k] .. key_offsets[k+1]).
 * Read range r (0 <= r < R): begin key 2r, end key 2r+1.
 * Write range w (0 <= w < W): begin key 2(R+w), end key 2(R+w)+1.
 * Ranges of transaction t: reads [read_offsets[t], read_offsets[t+1]),
 * writes [write_offsets[t], write_offsets[t+1]), in the transaction's order
 * (that order defines indexInTx for conflicting-key reports, SkipList.cpp:781).
 */
typedef struct fdbcs_packed_batch {
    int32_t n_txn;
    const int64_t* read_snapshot;           /* [n_txn] CommitTransactionRef::read_snapshot */
    const uint8_t* report_conflicting_keys; /* [n_txn] or NULL (= all false) */
    const int32_t* read_offsets;            /* [n_txn+1] */
    const int32_t* write_offsets;           /* [n_txn+1] */
    const uint8_t* key_bytes;               /* key arena */
    const int64_t* key_offsets;             /* [2*(R+W)+1] */
} fdbcs_packed_batch;

/* Per-phase device time (HIP events on the engine's stream, see fdbcs_set_timing), accumulated
 * since the last reset.  Phase names mirror the reference PerfDoubleCounters
 * D.CheckRead / D.Sort / D.CheckIntraBatch / D.Combine / D.MergeWrite /
 * D.RemoveBefore (SkipList.cpp:49-51). */
typedef struct fdbcs_stats {
    int64_t batches;
    int64_t transactions;
    int64_t read_ranges;
    int64_t write_ranges;
    double ms_upload;       /* H2D of packed batches */
    double ms_check_read;   /* history check (search + range max over both tiers; overlaps the sort) */
    double ms_sort;         /* endpoint sort */
    double ms_intra;        /* intra-batch candidate edges + batch-order resolution */
    double ms_combine;      /* union of committed writes */
    double ms_merge;        /* merge into the delta tier */
    double ms_gc;           /* removeBefore equivalent (runs with compactions) */
    double ms_total;        /* whole detect pipeline, device time */
    int64_t merge_bytes;    /* algorithmic bytes moved by the delta-merge copy kernel */
    int64_t merge_launches;
    double ms_merge_kernel; /* device time of the delta-merge copy kernel alone */
    int64_t compactions;    /* delta tier folded into the base tier */
    double ms_compact;      /* compaction phase (search + scan + copy) */
    int64_t compact_bytes;  /* algorithmic bytes moved by the compaction copy kernel */
    double ms_compact_kernel; /* device time of the compaction copy kernel alone */
    double ms_epilogue;     /* range-max rebuild + verdicts */
    int64_t intra_edges;    /* candidate intra-batch edges (sum over batches) */
    int64_t intra_rounds;   /* batch-order resolution rounds (sum over batches) */
    int64_t intra_fallbacks;/* batches resolved by the sequential MiniConflictSet replay */
    /* Roofline inputs of the other hot kernels (timing level >= 1), see roofline.py. */
    double ms_check_kernel; /* device time of the read-check kernel (D.CheckRead) */
    int64_t check_launches;
    int64_t check_reads;    /* read ranges checked (sum over launches) */
    int64_t check_history;  /* boundaries searched: base + delta tier size at check time (sum) */
    double ms_sort_kernel;  /* device time of the per-bucket sort kernel (D.Sort) */
    int64_t sort_launches;
    int64_t sort_items;     /* endpoints sorted (sum over launches) */
    int64_t gc_runs;        /* removeBefore passes (full, over the base tier after a compaction) */
    /* Host time inside fdbcs_batch_detect_async (milliseconds, summed): capacity checks and result
     * buffers, the host part of the upload, recording both stages, submitting them. */
    double host_ms_prepare;
    double host_ms_record;
    double host_ms_submit;
    int64_t compact_launches; /* compactions whose copy kernel was timed (compact_bytes counts these only) */
    /* Shapes of every batch, whatever the timing level (the roofline's byte models, roofline.py). */
    int64_t merge_bytes_all;   /* algorithmic bytes of every delta-merge copy */
    int64_t compact_bytes_all; /* algorithmic bytes of every compaction copy */
    int64_t delta_sum;         /* delta-tier boundaries at the start of each batch's merge, summed */
    int64_t base_sum;          /* base-tier boundaries after each batch, summed */
    int64_t segments_sum;      /* union segments of committed writes, summed */
    int64_t sort_big_buckets;  /* sort buckets past the per-wave capacity (ranked by their workgroup) */
    /* Device routing (fdbcs_batch_add_routed): batches, device time of their routing kernels
     * (events around them, every routed batch) and host time inside the call. */
    int64_t routed_batches;
    double ms_route_kernels;
    double host_ms_route;
    /* addTransaction of whole batches (fdbcs_batch_add_packed): host time inside the
     * calls (validation, normalization into pinned staging) and the calls' transactions. */
    double host_ms_add;
    int64_t added_txns;
    /* Launches of batch-order resolution left out of a batch's X half because the host had seen
     * its stage A find no candidate intra-batch edge (k_resolve, k_combine, k_intra_report). */
    int64_t x_launches_skipped;
} fdbcs_stats;

/* newConflictSet() — SkipList.cpp:739-741.  `device` = HIP ordinal. */
int fdbcs_new_conflict_set(int device, fdbcs_conflict_set** out);
/* clearConflictSet(cs, v) — SkipList.cpp:742-744: history reset to all-v, oldestVersion kept. */
int fdbcs_clear_conflict_set(fdbcs_conflict_set* cs, int64_t version);
/* destroyConflictSet(cs) — SkipList.cpp:745-747. */
void fdbcs_destroy_conflict_set(fdbcs_conflict_set* cs);

/* Raise-only oldestVersion (the effect of SkipList.cpp:880-882 without GC);
 * affects the next batch's TooOld test (SkipList.cpp:770). */
int fdbcs_set_oldest_version(fdbcs_conflict_set* cs, int64_t version);
int fdbcs_get_oldest_version(const fdbcs_conflict_set* cs, int64_t* out);
/* Boundaries held on the device, both tiers (SkipList::count, SkipList.cpp:386-394; equal to the
 * reference's count right after a compaction with GC, an upper bound otherwise). */
int fdbcs_history_size(fdbcs_conflict_set* cs, int64_t* out);
/* Bulk-load a history: boundaries sorted strictly ascending, boundary i holds
 * version versions[i] for keys in [key_i, key_{i+1}); keys below the first
 * boundary read `header_version`.  Used by benchmarks to prefill an MVCC window. */
int fdbcs_load_history(fdbcs_conflict_set* cs, int64_t n, const uint8_t* key_bytes,
                       const int64_t* key_offsets, const int64_t* versions, int64_t header_version);
int fdbcs_get_stats(fdbcs_conflict_set* cs, fdbcs_stats* out);
int fdbcs_reset_stats(fdbcs_conflict_set* cs);
/* Pre-size device capacity (history boundaries, history tail bytes, and the largest batch
 * shape) so later batches never reallocate; sizes are upper bounds, 0 keeps the current. */
int fdbcs_reserve(fdbcs_conflict_set* cs, int64_t boundaries, int64_t tail_bytes, int32_t max_txns,
                  int32_t max_reads, int32_t max_writes);
/* The history is two-tiered: every batch merges into a small delta tier; a
 * compaction folds the delta into the base tier, and removeBefore (GC) runs
 * with it when the oldest version moved.  Compaction happens when the delta may
 * exceed its limit (set_delta_limit; 0 = automatic, ~1/16 of the base) and, if
 * `every` > 0, at least every `every` batches (default 0).  Both knobs are
 * verdict-neutral: they only trade memory for speed. */
int fdbcs_set_gc_interval(fdbcs_conflict_set* cs, int32_t every);
int fdbcs_set_delta_limit(fdbcs_conflict_set* cs, int64_t boundaries);
/* Device timing of the pipeline (HIP events; each recorded event costs a few microseconds of
 * queue time, so production runs keep them off): 0 = none (default), 1 = the hot kernels only
 * (read check, bucket sort, the two history copy kernels: ms_*_kernel), 2 = every phase of
 * fdbcs_stats. */
int fdbcs_set_timing(fdbcs_conflict_set* cs, int32_t level);

/* ConflictBatch(cs, conflictingKeyRangeMap, arena) — SkipList.cpp:749-752.
 * report_keys != 0 enables conflictingKeyRangeMap collection for transactions
 * that set report_conflicting_keys. */
int fdbcs_batch_new(fdbcs_conflict_set* cs, int report_keys, fdbcs_batch** out);
void fdbcs_batch_destroy(fdbcs_batch* b);
/* ConflictBatch::addTransaction(tr) — SkipList.cpp:763-794.  Keys are copied. */
int fdbcs_batch_add_transaction(fdbcs_batch* b, int64_t read_snapshot, int report_conflicting_keys,
                                int32_t n_reads, const uint8_t* const* read_begin,
                                const int32_t* read_begin_len, const uint8_t* const* read_end,
                                const int32_t* read_end_len, int32_t n_writes,
                                const uint8_t* const* write_begin, const int32_t* write_begin_len,
                                const uint8_t* const* write_end, const int32_t* write_end_len);
/* addTransaction for every transaction of a packed batch, in order. */
int fdbcs_batch_add_packed(fdbcs_batch* b, const fdbcs_packed_batch* pb);
/* Stage the batch in HBM now (async H2D on the engine stream).  Optional:
 * detect uploads implicitly.  Lets callers keep PCIe out of a timed region. */
int fdbcs_batch_upload(fdbcs_batch* b);
/* Block until every stream of the conflict set is idle: uploads issued by fdbcs_batch_upload,
 * and every stage of every batch already submitted.  The engine's HIP runtime is not torch's
 * (INTEGRATION.md), so a caller timing HBM-resident batches calls this before starting its
 * clock.  No reference counterpart (the reference is synchronous, Resolver.actor.cpp:179-194). */
int fdbcs_sync(fdbcs_conflict_set* cs);
/* ConflictBatch::detectConflicts(now, newOldestVersion, nonConflicting, tooOld)
 * — SkipList.cpp:844-890.  verdicts[t] receives 0/1/2 per transaction
 * (Resolver.actor.cpp:196-204 encoding); counts are optional (NULL). */
int fdbcs_batch_detect_conflicts(fdbcs_batch* b, int64_t now, int64_t new_oldest_version,
                                 uint8_t* verdicts, int32_t* n_committed, int32_t* n_too_old);
/* Asynchronous form: enqueue the pipeline, return immediately; the verdicts of
 * the batch are fetched with fdbcs_batch_wait.  Batches must be waited in
 * submission order before the set is used for anything else. */
int fdbcs_batch_detect_async(fdbcs_batch* b, int64_t now, int64_t new_oldest_version);
int fdbcs_batch_wait(fdbcs_batch* b, uint8_t* verdicts, int32_t* n_committed, int32_t* n_too_old);
/* conflictingKeyRangeMap[txn] (SkipList.cpp:641-645, 822-825): read-range
 * indices (indexInTx) that conflicted, ascending.  Valid after detect. */
int fdbcs_batch_conflicting_reads(fdbcs_batch* b, int32_t txn, int32_t* idx_out, int32_t cap,
                                  int32_t* n_out);
/* ConflictBatch::GetTooOldTransactions (SkipList.cpp:836-842): indices of the transactions added
 * so far whose add-time TooOld test held (read_snapshot < oldestVersion with at least one read,
 * SkipList.cpp:770), ascending; valid right after the adds, before detect, as in the reference.
 * Writes at most cap indices (idx_out may be NULL to count).  A routed batch
 * (fdbcs_batch_add_routed) is judged at detect on the device: FDBCS_E_STATE (read its verdict
 * bytes instead). */
int fdbcs_batch_too_old(fdbcs_batch* b, int32_t* idx_out, int32_t cap, int32_t* n_out);
/* Device pointer to the batch's per-transaction verdict bytes (valid after
 * detect until the batch is destroyed) for on-device combine (RCCL). */
int fdbcs_batch_device_verdicts(fdbcs_batch* b, void** dptr);

/* On-device combine for key-range sharded resolvers (one per GPU).  Call after the batch's
 * transactions are added and before detect: txn_ids[t] in [0, n_global) is the global index (in
 * the proxy's batch) of the batch's transaction t.  Detect then also writes dev_out[0, n_global)
 * (device memory of this GPU, any allocator) with the conflict byte 2 - verdict of each routed
 * transaction and 0 elsewhere, complete when the batch is (fdbcs_batch_wait returns).  An
 * element-wise MAX all-reduce of dev_out over the resolvers holds 2 - min(verdict), the proxy's
 * combine (CommitProxyServer.actor.cpp:764-780). */
int fdbcs_batch_set_conflict_output(fdbcs_batch* b, const int32_t* txn_ids, int32_t n_global, uint8_t* dev_out);

/* Multi-resolver routing on the device: the commit proxy's split of a batch across resolvers
 * (CommitProxyServer.actor.cpp:118-187 with a static keyResolvers map; fdbrpc/RangeMap.h:126-129).
 * Each GPU is the proxy of one share of the global batch and the resolver of one key range.
 *   fdbcs_share_bytes / fdbcs_share_pack: the share in the engine's wire layout (host memory; no
 *     TooOld test, which stays with the resolvers).  The shares of all ranks are then gathered
 *     into one device buffer, `stride` bytes apart in rank order (an RCCL all-gather).
 *   fdbcs_batch_add_routed: on a new batch (the addTransaction step, SkipList.cpp:763-794): once
 *     the device word *ready_flag equals ready_value (the caller's stream sets it after the
 *     all-gather; NULL: the shares are already complete), the engine keeps, on the
 *     device, every range of the gathered shares that meets [lo_key, hi_key) (lo_len < 0: no lower
 *     bound, hi_len < 0: none above), unclipped, reads and writes alike; a transaction gets a
 *     sub-transaction iff one of its ranges is kept (:107-116), its snapshot copied.  Its TooOld
 *     test (SkipList.cpp:770) is made when the batch is detected, against the oldest version every
 *     earlier detect of this set left: the value addTransaction sees in the Resolver's order
 *     (Resolver.actor.cpp:139-150, 179-194), whether the routing was issued before or after the
 *     previous batch's detect.  Sub-transactions keep the global order.  cap_*: bounds on the
 *     routed batch, TooOld sub-transactions' ranges included (FDBCS_E_NOMEM at detect if passed).
 *     conflict_out (optional, n_global bytes of device memory, n_global = the transactions of all
 *     shares, FDBCS_E_INVALID at detect otherwise): as fdbcs_batch_set_conflict_output, with the
 *     global index of a sub-transaction = its position in the concatenated shares.  Conflicting-key
 *     reports are not collected for routed batches.  Detect and wait as for any batch; detect
 *     blocks until the routing kernels have run (issue the next batch's routing first).  The wait
 *     for the ready flag is bounded by FDBCS_ROUTE_TIMEOUT_MS (default 60000): past it detect
 *     returns FDBCS_E_TIMEOUT and the batch is empty again, to be routed anew.  The capacity
 *     (FDBCS_E_NOMEM) and n_global (FDBCS_E_INVALID) errors leave it empty the same way.
 *   fdbcs_batch_routed_info: the routed batch's sizes and device views of its global -> batch
 *     transaction map (int32[n_shares * max_share_txns], -1 where not routed) and of each kept
 *     read's index in its transaction (txReadConflictRangeIndexMap, :144-165). */
int fdbcs_share_bytes(const fdbcs_packed_batch* pb, int64_t* bytes);
int fdbcs_share_pack(const fdbcs_packed_batch* pb, void* out, int64_t cap, int64_t* used);
int fdbcs_batch_add_routed(fdbcs_batch* b, const void* shares, int64_t stride, int32_t n_shares, int32_t max_share_txns,
                           const uint8_t* lo_key, int32_t lo_len, const uint8_t* hi_key, int32_t hi_len,
                           int32_t cap_txns, int32_t cap_reads, int32_t cap_writes, int64_t cap_tail,
                           uint8_t* conflict_out, int64_t n_global, const uint32_t* ready_flag,
                           uint32_t ready_value);
int fdbcs_batch_routed_info(fdbcs_batch* b, int32_t* n_txn, int32_t* n_reads, int32_t* n_writes, void** inv_dev,
                            void** read_ids_dev);

/* Diagnostics (tuning, not part of the ConflictSet contract): average device time of one launch
 * of a pipeline kernel over `reps` back-to-back launches on the uploaded batch `b` against the
 * current history, with no batch in flight.  which: 0 = the read check (D.CheckRead); 1-2 = the
 * endpoint sort's kernels (partition, per-bucket sort; splitters of the last batch detected); 3-4 =
 * the split check's base / delta tier launch alone. */
int fdbcs_debug_kernel_time(fdbcs_batch* b, int which, int reps, double* us_per_launch);
/* Per-kernel device time accumulated since fdbcs_reset_stats: timing level 3 brackets every kernel
 * of every batch with events, level 1 the kernel named by fdbcs_set_timed_kernel on the sampled
 * batches.  Entry `index` (0-based; FDBCS_E_INVALID past the last): demangled kernel name (without
 * namespace and parameters) into name[cap], its timed launches and their total milliseconds. */
int fdbcs_kernel_profile(fdbcs_conflict_set* cs, int32_t index, char* name, int32_t cap, int64_t* launches,
                         double* ms);
/* The kernel timed at level 1 (a name fdbcs_kernel_profile reported; NULL or "" = none). */
int fdbcs_set_timed_kernel(fdbcs_conflict_set* cs, const char* name);
/* Diagnostics: on != 0 queues a bounded hold kernel on every stream of the set, so batches
 * submitted next wait behind it; on == 0 releases them, and they run back to back at the device's
 * own rate (the device-bound throughput, free of the submitting thread). */
int fdbcs_debug_hold(fdbcs_conflict_set* cs, int32_t on);

const char* fdbcs_strerror(int status);

#ifdef __cplusplus
}
#endif
#endif /* FDB_CONFLICT_SET_H */
