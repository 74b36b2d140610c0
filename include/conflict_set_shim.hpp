// conflict_set_shim.hpp — header-only C++ adapter restoring the reference signatures of
// fdbserver/ConflictSet.h (newConflictSet / clearConflictSet / destroyConflictSet /
// ConflictBatch::{addTransaction, detectConflicts, GetTooOldTransactions}) on top of the C-ABI
// in fdb_conflict_set.h.  A FoundationDB build drops SkipList.cpp, includes this header from one
// translation unit (e.g. a new fdbserver/ConflictSetGpu.cpp) and links libfdbcs.so; Resolver.actor.cpp
// (:179-194) and the skip-list test driver keep calling the same names.
//
// The transaction type is a template parameter so the header needs nothing from flow/ or
// fdbclient/: any type with `read_conflict_ranges`, `write_conflict_ranges` (elements with
// `.begin` / `.end` exposing `.begin()` and `.size()`, as KeyRangeRef/StringRef do),
// `read_snapshot` and `report_conflicting_keys` works (CommitTransaction.h:184-188).
// Errors from the engine raise std::runtime_error: the reference has no error returns and
// aborts on ASSERT (SkipList.cpp:221), and this keeps failures loud.
#pragma once

#include <stdint.h>

#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "fdb_conflict_set.h"

namespace fdbcs_shim {

inline void check(int rc, const char* what) {
    if (rc != FDBCS_OK) throw std::runtime_error(std::string(what) + ": " + fdbcs_strerror(rc));
}

// Device ordinal for new conflict sets (one handle per GPU, like one resolver per process).
inline int& default_device() {
    static int d = 0;
    return d;
}

}  // namespace fdbcs_shim

struct ConflictSet {
    fdbcs_conflict_set* h = nullptr;
};

inline ConflictSet* newConflictSet() {  // SkipList.cpp:739-741
    ConflictSet* cs = new ConflictSet();
    fdbcs_shim::check(fdbcs_new_conflict_set(fdbcs_shim::default_device(), &cs->h), "newConflictSet");
    return cs;
}
inline void clearConflictSet(ConflictSet* cs, int64_t v) {  // SkipList.cpp:742-744
    fdbcs_shim::check(fdbcs_clear_conflict_set(cs->h, v), "clearConflictSet");
}
inline void destroyConflictSet(ConflictSet* cs) {  // SkipList.cpp:745-747
    fdbcs_destroy_conflict_set(cs->h);
    delete cs;
}

// ConflictingKeyRangeMap: std::map<int, VectorRef<int>> in FDB, filled with push_back(arena, i)
// (SkipList.cpp:782-784, 822-825) when the three-argument constructor receives the Arena; with
// the two-argument constructor any map whose mapped type supports push_back(int) works.
template <class ConflictingKeyRangeMap = std::map<int, std::vector<int>>>
struct ConflictBatchT {
    enum TransactionCommitResult {  // ConflictSet.h:40-44
        TransactionConflict = 0,
        TransactionTooOld,
        TransactionCommitted,
    };

    explicit ConflictBatchT(ConflictSet* cs, ConflictingKeyRangeMap* conflictingKeyRangeMap = nullptr)
      : cs(cs), map(conflictingKeyRangeMap) {
        fdbcs_shim::check(fdbcs_batch_new(cs->h, map != nullptr, &b), "ConflictBatch");
        append = [](typename ConflictingKeyRangeMap::mapped_type& e, int i) { e.push_back(i); };
    }
    // ConflictBatch(cs, conflictingKeyRangeMap, resolveBatchReplyArena) — SkipList.cpp:749-752.
    template <class Arena>
    ConflictBatchT(ConflictSet* cs, ConflictingKeyRangeMap* conflictingKeyRangeMap, Arena* arena)
      : cs(cs), map(conflictingKeyRangeMap) {
        fdbcs_shim::check(fdbcs_batch_new(cs->h, map != nullptr, &b), "ConflictBatch");
        append = [arena](typename ConflictingKeyRangeMap::mapped_type& e, int i) { e.push_back(*arena, i); };
    }
    ~ConflictBatchT() { fdbcs_batch_destroy(b); }
    ConflictBatchT(const ConflictBatchT&) = delete;
    ConflictBatchT& operator=(const ConflictBatchT&) = delete;

    template <class CommitTransactionRef>
    void addTransaction(const CommitTransactionRef& tr) {  // SkipList.cpp:763-794
        std::vector<const uint8_t*> rb, re, wb, we;
        std::vector<int32_t> rbl, rel, wbl, wel;
        for (const auto& r : tr.read_conflict_ranges) {
            rb.push_back(r.begin.begin());
            rbl.push_back((int32_t)r.begin.size());
            re.push_back(r.end.begin());
            rel.push_back((int32_t)r.end.size());
        }
        for (const auto& w : tr.write_conflict_ranges) {
            wb.push_back(w.begin.begin());
            wbl.push_back((int32_t)w.begin.size());
            we.push_back(w.end.begin());
            wel.push_back((int32_t)w.end.size());
        }
        fdbcs_shim::check(fdbcs_batch_add_transaction(b, tr.read_snapshot, tr.report_conflicting_keys ? 1 : 0,
                                                      (int32_t)rb.size(), rb.data(), rbl.data(), re.data(), rel.data(),
                                                      (int32_t)wb.size(), wb.data(), wbl.data(), we.data(), wel.data()),
                          "addTransaction");
        report.push_back(tr.report_conflicting_keys);
        hasReads.push_back(!tr.read_conflict_ranges.empty());
    }

    // SkipList.cpp:844-890: nonConflicting / tooOld lists as in :869-876.
    void detectConflicts(int64_t now, int64_t newOldestVersion, std::vector<int>& nonConflicting,
                         std::vector<int>* tooOldTransactions = nullptr) {
        verdicts.assign(report.size(), 0);
        fdbcs_shim::check(fdbcs_batch_detect_conflicts(b, now, newOldestVersion, verdicts.data(), nullptr, nullptr),
                          "detectConflicts");
        // A TooOld transaction's conflict status is set to true (`conflict = tr.tooOld`,
        // SkipList.cpp:820,830), so without a tooOld list it lands in neither list (:869-876).
        for (int i = 0; i < (int)verdicts.size(); i++) {
            if (verdicts[i] == TransactionTooOld) {
                if (tooOldTransactions) tooOldTransactions->push_back(i);
            } else if (verdicts[i] == TransactionCommitted) {
                nonConflicting.push_back(i);
            }
        }
        if (map) {
            std::vector<int32_t> idx;
            for (int t = 0; t < (int)report.size(); t++) {
                // the reference creates the entry while registering a reporting transaction's read
                // ranges (SkipList.cpp:777-784): admitted (not TooOld) and with at least one read
                if (!report[t] || !hasReads[t] || verdicts[t] == TransactionTooOld) continue;
                auto& entry = (*map)[t];
                int32_t n = 0;
                fdbcs_shim::check(fdbcs_batch_conflicting_reads(b, t, nullptr, 0, &n), "conflictingReads");
                idx.resize(n > 0 ? n : 1);
                fdbcs_shim::check(fdbcs_batch_conflicting_reads(b, t, idx.data(), n, &n), "conflictingReads");
                for (int32_t i = 0; i < n; i++) append(entry, idx[i]);
            }
        }
    }

    // SkipList.cpp:836-842: the add-time TooOld decisions (SkipList.cpp:770), valid right after
    // addTransaction, before detectConflicts, as in the reference.
    void GetTooOldTransactions(std::vector<int>& tooOldTransactions) {
        int32_t n = 0;
        fdbcs_shim::check(fdbcs_batch_too_old(b, nullptr, 0, &n), "GetTooOldTransactions");
        std::vector<int32_t> idx(n > 0 ? n : 1);
        fdbcs_shim::check(fdbcs_batch_too_old(b, idx.data(), n, &n), "GetTooOldTransactions");
        for (int32_t i = 0; i < n; i++) tooOldTransactions.push_back(idx[i]);
    }

private:
    ConflictSet* cs;
    ConflictingKeyRangeMap* map;
    fdbcs_batch* b = nullptr;
    std::function<void(typename ConflictingKeyRangeMap::mapped_type&, int)> append;
    std::vector<bool> report;
    std::vector<bool> hasReads;
    std::vector<uint8_t> verdicts;
};

using ConflictBatch = ConflictBatchT<>;
