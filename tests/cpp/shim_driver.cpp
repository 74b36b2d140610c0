// Drives the reference-shaped C++ API (include/conflict_set_shim.hpp) with stand-in
// CommitTransactionRef/KeyRangeRef types, the way Resolver.actor.cpp:179-194 does.
// Prints one verdict digit per transaction per batch.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "conflict_set_shim.hpp"

struct Ref {  // StringRef-like
    std::string s;
    const uint8_t* begin() const { return (const uint8_t*)s.data(); }
    int size() const { return (int)s.size(); }
};
struct Range {
    Ref begin, end;
};
struct Arena {  // flow Arena stand-in: counts allocations made through it
    int pushes = 0;
};
struct IntVectorRef {  // VectorRef<int> stand-in: push_back(arena, v) like flow/Arena.h
    std::vector<int> v;
    void push_back(Arena& a, int x) {
        a.pushes++;
        v.push_back(x);
    }
    size_t size() const { return v.size(); }
};
struct Txn {
    std::vector<Range> read_conflict_ranges, write_conflict_ranges;
    int64_t read_snapshot = 0;
    bool report_conflicting_keys = false;
};

int main() {
    ConflictSet* cs = newConflictSet();
    // batch 1: T0 writes [k, k\0); T1 reads it (intra-batch conflict); T2 reads [a, b)
    {
        std::map<int, std::vector<int>> ckr;
        ConflictBatch batch(cs, &ckr);
        Txn t0, t1, t2;
        t0.write_conflict_ranges.push_back({{"k"}, {std::string("k\0", 2)}});
        t1.read_conflict_ranges.push_back({{"k"}, {std::string("k\0", 2)}});
        t1.report_conflicting_keys = true;
        t2.read_conflict_ranges.push_back({{"a"}, {"b"}});
        batch.addTransaction(t0);
        batch.addTransaction(t1);
        batch.addTransaction(t2);
        std::vector<int> ok, tooOld;
        batch.detectConflicts(10, 0, ok, &tooOld);
        printf("b1 commit=%zu tooold=%zu report1=%zu\n", ok.size(), tooOld.size(), ckr[1].size());
    }
    // batch 2: snapshot 5 reads of k see version 10 -> conflict; snapshot 10 commits
    {
        ConflictBatch batch(cs);
        Txn a, b;
        a.read_conflict_ranges.push_back({{"k"}, {"l"}});
        a.read_snapshot = 5;
        b.read_conflict_ranges.push_back({{"k"}, {"l"}});
        b.read_snapshot = 10;
        batch.addTransaction(a);
        batch.addTransaction(b);
        std::vector<int> ok;
        batch.detectConflicts(20, 0, ok);
        printf("b2 commit=%zu first=%d\n", ok.size(), ok.empty() ? -1 : ok[0]);
    }
    // batch 3: the Resolver's three-argument form with an Arena-backed map (Resolver.actor.cpp:179)
    {
        std::map<int, IntVectorRef> ckr;
        Arena arena;
        ConflictBatchT<std::map<int, IntVectorRef>> batch(cs, &ckr, &arena);
        Txn a;
        a.read_conflict_ranges.push_back({{"a"}, {"b"}});
        a.read_conflict_ranges.push_back({{"k"}, {"l"}});
        a.read_snapshot = 5;
        a.report_conflicting_keys = true;
        batch.addTransaction(a);
        std::vector<int> ok;
        batch.detectConflicts(30, 0, ok);
        printf("b3 commit=%zu report0=%zu idx=%d arena=%d\n", ok.size(), ckr[0].size(),
               ckr[0].size() ? ckr[0].v[0] : -1, arena.pushes);
    }
    // batch 4: raise oldestVersion to 35; batch 5 then holds a reader below it (TooOld, SkipList.cpp:770),
    // a writer-only transaction below it (not TooOld: it has no reads) and a reporting writer-only
    // transaction (no map entry: the entry is created in addTransaction's read loop, :781-784)
    {
        ConflictBatch batch(cs);
        std::vector<int> ok;
        batch.detectConflicts(40, 35, ok);
    }
    {
        std::map<int, std::vector<int>> ckr;
        ConflictBatch batch(cs, &ckr);
        Txn a, w, r;
        a.read_conflict_ranges.push_back({{"x"}, {"y"}});
        a.read_snapshot = 20;
        w.write_conflict_ranges.push_back({{"x"}, {"y"}});
        w.read_snapshot = 20;
        r.write_conflict_ranges.push_back({{"p"}, {"q"}});
        r.read_snapshot = 38;
        r.report_conflicting_keys = true;
        batch.addTransaction(a);
        batch.addTransaction(w);
        batch.addTransaction(r);
        std::vector<int> ok, tooOld, late;
        batch.detectConflicts(50, 35, ok, &tooOld);
        batch.GetTooOldTransactions(late);  // SkipList.cpp:836-842
        printf("b5 commit=%zu tooold=%zu late=%zu late0=%d entries=%zu\n", ok.size(), tooOld.size(), late.size(),
               late.empty() ? -1 : late[0], ckr.size());
    }
    // batch 6: without a tooOld list the reference files a TooOld transaction as non-conflicting
    // (its conflict status is never set, SkipList.cpp:869-876)
    {
        ConflictBatch batch(cs);
        Txn a;
        a.read_conflict_ranges.push_back({{"x"}, {"y"}});
        a.read_snapshot = 20;
        batch.addTransaction(a);
        std::vector<int> ok;
        batch.detectConflicts(60, 35, ok);
        printf("b6 commit=%zu first=%d\n", ok.size(), ok.empty() ? -1 : ok[0]);
    }
    destroyConflictSet(cs);
    return 0;
}
