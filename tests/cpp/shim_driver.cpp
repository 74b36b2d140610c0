// Drives the reference-shaped C++ API (include/conflict_set_shim.hpp) with stand-in
// CommitTransactionRef/KeyRangeRef types, the way Resolver.actor.cpp:179-194 does.
// Prints one verdict digit per transaction per batch.
#include <stdio.h>
#include <stdlib.h>
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

static std::string unhex(const std::string& h) {
    std::string out;
    if (h == "-") return out;
    for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back((char)strtol(h.substr(i, 2).c_str(), nullptr, 16));
    return out;
}

static void print_list(const char* name, const std::vector<int>& v) {
    printf(" %s=", name);
    for (size_t i = 0; i < v.size(); i++) printf(i ? ",%d" : "%d", v[i]);
}

// --lists FILE: replays the batches of FILE through two conflict sets, calling detectConflicts
// with a tooOld list on one and without it (nullptr, skipListTest's call shape, SkipList.cpp:1077)
// on the other, and prints both sets of lists per batch.  FILE lines:
//   S                         new scenario (fresh conflict sets)
//   C <version>               clearConflictSet on both
//   B <now> <newOldest> <T>   a batch of T transactions, each on a line:
//   T <snapshot> <report> <nr> <nw> <hex key> x 2(nr+nw)   ("-" = empty key)
static int run_lists(const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) return 2;
    ConflictSet *with = nullptr, *without = nullptr;
    char tok[8];
    int batch = 0;
    while (fscanf(f, "%7s", tok) == 1) {
        if (tok[0] == 'S') {
            if (with) destroyConflictSet(with), destroyConflictSet(without);
            with = newConflictSet();
            without = newConflictSet();
            batch = 0;
        } else if (tok[0] == 'C') {
            long long v;
            if (fscanf(f, "%lld", &v) != 1) return 3;
            clearConflictSet(with, v);
            clearConflictSet(without, v);
        } else if (tok[0] == 'B') {
            long long now, oldest;
            int T;
            if (fscanf(f, "%lld %lld %d", &now, &oldest, &T) != 3) return 3;
            std::vector<Txn> txns(T);
            for (int t = 0; t < T; t++) {
                long long snap;
                int rep, nr, nw;
                if (fscanf(f, "%7s %lld %d %d %d", tok, &snap, &rep, &nr, &nw) != 5) return 3;
                txns[t].read_snapshot = snap;
                txns[t].report_conflicting_keys = rep != 0;
                char buf[4096];
                for (int r = 0; r < nr + nw; r++) {
                    Range rg;
                    if (fscanf(f, "%4095s", buf) != 1) return 3;
                    rg.begin.s = unhex(buf);
                    if (fscanf(f, "%4095s", buf) != 1) return 3;
                    rg.end.s = unhex(buf);
                    (r < nr ? txns[t].read_conflict_ranges : txns[t].write_conflict_ranges).push_back(rg);
                }
            }
            ConflictBatch a(with), b(without);
            for (auto& t : txns) a.addTransaction(t), b.addTransaction(t);
            std::vector<int> nc, to, nc2, early;
            a.GetTooOldTransactions(early);  // before detect, as SkipList.cpp:836-842 allows
            a.detectConflicts(now, oldest, nc, &to);
            if (early != to) return 4;
            b.detectConflicts(now, oldest, nc2);
            printf("L %d with", batch);
            print_list("nc", nc);
            print_list("to", to);
            printf("\nL %d without", batch);
            print_list("nc", nc2);
            printf("\n");
            batch++;
        } else {
            return 3;
        }
    }
    if (with) destroyConflictSet(with), destroyConflictSet(without);
    fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 3 && strcmp(argv[1], "--lists") == 0) return run_lists(argv[2]);
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
        std::vector<int> ok, tooOld, late, early;
        batch.GetTooOldTransactions(early);  // right after the adds
        if (early.size() != 1 || early[0] != 0) return 5;
        batch.detectConflicts(50, 35, ok, &tooOld);
        batch.GetTooOldTransactions(late);  // SkipList.cpp:836-842
        printf("b5 commit=%zu tooold=%zu late=%zu late0=%d entries=%zu\n", ok.size(), tooOld.size(), late.size(),
               late.empty() ? -1 : late[0], ckr.size());
    }
    // batch 6: without a tooOld list a TooOld transaction lands in neither list: its conflict status
    // is set to true (`conflict = tr.tooOld`, SkipList.cpp:820,830) and :873 skips it
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
