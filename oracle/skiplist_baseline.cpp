// skiplist_baseline.cpp — TEST/BENCH INFRASTRUCTURE ONLY (never linked into the product).
//
// "Reference algorithm, restated": a clean-room C++ restatement of the resolver's conflict set as
// fdbserver/SkipList.cpp implements it, kept to the reference's data structure and its hot loops so
// that timing it on the GPU box's host is a fair CPU baseline (the reference binary itself cannot
// be built here).  It is cross-checked bit-exact against the semantic oracle
// (semantic_oracle.cpp) by tests/test_oracle.py and replayed on every bench run for parity.
//
// What it restates (every line number is fdbserver/SkipList.cpp):
//   * versioned skip list, 26 levels, LCG-driven random levels, per-level max versions, nodes of
//     [header | next pointers | max versions | key bytes] from 64 / 128-byte free lists   :210-297
//   * Finger descent with the alreadyChecked shortcut                                     :321-385
//   * read check: 16 CheckMax state machines advanced round-robin                          :426-458, :619-706
//   * striped interleaved find (stripes of 16 keys, back to front) and the merge of a stripe
//     (insert end at its inherited version, remove the interior, insert begin at `now`)     :414-424, :492-540, :574-617, :899-924
//   * bounded removeBefore resuming at removalKey (3 x |combined writes| + 10 nodes)       :542-571, :880-889
//   * MSD radix sortPoints (+5 byte offset, 0 terminator, then the endpoint class;
//     std::sort below 10 points)                                                           :89-132, :161-208
//   * MiniConflictSet over point indices (one bit per point) and the combine sweep         :797-834, :926-939
//   * addTransaction's TooOld rule and ConflictBatch::detectConflicts' order of phases     :763-794, :844-890
// Same C surface as the oracle (prefix slb_).  detect(..., gc): 0 = no GC, 1 = full removeBefore
// over the whole list (for history-size checks against the GPU engine's full GC), 2 = the
// reference's bounded, resumable removeBefore.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../include/fdb_conflict_set.h"

namespace {

constexpr int kLevels = 26;  // SkipList::MaxLevels (:212)

uint32_t g_rand = 0;  // skfastrand state (:42-47)
inline uint32_t lcg_next() {
    g_rand = g_rand * 1664525u + 1013904223u;
    return g_rand;
}
// randomLevel (:214-223): number of trailing ones of the top 25 bits of the LCG word.
inline int pick_level() {
    uint32_t bits = lcg_next() >> (32 - (kLevels - 1));
    int lv = 0;
    while (bits & 1u) {
        bits >>= 1;
        lv++;
    }
    return lv;
}

inline bool key_less(const uint8_t* a, int al, const uint8_t* b, int bl) {  // SkipList::less (:299-304)
    const int c = memcmp(a, b, (size_t)(uint32_t)std::min(al, bl));  // lengths are never negative
    return c < 0 || (c == 0 && al < bl);
}

// Node: {pointers, length} then next[pointers], maxVersion[pointers], key bytes (:227-297).
struct SNode {
    int32_t npt;
    int32_t klen;
    SNode** link() { return reinterpret_cast<SNode**>(this + 1); }
    int64_t* vmax() { return reinterpret_cast<int64_t*>(link() + npt); }
    uint8_t* key() { return reinterpret_cast<uint8_t*>(vmax() + npt); }
    int top() const { return npt - 1; }
    SNode* next(int l) { return link()[l]; }
    void set_next(int l, SNode* n) { link()[l] = n; }
    int64_t maxv(int l) { return vmax()[l]; }
    void set_maxv(int l, int64_t v) { vmax()[l] = v; }
    static size_t bytes(int npt, int klen) { return sizeof(SNode) + (size_t)npt * 16 + (size_t)klen; }
    // calcVersionForLevel (:269-275): max of level l-1 over this node's level-l span
    void recompute(int l) {
        SNode* stop = next(l);
        int64_t v = maxv(l - 1);
        for (SNode* y = next(l - 1); y != stop; y = y->next(l - 1)) v = std::max(v, y->maxv(l - 1));
        set_maxv(l, v);
    }
};

// FastAllocator<64> / <128> stand-ins (:248-257): size-class free lists over 4 MiB slabs.
struct Slabs {
    std::vector<void*> free64, free128, slabs;
    char* cur = nullptr;
    size_t left = 0;
    void* carve(size_t sz) {
        if (left < sz) {
            cur = (char*)malloc(1 << 22);
            slabs.push_back(cur);
            left = 1 << 22;
        }
        void* p = cur;
        cur += sz;
        left -= sz;
        return p;
    }
    void* get(size_t sz) {
        if (sz <= 64) {
            if (!free64.empty()) {
                void* p = free64.back();
                free64.pop_back();
                return p;
            }
            return carve(64);
        }
        if (sz <= 128) {
            if (!free128.empty()) {
                void* p = free128.back();
                free128.pop_back();
                return p;
            }
            return carve(128);
        }
        return malloc(sz);
    }
    void put(void* p, size_t sz) {
        if (sz <= 64)
            free64.push_back(p);
        else if (sz <= 128)
            free128.push_back(p);
        else
            free(p);
    }
    ~Slabs() {
        for (void* s : slabs) free(s);
    }
};

// Finger (:321-385): per level, the last node whose key is below the value.
struct Finger {
    SNode* at[kLevels];
    int level = kLevels;
    SNode* x = nullptr;
    SNode* seen = nullptr;  // alreadyChecked: the first node known not below the value
    const uint8_t* k = nullptr;
    int kl = 0;

    void start(const uint8_t* key, int len, SNode* head) {
        k = key;
        kl = len;
        x = head;
        seen = nullptr;
        level = kLevels;
    }
    void prefetch() {
        SNode* n = x->next(level - 1);
        _mm_prefetch((const char*)n, _MM_HINT_T0);
        _mm_prefetch((const char*)n + 64, _MM_HINT_T0);
    }
    // one step right at the current level, or one level down (returns true when it went down)
    bool step() {
        SNode* n = x->next(level - 1);
        if (n == seen || !key_less(n->key(), n->klen, k, kl)) {
            seen = n;
            level--;
            at[level] = x;
            return true;
        }
        x = n;
        return false;
    }
    void down() {
        while (!step()) {
        }
    }
    bool done() const { return level == 0; }
    SNode* hit() const {
        SNode* n = at[0]->next(0);
        return (n && n->klen == kl && !memcmp(n->key(), k, (size_t)kl)) ? n : nullptr;
    }
};

struct Point {  // KeyInfo (:77-87)
    const uint8_t* key;
    int32_t len;
    uint8_t begin, write;
    int32_t txn;
    int32_t* slot;  // pIndex
};
inline int point_class(const Point& p) { return p.begin * 2 + (p.write ^ p.begin); }  // extra_ordering (:89-91)
inline bool point_less(const Point& a, const Point& b) {                               // operator< (:117-132)
    const int c = memcmp(a.key, b.key, (size_t)std::min(a.len, b.len));
    if (c) return c < 0;
    if (a.len != b.len) return a.len < b.len;
    return point_class(a) < point_class(b);
}
// getCharacter (:94-115): digit of a point at a byte position; true once past every digit.
inline bool digit(const Point& p, int pos, int& d) {
    if (pos < p.len) {
        d = 5 + p.key[pos];
        return false;
    }
    if (pos == p.len) {
        d = 0;
        return false;
    }
    if (pos == p.len + 1) {
        d = point_class(p);
        return false;
    }
    d = 0;
    return true;
}

// sortPoints (:161-208): MSD radix, one counting pass per (range, byte position), a stack of tasks.
void radix_sort_points(std::vector<Point>& pts) {
    struct Task {
        int lo, n, pos;
    };
    std::vector<Task> todo{{0, (int)pts.size(), 0}};
    std::vector<Point> scratch;
    int cnt[261];
    while (!todo.empty()) {
        const Task t = todo.back();
        todo.pop_back();
        if (t.n < 10) {
            std::sort(pts.begin() + t.lo, pts.begin() + t.lo + t.n, point_less);
            continue;
        }
        memset(cnt, 0, sizeof(cnt));
        bool finished = true;
        int d;
        for (int i = t.lo; i < t.lo + t.n; i++) {
            finished &= digit(pts[i], t.pos, d);
            cnt[d]++;
        }
        if (finished) continue;
        int run = 0;
        for (int b = 0; b < 261; b++) {
            const int c = cnt[b];
            if (c > 1) todo.push_back({t.lo + run, c, t.pos + 1});
            cnt[b] = run;
            run += c;
        }
        scratch.resize(t.n);
        for (int i = t.lo; i < t.lo + t.n; i++) {
            digit(pts[i], t.pos, d);
            scratch[cnt[d]++] = pts[i];
        }
        std::copy(scratch.begin(), scratch.begin() + t.n, pts.begin() + t.lo);
    }
}

struct ReadRange {  // ReadConflictRange (:62-75)
    const uint8_t *b, *e;
    int32_t bl, el;
    int64_t snap;
    int32_t txn, idx;
};

struct SkipSet {
    Slabs mem;
    SNode* head = nullptr;
    int64_t count = 0;

    SNode* make(const uint8_t* k, int len, int lv) {  // Node::create (:244-266)
        SNode* n = (SNode*)mem.get(SNode::bytes(lv + 1, len));
        n->npt = lv + 1;
        n->klen = len;
        if (len) memcpy(n->key(), k, (size_t)len);
        return n;
    }
    void drop(SNode* n) { mem.put(n, SNode::bytes(n->npt, n->klen)); }

    void reset(int64_t v) {  // SkipList(Version) (:398-404)
        if (head) {
            for (SNode* x = head->next(0); x;) {
                SNode* nx = x->next(0);
                drop(x);
                x = nx;
            }
            drop(head);
        }
        head = make(nullptr, 0, kLevels - 1);
        for (int l = 0; l < kLevels; l++) {
            head->set_next(l, nullptr);
            head->set_maxv(l, v);
        }
        count = 0;
    }

    // insert(finger, version) (:591-610)
    void insert_at(const Finger& f, int64_t version) {
        const int lv = pick_level();
        SNode* x = make(f.k, f.kl, lv);
        x->set_maxv(0, version);
        for (int i = 0; i <= lv; i++) {
            x->set_next(i, f.at[i]->next(i));
            f.at[i]->set_next(i, x);
        }
        for (int i = 1; i <= lv; i++) {
            f.at[i]->recompute(i);
            x->recompute(i);
        }
        for (int i = lv + 1; i < kLevels; i++) {
            if (f.at[i]->maxv(i) >= version) break;
            f.at[i]->set_maxv(i, version);
        }
        count++;
    }

    // remove(start, end) (:574-589): unlink the nodes after start up to and including end.finger[0]
    void remove_between(const Finger& s, const Finger& e) {
        if (s.at[0] == e.at[0]) return;
        SNode* x = s.at[0]->next(0);
        for (int i = 0; i < kLevels; i++)
            if (s.at[i] != e.at[i]) s.at[i]->set_next(i, e.at[i]->next(i));
        for (;;) {
            SNode* nx = x->next(0);
            const bool last = x == e.at[0];
            drop(x);
            count--;
            if (last) break;
            x = nx;
        }
    }

    // addConflictRanges(fingers, n, version) (:414-424): back to front within a stripe
    void merge_stripe(const Finger* f, int n, int64_t version) {
        for (int r = n - 1; r >= 0; r--) {
            const Finger& fb = f[2 * r];
            const Finger& fe = f[2 * r + 1];
            if (!fe.hit()) insert_at(fe, fe.at[0]->maxv(0));
            remove_between(fb, fe);
            insert_at(fb, version);
        }
    }

    // find(values, results, temp, count) (:492-540): descend together while every value lies in the
    // same part of the list, then advance the fingers round-robin with prefetches.
    void find(const uint8_t* const* keys, const int32_t* lens, Finger* out, int* nextj, int n) {
        out[0].start(keys[0], lens[0], head);
        const uint8_t* ek = keys[n - 1];
        const int el = lens[n - 1];
        while (out[0].level > 1) {
            out[0].down();
            SNode* ac = out[0].seen;
            if (ac && key_less(ac->key(), ac->klen, ek, el)) break;
        }
        const int lv0 = out[0].level + 1;
        SNode* x = lv0 < kLevels ? out[0].at[lv0] : head;
        for (int i = 1; i < n; i++) {
            out[i].level = lv0;
            out[i].x = x;
            out[i].seen = nullptr;
            out[i].k = keys[i];
            out[i].kl = lens[i];
            for (int j = lv0; j < kLevels; j++) out[i].at[j] = out[0].at[j];
        }
        for (int i = 0; i < n - 1; i++) nextj[i] = i + 1;
        nextj[n - 1] = 0;
        int prev = n - 1, j = 0;
        for (;;) {
            Finger* f = &out[j];
            f->step();
            if (f->done()) {
                if (prev == j) break;
                nextj[prev] = nextj[j];
            } else {
                f->prefetch();
                prev = j;
            }
            j = nextj[j];
        }
    }

    // removeBefore(v, finger, nodeCount) (:542-571)
    int remove_before(int64_t v, Finger& f, int64_t budget) {
        int removed = 0;
        bool was_above = true;
        while (budget--) {
            SNode* x = f.at[0]->next(0);
            if (!x) break;
            _mm_prefetch((const char*)x->next(0), _MM_HINT_T0);
            _mm_prefetch((const char*)x->next(x->top() >= 1 ? 1 : 0), _MM_HINT_T0);
            const bool above = x->maxv(0) >= v;
            if (above || was_above) {
                for (int l = 0; l <= x->top(); l++) f.at[l] = x;
            } else {
                removed++;
                for (int l = 0; l <= x->top(); l++) f.at[l]->set_next(l, x->next(l));
                for (int i = 1; i <= x->top(); i++) f.at[i]->set_maxv(i, std::max(f.at[i]->maxv(i), x->maxv(i)));
                drop(x);
                count--;
            }
            was_above = above;
        }
        return removed;
    }
};

// CheckMax (:619-706): one read range's history check as a resumable state machine; advance()
// returns true when the verdict for the range is known.
struct ReadProbe {
    Finger s, e;
    int64_t snap;
    uint8_t* result;
    int state;
    std::vector<int32_t>* report;
    int32_t idx;

    void start(const ReadRange& r, SNode* head, uint8_t* status, std::vector<int32_t>* rep) {
        s.start(r.b, r.bl, head);
        e.start(r.e, r.el, head);
        snap = r.snap;
        result = &status[r.txn];
        report = rep;
        idx = r.idx;
        state = 0;
    }
    bool fine() { return true; }
    bool hit() {
        *result = 1;
        if (report) report->push_back(idx);
        return true;
    }
    bool advance() {
        if (state == 0) {
            // descend both fingers until they part; a shared span at or below the snapshot decides
            for (;;) {
                if (!s.step()) {
                    s.prefetch();
                    return false;
                }
                e.x = s.x;
                e.down();
                const int l = s.level;
                if (s.at[l] != e.at[l]) break;
                if (s.at[l]->maxv(l) <= snap) return fine();
                if (l == 0) return hit();
            }
            state = 1;
        }
        // end side: walk the spans between the diverged fingers at each level going down
        SNode* n = e.at[e.level];
        while (n->maxv(e.level) > snap) {
            if (e.done()) return hit();
            e.down();
            SNode* stop = e.at[e.level];
            while (n != stop) {
                if (n->maxv(e.level) > snap) return hit();
                n = n->next(e.level);
            }
        }
        // start side
        SNode* lim = e.at[s.level];
        for (;;) {
            SNode* after = s.at[s.level]->next(s.level);
            for (SNode* p = after; p != lim; p = p->next(s.level))
                if (p->maxv(s.level) > snap) return hit();
            if (s.at[s.level]->maxv(s.level) <= snap) return fine();
            lim = after;
            if (s.done()) {
                if (after->klen == s.kl && !memcmp(after->key(), s.k, (size_t)s.kl)) return fine();
                return hit();
            }
            s.down();
        }
    }
};

// SkipList::detectConflicts (:426-458): 16 probes in flight, a ring of the unfinished ones.
void check_reads(SkipSet& sl, const std::vector<ReadRange>& rr, uint8_t* status,
                 std::vector<std::vector<int32_t>>& confl, const uint8_t* report) {
    constexpr int M = 16;
    const int n = (int)rr.size();
    if (!n) return;
    ReadProbe probe[M];
    int nextj[M];
    auto rep_of = [&](const ReadRange& r) { return report[r.txn] ? &confl[r.txn] : nullptr; };
    int started = std::min(M, n);
    for (int i = 0; i < started; i++) {
        probe[i].start(rr[i], sl.head, status, rep_of(rr[i]));
        nextj[i] = i + 1;
    }
    nextj[started - 1] = 0;
    int prev = started - 1, j = 0;
    for (;;) {
        if (probe[j].advance()) {
            if (started == n) {
                if (prev == j) break;
                nextj[prev] = nextj[j];
                j = prev;
            } else {
                const int q = started++;
                probe[j].start(rr[q], sl.head, status, rep_of(rr[q]));
            }
        }
        prev = j;
        j = nextj[j];
    }
}

struct ConflictSet {
    SkipSet list;
    std::string removal_key;  // ConflictSet::removalKey (:735)
    int64_t oldest = 0;
    // The oldest version the next batch's addTransaction saw, when the caller added it before the
    // previous batch's detect (a ConflictBatch reads cs->oldestVersion at add, SkipList.cpp:770);
    // INT64_MIN: added right before its detect, as the Resolver does.  One-shot.
    int64_t add_oldest = INT64_MIN;
    double last[8] = {};  // seconds of the last detect: add, sort, check, intra, combine, merge, gc, total
};

inline double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

}  // namespace

extern "C" {

void* slb_new(void) {
    ConflictSet* cs = new ConflictSet();
    cs->list.reset(0);
    return cs;
}
void slb_destroy(void* p) {
    ConflictSet* cs = (ConflictSet*)p;
    cs->list.reset(0);
    cs->list.drop(cs->list.head);
    cs->list.head = nullptr;
    delete cs;
}
void slb_clear(void* p, int64_t v) { ((ConflictSet*)p)->list.reset(v); }  // clearConflictSet (:742-744)
void slb_set_oldest(void* p, int64_t v) {
    ConflictSet* cs = (ConflictSet*)p;
    if (v > cs->oldest) cs->oldest = v;
}
int64_t slb_oldest(void* p) { return ((ConflictSet*)p)->oldest; }
void slb_set_add_oldest(void* p, int64_t v) { ((ConflictSet*)p)->add_oldest = v; }
int64_t slb_history_size(void* p) { return ((ConflictSet*)p)->list.count; }
void slb_last_times(void* p, double* out) { memcpy(out, ((ConflictSet*)p)->last, sizeof(double) * 8); }

// Prefill: boundaries arrive sorted, so every level is appended at its tail, then the level
// maxima are computed bottom-up (the reference has no bulk load; the resulting list is one the
// reference could have built by inserting the same keys).
void slb_load_history(void* p, int64_t n, const uint8_t* bytes, const int64_t* offs, const int64_t* vers,
                      int64_t header) {
    SkipSet& s = ((ConflictSet*)p)->list;
    s.reset(header);
    SNode* tails[kLevels];
    for (int l = 0; l < kLevels; l++) tails[l] = s.head;
    for (int64_t i = 0; i < n; i++) {
        const int lv = pick_level();
        SNode* x = s.make(bytes + offs[i], (int)(offs[i + 1] - offs[i]), lv);
        x->set_maxv(0, vers[i]);
        for (int l = 0; l <= lv; l++) {
            x->set_next(l, nullptr);
            tails[l]->set_next(l, x);
            tails[l] = x;
        }
        s.count++;
    }
    for (int l = 1; l < kLevels; l++)
        for (SNode* x = s.head; x; x = x->next(l)) x->recompute(l);
}

// ConflictBatch: addTransaction for every transaction (:763-794), then detectConflicts (:844-890).
int64_t slb_detect(void* p, const fdbcs_packed_batch* pb, int64_t now, int64_t newOldest, uint8_t* verdicts,
                   int32_t* conf_off, int32_t* conf_idx, int64_t cap, int gc) {
    const int64_t add_oldest = ((ConflictSet*)p)->add_oldest != INT64_MIN ? ((ConflictSet*)p)->add_oldest
                                                                           : ((ConflictSet*)p)->oldest;
    ((ConflictSet*)p)->add_oldest = INT64_MIN;
    ConflictSet* cs = (ConflictSet*)p;
    SkipSet& sl = cs->list;
    const double t0 = now_s();
    const int T = pb->n_txn;
    const int R = T ? pb->read_offsets[T] : 0;
    const int W = T ? pb->write_offsets[T] : 0;
    auto K = [&](int64_t k) { return pb->key_bytes + pb->key_offsets[k]; };
    auto KL = [&](int64_t k) { return (int32_t)(pb->key_offsets[k + 1] - pb->key_offsets[k]); };

    // ---- addTransaction
    std::vector<uint8_t> too_old(T, 0), report(T, 0), status(T, 0);
    std::vector<int32_t> ridx(2 * (size_t)R), widx(2 * (size_t)W);  // readRanges / writeRanges index pairs
    std::vector<Point> pts;
    pts.reserve(2 * (size_t)(R + W));
    std::vector<ReadRange> reads;
    reads.reserve(R);
    std::vector<std::vector<int32_t>> confl(T);
    for (int t = 0; t < T; t++) {
        const int r0 = pb->read_offsets[t], r1 = pb->read_offsets[t + 1];
        const int w0 = pb->write_offsets[t], w1 = pb->write_offsets[t + 1];
        report[t] = pb->report_conflicting_keys ? pb->report_conflicting_keys[t] : 0;
        if (pb->read_snapshot[t] < add_oldest && r1 > r0) {  // :770
            too_old[t] = 1;
            continue;
        }
        for (int r = r0; r < r1; r++) {
            pts.push_back({K(2 * r), KL(2 * r), 1, 0, t, &ridx[2 * r]});
            pts.push_back({K(2 * r + 1), KL(2 * r + 1), 0, 0, t, &ridx[2 * r + 1]});
            reads.push_back({K(2 * r), K(2 * r + 1), KL(2 * r), KL(2 * r + 1), pb->read_snapshot[t], t, r - r0});
        }
        for (int w = w0; w < w1; w++) {
            const int64_t k = 2 * ((int64_t)R + w);
            pts.push_back({K(k), KL(k), 1, 1, t, &widx[2 * w]});
            pts.push_back({K(k + 1), KL(k + 1), 0, 1, t, &widx[2 * w + 1]});
        }
    }
    const double t1 = now_s();

    // ---- sortPoints
    radix_sort_points(pts);
    const double t2 = now_s();

    // ---- checkReadConflictRanges
    check_reads(sl, reads, status.data(), confl, report.data());
    const double t3 = now_s();

    // ---- checkIntraBatchConflicts: MiniConflictSet over point indices (:797-834)
    for (size_t i = 0; i < pts.size(); i++) *pts[i].slot = (int32_t)i;
    std::vector<bool> mcs(pts.size(), false);
    for (int t = 0; t < T; t++) {
        if (status[t]) continue;
        bool c = too_old[t];
        if (!c) {
            for (int r = pb->read_offsets[t]; r < pb->read_offsets[t + 1]; r++) {
                bool any = false;
                for (int i = ridx[2 * r]; i < ridx[2 * r + 1] && !any; i++) any = mcs[i];
                if (any) {
                    if (report[t]) confl[t].push_back(r - pb->read_offsets[t]);
                    c = true;
                    break;
                }
            }
        }
        status[t] = c;
        if (!c)
            for (int w = pb->write_offsets[t]; w < pb->write_offsets[t + 1]; w++)
                for (int i = widx[2 * w]; i < widx[2 * w + 1]; i++) mcs[i] = true;
    }
    const double t4 = now_s();

    // ---- combineWriteConflictRanges (:926-939)
    std::vector<const uint8_t*> ck;
    std::vector<int32_t> cl;
    int active = 0;
    for (const Point& q : pts) {
        if (!q.write || status[q.txn]) continue;
        if (q.begin) {
            if (++active == 1) {
                ck.push_back(q.key);
                cl.push_back(q.len);
                ck.push_back(nullptr);
                cl.push_back(0);
            }
        } else if (--active == 0) {
            ck.back() = q.key;
            cl.back() = q.len;
        }
    }
    const double t5 = now_s();

    // ---- mergeWriteConflictRanges: stripes of 16 keys, back to front (:899-924)
    const int nstr = (int)ck.size();
    if (nstr) {
        constexpr int kStripe = 16;
        Finger f[kStripe];
        int tmp[kStripe];
        const int stripes = (nstr + kStripe - 1) / kStripe;
        int ss = nstr - (stripes - 1) * kStripe;
        for (int s = stripes - 1; s >= 0; s--) {
            sl.find(&ck[(size_t)s * kStripe], &cl[(size_t)s * kStripe], f, tmp, ss);
            sl.merge_stripe(f, ss / 2, now);
            ss = kStripe;
        }
    }
    const double t6 = now_s();

    for (int t = 0; t < T; t++)  // :869-876
        verdicts[t] = too_old[t] ? FDBCS_TRANSACTION_TOO_OLD
                                 : (status[t] ? FDBCS_TRANSACTION_CONFLICT : FDBCS_TRANSACTION_COMMITTED);

    // ---- removeBefore (:880-889)
    if (newOldest > cs->oldest) {
        cs->oldest = newOldest;
        if (gc == 2) {
            Finger f;
            int tmp;
            const uint8_t* rk = (const uint8_t*)cs->removal_key.data();
            const int32_t rl = (int32_t)cs->removal_key.size();
            sl.find(&rk, &rl, &f, &tmp, 1);
            sl.remove_before(cs->oldest, f, (int64_t)(nstr / 2) * 3 + 10);
            SNode* nx = f.at[0]->next(0);  // Finger::getValue (:381-384)
            cs->removal_key.assign(nx ? (const char*)nx->key() : "", nx ? (size_t)nx->klen : 0);
        } else if (gc == 1) {
            Finger f;
            int tmp;
            const uint8_t* rk = (const uint8_t*)"";
            const int32_t rl = 0;
            sl.find(&rk, &rl, &f, &tmp, 1);
            sl.remove_before(cs->oldest, f, INT64_MAX);
        }
    }
    const double t7 = now_s();
    const double times[8] = {t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t7 - t6, t7 - t0};
    memcpy(cs->last, times, sizeof(times));

    int64_t n = 0;
    conf_off[0] = 0;
    for (int t = 0; t < T; t++) {
        std::sort(confl[t].begin(), confl[t].end());
        for (int i : confl[t]) {
            if (n >= cap) return -1;
            conf_idx[n++] = i;
        }
        conf_off[t + 1] = (int32_t)n;
    }
    return n;
}

}  // extern "C"
