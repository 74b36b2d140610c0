// skiplist_baseline.cpp — TEST/BENCH INFRASTRUCTURE ONLY (never linked into the product).
//
// Performance-faithful CPU restatement of the reference resolver data structure
// (fdbserver/SkipList.cpp): a versioned skip list whose level-0 nodes are
// history boundaries and whose level-l "max version" covers the level-l span
// (SkipList.cpp:210-241), range-max read checks (the job of CheckMax,
// SkipList.cpp:619-706), a word-parallel MiniConflictSet (SkipList.cpp:797-834),
// the write-range combine sweep (SkipList.cpp:926-939), merge of committed writes
// (SkipList.cpp:414-424, 574-617) and removeBefore GC (SkipList.cpp:542-571).
// It is timed single-threaded by bench.py as the "cpu_baseline" (kind "port":
// the reference binary itself cannot be built here), and is
// cross-checked bit-exact against semantic_oracle.cpp by tests/.
// Same C surface as the oracle, prefix slb_.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../include/fdb_conflict_set.h"

namespace {

constexpr int kLevels = 26;  // SkipList::MaxLevels (SkipList.cpp:212)

inline int cmpBytes(const uint8_t* a, int al, const uint8_t* b, int bl) {
    int c = memcmp(a, b, (size_t)std::min(al, bl));
    if (c) return c < 0 ? -1 : 1;
    return (al > bl) - (al < bl);
}

struct Node {
    int32_t height;  // number of levels (>= 1)
    int32_t len;
    // followed by: Node* next[height]; int64_t maxv[height]; uint8_t key[len]
    Node** nexts() { return reinterpret_cast<Node**>(this + 1); }
    int64_t* maxv() { return reinterpret_cast<int64_t*>(nexts() + height); }
    uint8_t* key() { return reinterpret_cast<uint8_t*>(maxv() + height); }
    static size_t bytes(int h, int len) { return sizeof(Node) + (size_t)h * 16 + (size_t)len; }
};

// Size-class free lists stand in for FastAllocator<64/128> (SkipList.cpp:244-266).
struct Pool {
    std::vector<void*> free64, free128;
    std::vector<void*> slabs;
    char* cur = nullptr;
    size_t left = 0;
    void* raw(size_t sz) {
        if (left < sz) {
            size_t slab = 1 << 22;
            cur = (char*)malloc(slab);
            slabs.push_back(cur);
            left = slab;
        }
        void* p = cur;
        cur += sz;
        left -= sz;
        return p;
    }
    void* alloc(size_t sz) {
        if (sz <= 64) {
            if (!free64.empty()) { void* p = free64.back(); free64.pop_back(); return p; }
            return raw(64);
        }
        if (sz <= 128) {
            if (!free128.empty()) { void* p = free128.back(); free128.pop_back(); return p; }
            return raw(128);
        }
        return malloc(sz);
    }
    void release(void* p, size_t sz) {
        if (sz <= 64) free64.push_back(p);
        else if (sz <= 128) free128.push_back(p);
        else free(p);
    }
    ~Pool() { for (void* s : slabs) free(s); }
};

struct SkipSet {
    Pool pool;
    Node* head = nullptr;
    uint32_t seed = 1;
    int64_t oldest = 0;
    int64_t count = 0;

    int pickHeight() {  // geometric, p = 1/2 (SkipList.cpp:214-223), LCG as SkipList.cpp:42-47
        seed = seed * 1664525u + 1013904223u;
        uint32_t bits = seed >> 7;
        int h = 1;
        while ((bits & 1) && h < kLevels) { bits >>= 1; h++; }
        return h;
    }
    Node* make(const uint8_t* k, int len, int h) {
        Node* n = (Node*)pool.alloc(Node::bytes(h, len));
        n->height = h;
        n->len = len;
        if (len) memcpy(n->key(), k, (size_t)len);
        return n;
    }
    void drop(Node* n) { pool.release(n, Node::bytes(n->height, n->len)); }

    void reset(int64_t v) {
        if (head) {
            Node* x = head->nexts()[0];
            while (x) { Node* nx = x->nexts()[0]; drop(x); x = nx; }
            drop(head);
        }
        head = make(nullptr, 0, kLevels);
        for (int l = 0; l < kLevels; l++) { head->nexts()[l] = nullptr; head->maxv()[l] = v; }
        count = 0;
    }

    // preds[l] = last node at level l with key < k (strict: ge == false) or <= k.
    void descend(const uint8_t* k, int len, bool orEqual, Node** preds) {
        Node* x = head;
        for (int l = kLevels - 1; l >= 0; l--) {
            for (;;) {
                Node* n = x->nexts()[l];
                if (!n) break;
                int c = cmpBytes(n->key(), n->len, k, len);
                if (c < 0 || (orEqual && c == 0)) {
                    __builtin_prefetch(n->nexts()[l < n->height ? l : 0]);
                    x = n;
                } else break;
            }
            preds[l] = x;
        }
    }

    // maxv[l] of `x` = max of level-(l-1) maxv over its level-l span (calcVersionForLevel, SkipList.cpp:268-275).
    static void recompute(Node* x, int l) {
        Node* end = x->nexts()[l];
        int64_t v = x->maxv()[l - 1];
        for (Node* y = x->nexts()[l - 1]; y != end; y = y->nexts()[l - 1]) v = std::max(v, y->maxv()[l - 1]);
        x->maxv()[l] = v;
    }

    // Range max over segments meeting [b, e), early exit once > snap.
    bool conflicts(const uint8_t* b, int bl, const uint8_t* e, int el, int64_t snap) {
        Node* preds[kLevels];
        int c = cmpBytes(b, bl, e, el);
        if (c == 0) {
            descend(b, bl, false, preds);
            return preds[0]->maxv()[0] > snap;
        }
        descend(b, bl, true, preds);
        Node* y = preds[0];
        if (y->maxv()[0] > snap) return true;
        y = y->nexts()[0];
        while (y && cmpBytes(y->key(), y->len, e, el) < 0) {
            int l = y->height - 1;
            while (l > 0) {
                Node* n = y->nexts()[l];
                if (n && cmpBytes(n->key(), n->len, e, el) <= 0) break;
                l--;
            }
            // the level-l span of y lies inside (b, e): its max is exact (or, after GC,
            // high by versions below oldestVersion, which no admitted snapshot sees).
            if (y->maxv()[l] > snap) return true;
            y = y->nexts()[l];
        }
        return false;
    }

    void insertAfter(Node** preds, const uint8_t* k, int len, int64_t v, Node** outNode) {
        int h = pickHeight();
        Node* n = make(k, len, h);
        for (int l = 0; l < h; l++) {
            n->nexts()[l] = preds[l]->nexts()[l];
            preds[l]->nexts()[l] = n;
        }
        n->maxv()[0] = v;
        for (int l = 1; l < h; l++) { recompute(preds[l], l); recompute(n, l); }
        count++;
        if (outNode) *outNode = n;
    }

    // History := now on [b, e).
    void assign(const uint8_t* b, int bl, const uint8_t* e, int el, int64_t now) {
        Node* pe[kLevels];
        descend(e, el, false, pe);
        Node* at = pe[0]->nexts()[0];
        if (!(at && cmpBytes(at->key(), at->len, e, el) == 0)) {
            int64_t inherited = pe[0]->maxv()[0];
            Node* en;
            insertAfter(pe, e, el, inherited, &en);
            // levels above the end node's height: their span max is unchanged (duplicate version).
        }
        Node* pb[kLevels];
        descend(b, bl, false, pb);
        // unlink every node with key in [b, e)
        Node* x = pb[0]->nexts()[0];
        while (x && cmpBytes(x->key(), x->len, e, el) < 0) {
            Node* nx = x->nexts()[0];
            for (int l = 0; l < x->height; l++)
                if (pb[l]->nexts()[l] == x) pb[l]->nexts()[l] = x->nexts()[l];
            drop(x);
            count--;
            x = nx;
        }
        Node* bn;
        int h = pickHeight();
        bn = make(b, bl, h);
        for (int l = 0; l < h; l++) { bn->nexts()[l] = pb[l]->nexts()[l]; pb[l]->nexts()[l] = bn; }
        bn->maxv()[0] = now;
        count++;
        for (int l = 1; l < kLevels; l++) {
            recompute(pb[l], l);
            if (l < h) recompute(bn, l);
        }
    }

    // removeBefore over the whole list (SkipList.cpp:542-571).
    void removeBefore(int64_t v) {
        Node* preds[kLevels];
        for (int l = 0; l < kLevels; l++) preds[l] = head;
        bool wasAbove = true;
        Node* x = head->nexts()[0];
        while (x) {
            Node* nx = x->nexts()[0];
            bool isAbove = x->maxv()[0] >= v;
            if (isAbove || wasAbove) {
                for (int l = 0; l < x->height; l++) preds[l] = x;
            } else {
                for (int l = 0; l < x->height; l++) {
                    preds[l]->nexts()[l] = x->nexts()[l];
                    if (l) preds[l]->maxv()[l] = std::max(preds[l]->maxv()[l], x->maxv()[l]);
                }
                drop(x);
                count--;
            }
            wasAbove = isAbove;
            x = nx;
        }
    }
};

struct Pt {
    const uint8_t* key;
    int32_t len;
    uint8_t cls;  // read-end 0 < write-end 1 < write-begin 2 < read-begin 3 (SkipList.cpp:89-91)
    int32_t txn;
    int32_t* slot;
};

}  // namespace

extern "C" {

void* slb_new(void) {
    SkipSet* s = new SkipSet();
    s->reset(0);
    return s;
}
void slb_destroy(void* p) {
    SkipSet* s = (SkipSet*)p;
    s->reset(0);
    s->drop(s->head);
    s->head = nullptr;
    delete s;
}
void slb_clear(void* p, int64_t v) { ((SkipSet*)p)->reset(v); }
void slb_set_oldest(void* p, int64_t v) {
    SkipSet* s = (SkipSet*)p;
    if (v > s->oldest) s->oldest = v;
}
int64_t slb_oldest(void* p) { return ((SkipSet*)p)->oldest; }
int64_t slb_history_size(void* p) { return ((SkipSet*)p)->count; }

void slb_load_history(void* p, int64_t n, const uint8_t* bytes, const int64_t* offs, const int64_t* vers,
                      int64_t header) {
    SkipSet* s = (SkipSet*)p;
    s->reset(header);
    // boundaries arrive sorted: append at the tail of every level, then fix maxima bottom-up.
    Node* tails[kLevels];
    for (int l = 0; l < kLevels; l++) tails[l] = s->head;
    for (int64_t i = 0; i < n; i++) {
        int h = s->pickHeight();
        Node* x = s->make(bytes + offs[i], (int)(offs[i + 1] - offs[i]), h);
        x->maxv()[0] = vers[i];
        for (int l = 0; l < h; l++) { x->nexts()[l] = nullptr; tails[l]->nexts()[l] = x; tails[l] = x; }
        s->count++;
    }
    for (int l = 1; l < kLevels; l++)
        for (Node* x = s->head; x; x = x->nexts()[l]) SkipSet::recompute(x, l);
}

int64_t slb_detect(void* p, const fdbcs_packed_batch* pb, int64_t now, int64_t newOldest, uint8_t* verdicts,
                   int32_t* conf_off, int32_t* conf_idx, int64_t cap, int gc) {
    SkipSet* s = (SkipSet*)p;
    const int T = pb->n_txn;
    const int R = pb->read_offsets[T];
    auto K = [&](int64_t k) { return pb->key_bytes + pb->key_offsets[k]; };
    auto KL = [&](int64_t k) { return (int)(pb->key_offsets[k + 1] - pb->key_offsets[k]); };

    std::vector<uint8_t> tooOld(T, 0), status(T, 0), report(T, 0);
    std::vector<int32_t> rIdx, wIdx;  // point index pairs per range
    rIdx.assign((size_t)2 * R, 0);
    wIdx.assign((size_t)2 * pb->write_offsets[T], 0);
    std::vector<Pt> pts;
    pts.reserve((size_t)2 * (R + pb->write_offsets[T]));
    std::vector<std::vector<int>> confl(T);
    for (int t = 0; t < T; t++) {
        int r0 = pb->read_offsets[t], r1 = pb->read_offsets[t + 1];
        int w0 = pb->write_offsets[t], w1 = pb->write_offsets[t + 1];
        report[t] = pb->report_conflicting_keys ? pb->report_conflicting_keys[t] : 0;
        if (pb->read_snapshot[t] < s->oldest && r1 > r0) { tooOld[t] = 1; continue; }  // SkipList.cpp:770
        for (int r = r0; r < r1; r++) {
            pts.push_back({K(2 * r), KL(2 * r), 3, t, &rIdx[2 * r]});
            pts.push_back({K(2 * r + 1), KL(2 * r + 1), 0, t, &rIdx[2 * r + 1]});
        }
        for (int w = w0; w < w1; w++) {
            int64_t kb = 2 * (int64_t)(R + w);
            pts.push_back({K(kb), KL(kb), 2, t, &wIdx[2 * w]});
            pts.push_back({K(kb + 1), KL(kb + 1), 1, t, &wIdx[2 * w + 1]});
        }
    }
    std::sort(pts.begin(), pts.end(), [](const Pt& a, const Pt& b) {
        int c = cmpBytes(a.key, a.len, b.key, b.len);
        return c ? c < 0 : a.cls < b.cls;
    });

    // history check
    for (int t = 0; t < T; t++) {
        if (tooOld[t]) continue;
        for (int r = pb->read_offsets[t]; r < pb->read_offsets[t + 1]; r++) {
            if (s->conflicts(K(2 * r), KL(2 * r), K(2 * r + 1), KL(2 * r + 1), pb->read_snapshot[t])) {
                status[t] = 1;
                if (report[t]) confl[t].push_back(r - pb->read_offsets[t]);
            }
        }
    }

    // intra-batch, word-parallel MiniConflictSet
    for (size_t i = 0; i < pts.size(); i++) *pts[i].slot = (int32_t)i;
    std::vector<uint64_t> bits((pts.size() + 64) / 64, 0);
    auto anySet = [&](int a, int b) {
        while (a < b && (a & 63)) { if (bits[a >> 6] >> (a & 63) & 1) return true; a++; }
        while (a + 64 <= b) { if (bits[a >> 6]) return true; a += 64; }
        while (a < b) { if (bits[a >> 6] >> (a & 63) & 1) return true; a++; }
        return false;
    };
    auto setRange = [&](int a, int b) {
        while (a < b && (a & 63)) { bits[a >> 6] |= 1ull << (a & 63); a++; }
        while (a + 64 <= b) { bits[a >> 6] = ~0ull; a += 64; }
        while (a < b) { bits[a >> 6] |= 1ull << (a & 63); a++; }
    };
    for (int t = 0; t < T; t++) {
        if (status[t]) continue;
        bool c = tooOld[t];
        for (int r = pb->read_offsets[t]; r < pb->read_offsets[t + 1] && !c; r++) {
            if (anySet(rIdx[2 * r], rIdx[2 * r + 1])) {
                c = true;
                if (report[t]) confl[t].push_back(r - pb->read_offsets[t]);
            }
        }
        status[t] = c;
        if (!c)
            for (int w = pb->write_offsets[t]; w < pb->write_offsets[t + 1]; w++) setRange(wIdx[2 * w], wIdx[2 * w + 1]);
    }

    // combine committed writes (sweep over sorted endpoints)
    std::vector<std::pair<const Pt*, const Pt*>> comb;
    int active = 0;
    for (const Pt& q : pts) {
        if (!(q.cls == 1 || q.cls == 2) || status[q.txn]) continue;
        if (q.cls == 2) {
            if (++active == 1) comb.push_back({&q, nullptr});
        } else if (--active == 0) comb.back().second = &q;
    }
    for (size_t i = comb.size(); i-- > 0;)
        s->assign(comb[i].first->key, comb[i].first->len, comb[i].second->key, comb[i].second->len, now);

    for (int t = 0; t < T; t++)
        verdicts[t] = tooOld[t] ? FDBCS_TRANSACTION_TOO_OLD
                                : (status[t] ? FDBCS_TRANSACTION_CONFLICT : FDBCS_TRANSACTION_COMMITTED);

    if (newOldest > s->oldest) {
        s->oldest = newOldest;
        if (gc) s->removeBefore(newOldest);
    }
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
