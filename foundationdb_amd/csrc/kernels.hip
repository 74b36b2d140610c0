// kernels.hip — gfx950 (CDNA4) kernels of the MVCC conflict-resolution engine.
//
// The reference resolves a batch on one CPU thread with a versioned skip list
// (fdbserver/SkipList.cpp:844-890).  Here the history is a sorted boundary array
// in HBM (structure of arrays, a base and a delta tier) with a 64-ary range-max
// hierarchy, and every phase of ConflictBatch::detectConflicts is a data-parallel
// kernel.  Per batch, three chains on three streams (engine.cpp):
//
//   stage A   D.Sort             k_sort_partition, k_sort_bucket (cold start: k_sample, k_quant_cold)
//             D.CheckIntraBatch  k_scan<EdgePairScan>, k_edge_fill: candidate edges (one per write group)
//   stage B X D.CheckRead        k_check_lanes (both tiers and the previous batch's union segments)
//                                or k_check_lanes_tier<base / delta> (split check; other workgroups
//                                of the delta-tier launch search the segments)
//             D.CheckIntraBatch  k_resolve_pre (statuses, or the pre-pass), k_resolve (batch-order rounds)
//             D.Combine          in k_resolve_pre without candidate edges, else k_combine
//   stage B Y D.MergeWrite       k_seg_prep, k_merge_copy<BatchIns>; compaction: k_compact_search,
//                                k_scan<CompactSumScan>, k_merge_copy<CompactIns>
//             D.RemoveBefore     k_scan<GcScan> (with a compaction); k_epilogue: levels, index, scalars
//   routing   (multi-resolver)   k_route_mark, k_scan<RouteScan>, k_route_write
//
// Memory-bound integer/byte work: no MFMA anywhere (BASELINE.json north_star).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include <limits.h>

#include "engine.h"
#include "lane_xor.h"

namespace fdbcs {

thread_local LaunchList* t_record = nullptr;
thread_local uint8_t t_group = 0;
thread_local hipError_t t_launch_error = hipSuccess;

// ------------------------------------------------------------------ helpers

// History tails are 8-byte aligned and Hist::lt.y counts 8-byte units (32 GiB of tail arena per
// conflict set with a 32-bit offset).
__device__ __forceinline__ const uint8_t* hist_tail(const uint8_t* htail, uint32_t unit) {
    return htail + 8 * (size_t)unit;
}
__device__ __forceinline__ uint32_t tail_units(uint32_t len) { return len > 16u ? (len - 16u + 7u) / 8u : 0u; }

// Copy the n tail bytes at src (any alignment; the arena has >= 16 bytes of slack past them) to the
// 8-aligned dst as whole words; the bytes past n in the last word are never compared (tail_cmp).
__device__ __forceinline__ void copy_tail_words(uint8_t* dst, const uint8_t* src, uint32_t n) {
    const uintptr_t a = (uintptr_t)src;
    const uint64_t* w = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    uint64_t* d = (uint64_t*)dst;
    for (uint32_t i = 0; i < (n + 7u) / 8u; i++) d[i] = sh ? (w[i] >> sh) | (w[i + 1] << (64u - sh)) : w[i];
}

__device__ __forceinline__ int hist_cmp(const Hist& h, int64_t i, const uint8_t* htail, const DKey& q,
                                        const uint8_t* qtail) {
    ulonglong2 k = h.key[i];
    if (k.x != q.hi) return k.x < q.hi ? -1 : 1;
    if (k.y != q.lo) return k.y < q.lo ? -1 : 1;
    uint2 lt = h.lt[i];
    if (lt.x > 16u && q.len > 16u) return tail_cmp(hist_tail(htail, lt.y), lt.x, qtail + q.tail, q.len);
    return (lt.x > q.len) - (lt.x < q.len);
}

__device__ __forceinline__ bool prefix_less(const ulonglong2& k, const DKey& q) {
    return k.x < q.hi || (k.x == q.hi && k.y < q.lo);
}

// Full key comparison of boundary i with q, given its prefix already loaded.
__device__ __forceinline__ int probe_cmp(const Hist& h, int64_t i, const ulonglong2& k, const uint8_t* htail,
                                         const DKey& q, const uint8_t* qtail) {
    if (k.x != q.hi) return k.x < q.hi ? -1 : 1;
    if (k.y != q.lo) return k.y < q.lo ? -1 : 1;
    return hist_cmp(h, i, htail, q, qtail);  // equal prefixes: length / tail
}
// The same with a word-at-a-time tail comparison (one pair of 8-byte words live, not four): keeps
// the read check's register footprint low; equal 16-byte prefixes are the rare path.
__device__ __forceinline__ int probe_cmp_lean(const Hist& h, int64_t i, const ulonglong2& k, const uint8_t* htail,
                                              const DKey& q, const uint8_t* qtail) {
    if (k.x != q.hi) return k.x < q.hi ? -1 : 1;
    if (k.y != q.lo) return k.y < q.lo ? -1 : 1;
    const uint2 lt = h.lt[i];
#if defined(__HIP_DEVICE_COMPILE__)
    if (lt.x > 16u && q.len > 16u) {
        const uint8_t* ta = hist_tail(htail, lt.y);
        const uint8_t* tb = qtail + q.tail;
        const uint32_t nb = (lt.x < q.len ? lt.x : q.len) - 16u;
        for (uint32_t o = 0; o < nb; o += 8) {
            const int vb = (int)(nb - o);
            const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
            const uint64_t x = tail_word(ta + o) & msk, y = tail_word(tb + o) & msk;
            if (x != y) return x < y ? -1 : 1;
        }
    }
#endif
    return (lt.x > q.len) - (lt.x < q.len);
}

// ---- long-key probes (batches with keys over 16 bytes: C4 tuple keys)
//
// Keys of one tuple subspace/user share their 16-byte prefix, so the last rounds of a lookup tie
// on the prefix and compare tails.  The generic probe loads the boundary's (len, tail) only after
// its prefix tied, then the two tails 32 bytes per dependent round, each tail word through two
// unaligned loads.  The long-key probe instead holds the query's tail words in registers for the
// whole lookup (kQW words), loads the boundary's (len, tail) beside its prefix, and reads the
// history tail (8-byte aligned in its arena) as whole words, kHW per round: one dependent round
// after the prefix for tails up to 48 bytes, two up to 96.
constexpr int kQW = 12;  // query tail words in registers: keys up to 112 bytes compare without reloads
[[maybe_unused]] constexpr int kHW = 6;  // history tail words per load round
struct QTail {
    uint64_t w[kQW];  // big-endian words of query bytes [16, 16 + 8 kQW), garbage past the key's end
};

__device__ __forceinline__ void load_qtail(QTail& qt, const DKey& q, const uint8_t* qtail) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t n = q.len > 16u ? q.len - 16u : 0u;
    const uintptr_t a = (uintptr_t)(qtail + q.tail);
    const uint64_t* w = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint32_t cnt = ((uint32_t)(a & 7u) + n + 7u) / 8u;  // aligned words holding the tail
    uint64_t raw[kQW + 1];
#pragma unroll
    for (int j = 0; j <= kQW; j++) raw[j] = (uint32_t)j < cnt ? w[j] : 0ull;
#pragma unroll
    for (int j = 0; j < kQW; j++) qt.w[j] = __builtin_bswap64(sh ? (raw[j] >> sh) | (raw[j + 1] << (64u - sh)) : raw[j]);
#endif
}

// probe_cmp with the boundary's (len, tail) already loaded and the query tail in registers.
__device__ __forceinline__ int probe_cmp_long(const ulonglong2& k, const uint2& lt, const uint8_t* htail, const DKey& q,
                                              const QTail& qt, const uint8_t* qtail) {
    if (k.x != q.hi) return k.x < q.hi ? -1 : 1;
    if (k.y != q.lo) return k.y < q.lo ? -1 : 1;
#if defined(__HIP_DEVICE_COMPILE__)
    if (lt.x > 16u && q.len > 16u) {
        const uint64_t* ha = (const uint64_t*)hist_tail(htail, lt.y);
        const uint32_t n = (lt.x < q.len ? lt.x : q.len) - 16u;  // common tail bytes
        const int nw = (int)((n + 7u) / 8u);
#pragma unroll
        for (int j0 = 0; j0 < kQW; j0 += kHW) {
            if (j0 >= nw) break;
            uint64_t x[kHW];
#pragma unroll
            for (int u = 0; u < kHW; u++) x[u] = j0 + u < nw ? ha[j0 + u] : 0ull;
#pragma unroll
            for (int u = 0; u < kHW; u++) {
                const int j = j0 + u;
                const int vb = (int)n - 8 * j;  // bytes of word j inside the shorter tail
                if (vb <= 0) break;
                const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
                const uint64_t hx = __builtin_bswap64(x[u]) & msk, qy = qt.w[j] & msk;
                if (hx != qy) return hx < qy ? -1 : 1;
            }
        }
        if (nw > kQW)  // both tails run past the registers: the rest from memory
            return tail_cmp(hist_tail(htail, lt.y) + 8 * kQW, lt.x - 8 * kQW, qtail + q.tail + 8 * kQW,
                            q.len - 8 * kQW);
    }
#endif
    return (lt.x > q.len) - (lt.x < q.len);
}

// ---- cooperative search: kArity lanes per query, one kArity-entry tree node per level
//
// Each lane of an aligned kArity-lane group loads one entry of the node, so a level is one
// coalesced kArity*16-byte access (one 128-byte line at kArity 8).  All lanes of a group call with
// the same query and get the same result.  gmask(): the group's bits of a wave ballot.
__device__ __forceinline__ uint32_t gmask(bool pred) {
    const uint64_t m = __ballot(pred);
    return (uint32_t)(m >> (threadIdx.x & 63 & ~(kArity - 1))) & ((1u << kArity) - 1u);
}

// Directory slot of a 16-byte prefix (MaxLevels::dir_p .. dir_w), monotone over all keys: keys
// below the loaded keys' common prefix take slot 0, keys above it dir_top, keys under it 1 + the
// mixed-radix code of the next dir_e bytes (each byte's offset in its position's value range; the
// code ends at the first byte outside its range).  ALU only.  Both tiers' directories
// (k_directory, the epilogue's delta fill) and every lookup use it.
__device__ __forceinline__ uint32_t dir_slot(const MaxLevels& m, uint64_t hi, uint64_t lo) {
    const uint32_t p = m.dir_p;
    if (p) {
        const uint64_t mh = p >= 8 ? ~0ull : ~0ull << (64 - 8 * p);
        const uint64_t ml = p <= 8 ? 0ull : ~0ull << (128 - 8 * p);
        const uint64_t xh = hi & mh, xl = lo & ml;
        if (xh != m.dir_phi || xl != m.dir_plo)
            return (xh < m.dir_phi || (xh == m.dir_phi && xl < m.dir_plo)) ? 0u : m.dir_top;
    }
    // the bytes after the prefix, left-aligned: position p + i is byte i of h
    const uint64_t h = p == 0 ? hi : (p < 8 ? (hi << (8 * p)) | (lo >> (64 - 8 * p)) : lo << (8 * (p - 8)));
    uint32_t code = 1;
    bool live = true;
#pragma unroll
    for (int i = 0; i < kDirPos; i++) {
        const uint32_t b = (uint32_t)(h >> (56 - 8 * i)) & 255u;
        const uint32_t pos = m.dir_pos[i];
        const uint32_t l = pos & 255u, d = (pos >> 8) & 511u, s = pos >> 17;
        const uint32_t r = b < l ? 0u : (b - l < d ? b - l : d);
        if (live && (uint32_t)i < m.dir_e) code += (r >> s) * m.dir_w[i];
        live = live && b >= l && b - l < d;
    }
    return code;
}

// The directory range of q's slot, in skey8 entries (every 8th boundary): entries [d8a, d8b) share
// q's slot, every entry before d8a lies below q and every entry from d8b on above it (dir_slot is
// monotone over the 16-byte prefix).  Both tiers' directories count skey8 entries (base:
// k_directory, exact; delta: the epilogue's fill, entries of the current epoch only).  false: no
// directory, or a delta slot of another epoch.
__device__ __forceinline__ bool dir_range8(const MaxLevels& m, const DKey& q, int64_t& d8a, int64_t& d8b) {
    if (!m.dir && !m.edir_epoch) return false;
    const uint32_t dv = dir_slot(m, q.hi, q.lo);
    if (m.dir) {
        d8a = m.dir[dv];
        d8b = m.dir[dv + 1];
        return true;
    }
    const uint64_t x0 = m.edir[dv], x1 = m.edir[dv + 1];
    d8a = (uint32_t)x0;
    d8b = (uint32_t)x1;
    return (uint32_t)(x0 >> 32) == m.edir_epoch && (uint32_t)(x1 >> 32) == m.edir_epoch;
}

// LONG: the long-key probes above (the batch has keys over 16 bytes); same result.
template <bool LONG = false>
__device__ __forceinline__ int64_t group_lower_bound(const Hist& h, const MaxLevels& m, int64_t n, const DKey& q,
                                                     const uint8_t* htail, const uint8_t* qtail, bool& eq) {
    const int gl = threadIdx.x & (kArity - 1);
    const int g0 = threadIdx.x & 63 & ~(kArity - 1);  // first lane of the group
    eq = false;
    if (n <= 0) return 0;
    QTail qt;
    if constexpr (LONG) load_qtail(qt, q, qtail);  // in flight during the descent
    // one probe of boundary p (prefix k): the long-key form loads (len, tail) beside the prefix
    auto probe = [&](int64_t p, const ulonglong2* kp) -> int {
        if constexpr (LONG) {
            const ulonglong2 k = *kp;
            const uint2 lt = h.lt[p];
            return probe_cmp_long(k, lt, htail, q, qt, qtail);
        } else {
            return probe_cmp(h, p, *kp, htail, q, qtail);
        }
    };
    int64_t sz[kIdxLevels];
    sz[0] = (n + kFan - 1) / kFan;
#pragma unroll
    for (int L = 1; L < kIdxLevels; L++) sz[L] = (sz[L - 1] + kArity - 1) / kArity;
    int top = 0;
    while (top + 1 < kIdxLevels && sz[top] > kArity) top++;
    // c = number of entries of level `top` whose prefix is < q.  When level 0 is probed, also learn
    // whether the first sample not below q shares q's prefix (`bknown`: it does not).
    auto prefix_eq = [&](const ulonglong2& k) { return k.x == q.hi && k.y == q.lo; };
    int64_t c = 0;
    bool bknown = false;
    // the top level's first group is loaded beside the directory slot (no added round trip when
    // the slot is crowded and the tree is taken)
    const bool v_top = gl < sz[top];
    const ulonglong2 e_top = m.skey[top][v_top ? gl : 0];
    bool direct = false;
    int64_t d8a, d8b;
    if (dir_range8(m, q, d8a, d8b)) {
        // radix directory: the level-0 samples (every 8th skey8 entry) sharing q's directory bits
        // are [d0, d1); a slot of at most two groups is counted directly at level 0
        const int64_t d0 = (d8a + 7) >> 3, d1 = (d8b + 7) >> 3;
        if (d1 - d0 <= 2 * kArity && d1 <= sz[0]) {
            direct = true;
            c = d0;
            bknown = true;  // all of the slot below q: the next sample's first two bytes are greater
            for (int64_t j0 = d0; j0 < d1; j0 += kArity) {
                const bool v = j0 + gl < d1;
                const ulonglong2 e = m.skey[0][v ? j0 + gl : 0];
                const int k = __popc(gmask(v && prefix_less(e, q)));
                c += k;
                if (k < __popc(gmask(v))) {
                    bknown = !((gmask(v && prefix_eq(e)) >> k) & 1u);
                    break;
                }
            }
        }
    }
    if (!direct) {
        for (int64_t j0 = 0; j0 < sz[top]; j0 += kArity) {
            const bool v = j0 == 0 ? v_top : j0 + gl < sz[top];
            const ulonglong2 e = j0 == 0 ? e_top : m.skey[top][v ? j0 + gl : 0];
            const int k = __popc(gmask(v && prefix_less(e, q)));
            if (top == 0 && k < __popc(gmask(v))) bknown = !((gmask(v && prefix_eq(e)) >> k) & 1u);
            c += k;
            if (k < kArity) break;
        }
        for (int L = top; L > 0; L--) {
            if (c == 0) continue;  // nothing below q at this level: nothing below it underneath either
            // entries of level L-1 below q: [0, c') with c' in [A(c-1)+1, Ac]
            const int64_t base = (int64_t)kArity * (c - 1) + 1;
            const int64_t end = min((int64_t)kArity * c, sz[L - 1]);
            const bool v = base + gl < end;
            const ulonglong2 e = m.skey[L - 1][v ? base + gl : 0];
            const int k = __popc(gmask(v && prefix_less(e, q)));
            if (L == 1 && k < __popc(gmask(v))) bknown = !((gmask(v && prefix_eq(e)) >> k) & 1u);
            c = base + k;
        }
    }
    // c = #samples below q; samples equal to q's prefix (shared prefixes) widen the block
    int64_t b = c;
    for (; !bknown;) {
        const bool v = b + gl < sz[0];
        const ulonglong2 k = m.skey[0][v ? b + gl : 0];
        const uint32_t same = gmask(v && k.x == q.hi && k.y == q.lo);
        const int run = __ffs(~same) - 1;  // leading lanes equal to q's prefix
        b += run;
        if (run < kArity) break;
    }
    int64_t lo = c > 0 ? kFan * (c - 1) + 1 : 0;
    const int64_t hi = min(n, kFan * b);
    if (b == c && m.skey8) {
        // Boundary 64(c-1) < q < boundary 64c (sample c's prefix is greater): the answer lies in one
        // 64-boundary block.  Round one probes the starts of its eight 8-groups through skey8 (one
        // 128-byte line, not eight); round two the seven keys after the last start below q (one
        // line).  Prefix ties compare lengths / tails against the boundary itself (probe_cmp).
        const int64_t B = c > 0 ? kFan * (c - 1) : 0;
        const int64_t p8 = B + 8 * gl;
        const bool v8 = p8 < hi;
        int r8 = 1;
        if (v8) r8 = probe(p8, &m.skey8[p8 / 8]);
        const int k8 = __popc(gmask(v8 && r8 < 0));  // group starts below q
        const int r_first = __shfl(r8, g0, 64);
        if (k8 == 0) {  // c == 0 and q <= boundary 0
            eq = hi > 0 && r_first == 0;
            return 0;
        }
        const int64_t g = B + 8 * (k8 - 1);  // boundary g < q; the answer is in (g, min(g + 8, hi)]
        const int64_t gend = min(g + 8, hi);
        const int64_t pk = g + 1 + gl;
        const bool vk = gl < 7 && pk < gend;
        int rk = 1;
        if (vk) rk = probe(pk, &h.key[pk]);
        const int k1 = __popc(gmask(vk && rk < 0));
        const int64_t lb = g + 1 + k1;
        const int r_stop = __shfl(rk, g0 + (k1 < 7 ? k1 : 6), 64);
        const int r_next = __shfl(r8, g0 + (k8 < kArity ? k8 : kArity - 1), 64);
        if (lb < gend)
            eq = r_stop == 0;  // the probe that stopped the count
        else if (lb < hi)
            eq = r_next == 0;  // lb = g + 8: the next group's start, probed in round one
        return lb;
    }
    // lower_bound in [lo, lo + span]: rounds of kArity probes at a shrinking stride.  span <= 64
    // normally; a long run of boundaries sharing q's 16-byte prefix (tuple keys) only starts the
    // stride higher, so the lanes still compare tails side by side.
    int64_t span = hi - lo;
    int64_t stride0 = kFan / kArity;
    while (stride0 * kArity < span) stride0 *= kArity;
    bool eq_cand = false;  // cmp == 0 at the last probe that stopped a count (the answer, if < hi)
    for (int64_t stride = stride0; span > 0; stride = stride > kArity ? stride / kArity : 1) {
        const int64_t p = lo + stride * (gl + 1) - 1;
        const bool v = stride * (gl + 1) <= span && p < hi;
        int r = 1;
        if (v) r = probe(p, &h.key[p]);
        const uint32_t valid = gmask(v);
        const int cnt = __popc(gmask(v && r < 0));
        const int stop = __shfl(r, g0 + (cnt < kArity ? cnt : kArity - 1), 64);
        if (cnt < __popc(valid)) eq_cand = stop == 0;  // lane cnt probed a key >= q
        lo += stride * cnt;
        span = cnt < __popc(valid) ? stride - 1 : span - stride * cnt;
        if (stride == 1) break;
    }
    if (lo < hi) eq = eq_cand;
    return lo;
}

// Entry i of the top level (the max over its kL3Rep replicas).
__device__ __forceinline__ int64_t l3_at(const int64_t* a, int64_t i) {
    int64_t v[kL3Rep];
#pragma unroll
    for (int r = 0; r < kL3Rep; r++) v[r] = a[(i * kL3Rep + r) * kL3Pad];
    int64_t best = v[0];
#pragma unroll
    for (int r = 1; r < kL3Rep; r++) best = v[r] > best ? v[r] : best;
    return best;
}

// Max of lvl[0][lo, hi) through the 64-ary hierarchy; stops early once above `snap`.
__device__ __forceinline__ int64_t range_max(const MaxLevels& m, int64_t lo, int64_t hi, int64_t snap) {
    int64_t best = LLONG_MIN;
    for (int L = 0; L < kMaxLevels; L++) {
        const int64_t* a = m.lvl[L];
        if (hi - lo <= 2 * kFan || L == kMaxLevels - 1) {
            for (int64_t i = lo; i < hi; i++) {
                int64_t v = L == kMaxLevels - 1 ? l3_at(a, i) : a[i];
                best = v > best ? v : best;
                if (best > snap) return best;
            }
            return best;
        }
        int64_t lo2 = (lo + kFan - 1) / kFan, hi2 = hi / kFan;
        for (int64_t i = lo; i < lo2 * kFan; i++) {
            int64_t v = a[i];
            best = v > best ? v : best;
        }
        for (int64_t i = hi2 * kFan; i < hi; i++) {
            int64_t v = a[i];
            best = v > best ? v : best;
        }
        if (best > snap) return best;
        lo = lo2;
        hi = hi2;
    }
    return best;
}

// Exclusive block-wide sum over all threads of the block (blockDim multiple of 64).
template <typename T>
__device__ __forceinline__ T block_excl_sum(T v, T* sh, T* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        T s = lane < nw ? sh[lane] : T(0);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            T y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < nw) sh[lane] = s;
    }
    __syncthreads();
    T before = wid ? sh[wid - 1] : T(0);
    *total = sh[nw - 1];
    __syncthreads();
    return before + x - v;
}

// Single-workgroup exclusive scan of n elements given by load(i); store(i, prefix).
// Returns the total.  Each thread owns 4 consecutive elements per 4*blockDim chunk.
template <typename T, typename Load, typename Store>
__device__ T wg_scan(int64_t n, Load load, Store store, T* sh) {
    T carry = 0;
    const int64_t chunk = 4 * (int64_t)blockDim.x;
    for (int64_t base = 0; base < n; base += chunk) {
        int64_t i0 = base + 4 * (int64_t)threadIdx.x;
        T v[4];
        T s = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = (i0 + k < n) ? load(i0 + k) : T(0);
            s += v[k];
        }
        T tot;
        T run = carry + block_excl_sum<T>(s, sh, &tot);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (i0 + k < n) store(i0 + k, run);
            run += v[k];
        }
        carry += tot;
    }
    return carry;
}

// ------------------------------------------------------------------ D.CheckRead

// Does some segment of one tier meeting the read [kb, ke) hold a version > snap?  lb / lb_eq locate
// kb, j = lower_bound(ke).  Degenerate [b, b) reads look at the greatest boundary < b (fingers
// never diverge, SkipList.cpp:650-666).
__device__ __forceinline__ bool tier_conflict(const Hist& h, const MaxLevels& m, int64_t hdr, int64_t lb, bool lb_eq,
                                              int64_t j, bool degenerate, int64_t snap) {
    if (degenerate) return (lb > 0 ? h.ver[lb - 1] : hdr) > snap;
    const int64_t ub = lb + (lb_eq ? 1 : 0);
    // segments [ub-1, j): the one containing b (header if ub == 0) and boundaries in (b, e)
    if (ub == 0) return hdr > snap || range_max(m, 0, j, snap) > snap;
    return range_max(m, ub - 1, j, snap) > snap;
}

// ---- per-lane lookups (SkipList.cpp:426-458 + CheckMax :619-706, as the step-function rule of
// SURVEY A.2)
//
// The history is the base tier overlaid by the delta tier; every delta version is >= the base
// versions it covers (versions only grow), so the max over the overlay equals the max of the two
// tiers' maxima, and holes (kHole) never conflict.
//
// One lane per lookup.  Round 3's cooperative lookups (group_lower_bound, still used by the
// segment search of small batches) gave each lookup kArity lanes that load one node entry each,
// so a wave served kArity lookups and the wave's instruction stream (ballots, shuffles, 64-bit
// compares) was paid per kArity lookups: at C2 12,500 waves of ~350 VALU + ~260 SALU instructions
// each, 77 % of their life waiting on loads (rocprofv3 SQ counters), the chip never holding all
// of them at once.  Here a lane issues a whole node's (or directory slot's)
// entries itself, up to kLaneProbe independent 16-byte loads in flight, and counts them in
// registers: the same dependent rounds per lookup, 64 lookups per wave, every wave of a C2 batch
// resident at once.
constexpr int kLaneProbe = 16;  // entries one lane loads per round (a directory slot of two groups)

// Number of the first cnt (<= N) entries of a[base, ...) whose 16-byte prefix is below q's, and
// whether the first entry not below it has q's prefix (eq_next; false if all are below).
template <int N>
__device__ __forceinline__ int lane_count(const ulonglong2* a, int64_t base, int cnt, const DKey& q, bool& eq_next) {
    ulonglong2 k[N];
#pragma unroll
    for (int i = 0; i < N; i++)
        if (i < cnt) k[i] = a[base + i];
    int c = 0;
    eq_next = false;
    bool stop = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (i < cnt && !stop) {
            if (prefix_less(k[i], q)) {
                c++;
            } else {
                stop = true;
                eq_next = k[i].x == q.hi && k[i].y == q.lo;
            }
        }
    }
    return c;
}

// The level-0 samples of a tier below q's 16-byte prefix (c) and the end of the run of samples
// sharing that prefix (b >= c), by one lane: the radix directory slot (at most kLaneProbe level-0
// samples) or the kArity-ary sample tree, each node's entries loaded by the lane as independent
// 16-byte loads.  Boundary 64(c-1) lies below q and boundary 64b (if any) above it.
__device__ __forceinline__ void lane_sample_range(const MaxLevels& m, int64_t n, const DKey& q, int64_t& c_out,
                                                  int64_t& b_out) {
    int64_t sz[kIdxLevels];
    sz[0] = (n + kFan - 1) / kFan;
#pragma unroll
    for (int L = 1; L < kIdxLevels; L++) sz[L] = (sz[L - 1] + kArity - 1) / kArity;
    int top = 0;
    while (top + 1 < kIdxLevels && sz[top] > kArity) top++;
    int64_t c = 0;      // level-0 samples whose prefix is below q
    bool bknown = false;  // the sample at c (if any) is known not to share q's prefix
    bool direct = false;
    int64_t w0 = -1, w1 = -1;  // a directory slot too wide to count at level 0
    int64_t d8a, d8b;
    if (dir_range8(m, q, d8a, d8b)) {
        // the level-0 samples (every 8th skey8 entry) in q's slot: [d0, d1)
        const int64_t d0 = (d8a + 7) >> 3, d1 = (d8b + 7) >> 3;
        if (d1 - d0 <= kLaneProbe && d1 <= sz[0]) {
            direct = true;
            bool eqn;
            const int cnt = (int)(d1 - d0);
            const int k = lane_count<kLaneProbe>(m.skey[0], d0, cnt, q, eqn);
            c = d0 + k;
            // all of the slot below q: the next sample's first two bytes are greater
            bknown = k < cnt ? !eqn : true;
        } else if (d1 <= sz[0]) {
            w0 = d0;
            w1 = d1;
        }
    }
    if (!direct) {
        // A wide slot (keys whose directory bits take few values: C4's decimal digits after the
        // shared prefix) still bounds q: samples before w0 lie below it and from w1 on above it, so
        // the descent starts at the lowest level whose entries over [w0, w1) fit one probe round
        // (entry j of level L is sample j A^L) instead of at the top.
        int lv = top;
        bool started = false;
        if (w0 >= 0) {
            int64_t span = 1;
            for (int L = 1; L < top; L++) {
                span *= kArity;
                const int64_t a = w0 / span, z = (w1 - 1) / span;
                if (z - a + 1 <= kLaneProbe) {
                    bool eqn;
                    c = a + lane_count<kLaneProbe>(m.skey[L], a, (int)(z - a + 1), q, eqn);
                    lv = L;
                    started = true;
                    break;
                }
            }
        }
        for (int64_t j0 = 0; !started && j0 < sz[top]; j0 += kArity) {
            const int cnt = (int)min((int64_t)kArity, sz[top] - j0);
            bool eqn;
            const int k = lane_count<kArity>(m.skey[top], j0, cnt, q, eqn);
            if (top == 0 && k < cnt) bknown = !eqn;
            c += k;
            if (k < cnt) break;
        }
        for (int L = lv; L > 0; L--) {
            if (c == 0) continue;  // nothing below q at this level: nothing below it underneath either
            const int64_t base = (int64_t)kArity * (c - 1) + 1;
            const int64_t end = min((int64_t)kArity * c, sz[L - 1]);
            bool eqn;
            const int cnt = (int)(end - base);
            const int k = lane_count<kArity>(m.skey[L - 1], base, cnt, q, eqn);
            if (L == 1 && k < cnt) bknown = !eqn;
            c = base + k;
        }
    }
    // samples sharing q's prefix widen the block
    int64_t b = c;
    while (!bknown && b < sz[0]) {
        const ulonglong2 k = m.skey[0][b];
        if (k.x != q.hi || k.y != q.lo) break;
        b++;
    }
    c_out = c;
    b_out = b;
}

// std::lower_bound of q over the n boundaries of a tier by one lane (the result and eq as
// group_lower_bound's): lane_sample_range down to one 64-boundary block, then the block's eight
// group starts (skey8) and the seven boundaries after the last start below q; prefix ties compare
// lengths and tails against the boundary itself (probe_cmp_lean).  A run of boundaries sharing q's
// 16-byte prefix over more than one block (tuple subspaces) falls back to a binary search.
__device__ __forceinline__ int64_t lane_lower_bound(const Hist& h, const MaxLevels& m, int64_t n, const DKey& q,
                                                    const uint8_t* htail, const uint8_t* qtail, bool& eq) {
    eq = false;
    if (n <= 0) return 0;
    // Directory slot of at most kLaneProbe skey8 entries (C2: ~10 per slot of the base, ~2 of the
    // delta): the group starts of q's slot are probed at once, so the lookup takes three dependent
    // rounds (directory, group starts, the seven boundaries after the last start below q) instead
    // of four (the level-0 samples first).  Entries before the slot lie below q, entries past it
    // above q (dir_range8); prefix ties compare against the boundary itself (probe_cmp_lean).
    int64_t d8a, d8b;
    const int64_t n8 = (n + 7) >> 3;
    if (dir_range8(m, q, d8a, d8b) && d8b - d8a <= kLaneProbe && d8b <= n8) {
        const int cnt = (int)(d8b - d8a);
        ulonglong2 s8[kLaneProbe];
#pragma unroll
        for (int i = 0; i < kLaneProbe; i++)
            if (i < cnt) s8[i] = m.skey8[d8a + i];
        int r8[kLaneProbe];
        int k8 = 0;
        bool stop = false;
#pragma unroll
        for (int i = 0; i < kLaneProbe; i++) {
            r8[i] = 1;
            if (i < cnt && !stop) {
                r8[i] = probe_cmp_lean(h, 8 * (d8a + i), s8[i], htail, q, qtail);
                if (r8[i] < 0) k8++; else stop = true;
            }
        }
        const int64_t g = d8a + k8 - 1;  // the last group start below q (-1: none)
        if (g < 0) {                     // q <= boundary 0 (probed when the slot holds entry 0)
            eq = cnt > 0 && r8[0] == 0;
            return 0;
        }
        const int64_t B = 8 * g, gend = min(B + 8, n);
        const int nk = (int)(gend - B - 1);
        ulonglong2 kk[7];
#pragma unroll
        for (int i = 0; i < 7; i++)
            if (i < nk) kk[i] = h.key[B + 1 + i];
        int k1 = 0, r_stop = 1;
        stop = false;
#pragma unroll
        for (int i = 0; i < 7; i++) {
            if (i < nk && !stop) {
                const int r = probe_cmp_lean(h, B + 1 + i, kk[i], htail, q, qtail);
                if (r < 0) {
                    k1++;
                } else {
                    stop = true;
                    r_stop = r;
                }
            }
        }
        const int64_t lb = B + 1 + k1;
        if (lb < gend)
            eq = r_stop == 0;
        else if (lb < n)  // lb = 8(g + 1): the next group start, probed above unless past the slot
            eq = k8 < cnt && r8[k8] == 0;
        return lb;
    }
    int64_t c, b;
    lane_sample_range(m, n, q, c, b);
    const int64_t hi = min(n, kFan * b);
    if (b == c) {
        // boundary 64(c-1) < q < boundary 64c: one 64-boundary block; its group starts, then the
        // boundaries after the last start below q
        const int64_t B = c > 0 ? kFan * (c - 1) : 0;
        const int n8 = (int)min((int64_t)8, (hi - B + 7) / 8);  // group starts below hi
        ulonglong2 s8[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (i < n8) s8[i] = m.skey8[B / 8 + i];
        int r8[8];
        int k8 = 0;
        bool stop = false;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            r8[i] = 1;
            if (i < n8 && !stop) {
                r8[i] = probe_cmp_lean(h, B + 8 * i, s8[i], htail, q, qtail);
                if (r8[i] < 0) k8++; else stop = true;
            }
        }
        if (k8 == 0) {  // c == 0 and q <= boundary 0
            eq = hi > 0 && r8[0] == 0;
            return 0;
        }
        const int64_t g = B + 8 * (k8 - 1);  // boundary g < q; the answer lies in (g, min(g + 8, hi)]
        const int64_t gend = min(g + 8, hi);
        const int nk = (int)(gend - g - 1);
        ulonglong2 kk[7];
#pragma unroll
        for (int i = 0; i < 7; i++)
            if (i < nk) kk[i] = h.key[g + 1 + i];
        int k1 = 0;
        int r_stop = 1;
        stop = false;
#pragma unroll
        for (int i = 0; i < 7; i++) {
            if (i < nk && !stop) {
                const int r = probe_cmp_lean(h, g + 1 + i, kk[i], htail, q, qtail);
                if (r < 0) {
                    k1++;
                } else {
                    stop = true;
                    r_stop = r;
                }
            }
        }
        const int64_t lb = g + 1 + k1;
        if (lb < gend)
            eq = r_stop == 0;
        else if (lb < hi)
            eq = k8 < 8 && r8[k8] == 0;  // lb = g + 8: the next group's start, probed above
        return lb;
    }
    // a run of boundaries sharing q's prefix across blocks: binary search with full compares
    int64_t lo = c > 0 ? kFan * (c - 1) + 1 : 0, hh = hi;
    while (lo < hh) {
        const int64_t mid = (lo + hh) >> 1;
        const int r = hist_cmp(h, mid, htail, q, qtail);
        if (r < 0) {
            lo = mid + 1;
        } else {
            hh = mid;
            eq = r == 0;
        }
    }
    if (lo >= hi) eq = false;
    return lo;
}

// ---- per-lane lookups of long keys (batches with keys over 24 bytes: C4 tuple keys)
//
// Keys of one tuple subspace / user share their 16-byte prefix, so a lookup that reaches their run
// compares tails.  One lane per lookup, in three steps: lane_sample_range; the run [s, e) of
// boundaries sharing q's prefix, by prefix-only counts (the group starts of skey8, then the seven
// boundaries after a start: no tails); inside the run a (kRunProbes + 1)-ary search by full
// compares, whose probes' (len, tail offset) and then tails are loaded together against the query
// tail held in registers (QTail): two dependent loads per round.  Keys between two probes share
// with q at least the tail words both probes share with it, so later rounds load and compare only
// the words from there on (C4: the item bytes after a user's ~20-85 shared bytes).
#ifndef FDBCS_RUN_PROBES
#define FDBCS_RUN_PROBES 3
#endif
[[maybe_unused]] constexpr int kRunProbes = FDBCS_RUN_PROBES;

// Boundaries of [lo1, hi) whose prefix is below q's, counted among the n <= N from `base` (sorted).
template <int N>
__device__ __forceinline__ int lane_count_below(const ulonglong2* a, int64_t base, int n, const DKey& q, bool not_above) {
    ulonglong2 k[N];
#pragma unroll
    for (int i = 0; i < N; i++)
        if (i < n) k[i] = a[base + i];
    int c = 0;
#pragma unroll
    for (int i = 0; i < N; i++)
        if (i < n) c += (not_above ? !(q.hi < k[i].x || (q.hi == k[i].x && q.lo < k[i].y)) : prefix_less(k[i], q)) ? 1 : 0;
    return c;
}

// The run of boundaries of [lo1, hi) sharing q's 16-byte prefix: s = the first whose prefix is not
// below q's, e = the first whose prefix is above it (hi if none).  Boundaries before lo1 lie below
// q's prefix, hi and after it above.
__device__ __forceinline__ void lane_prefix_run(const Hist& h, const MaxLevels& m, int64_t lo1, int64_t hi,
                                                const DKey& q, int64_t& s, int64_t& e) {
    const int64_t G0 = (lo1 + 7) / 8;                           // group starts 8g in [lo1, hi)
    const int64_t NG = hi > 8 * G0 ? (hi - 1) / 8 - G0 + 1 : 0;
    if (NG > kLaneProbe) {  // a run over several blocks (a hot subspace): binary searches on prefixes
        int64_t lo = lo1, hh = hi;
        while (lo < hh) {
            const int64_t mid = (lo + hh) >> 1;
            if (prefix_less(h.key[mid], q)) lo = mid + 1; else hh = mid;
        }
        s = lo;
        hh = hi;
        while (lo < hh) {
            const int64_t mid = (lo + hh) >> 1;
            const ulonglong2 k = h.key[mid];
            if (!(q.hi < k.x || (q.hi == k.x && q.lo < k.y))) lo = mid + 1; else hh = mid;
        }
        e = lo;
        return;
    }
    ulonglong2 g[kLaneProbe];
#pragma unroll
    for (int i = 0; i < kLaneProbe; i++)
        if (i < NG) g[i] = m.skey8[G0 + i];
    int kl = 0, kle = 0;
#pragma unroll
    for (int i = 0; i < kLaneProbe; i++) {
        if (i < NG) {
            kl += prefix_less(g[i], q) ? 1 : 0;
            kle += (q.hi < g[i].x || (q.hi == g[i].x && q.lo < g[i].y)) ? 0 : 1;
        }
    }
    // s lies in [as, bs], e in [ae, be]: at most seven boundaries after a group start each
    const int64_t as = kl > 0 ? 8 * (G0 + kl - 1) + 1 : lo1, bs = kl < NG ? 8 * (G0 + kl) : hi;
    const int64_t ae = kle > 0 ? 8 * (G0 + kle - 1) + 1 : lo1, be = kle < NG ? 8 * (G0 + kle) : hi;
    ulonglong2 ks[7], ke[7];
    const int ns = (int)(bs - as), ne = (int)(be - ae);
#pragma unroll
    for (int i = 0; i < 7; i++) {
        if (i < ns) ks[i] = h.key[as + i];
        if (i < ne) ke[i] = h.key[ae + i];
    }
    int cs = 0, ce = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        if (i < ns) cs += prefix_less(ks[i], q) ? 1 : 0;
        if (i < ne) ce += (q.hi < ke[i].x || (q.hi == ke[i].x && q.lo < ke[i].y)) ? 0 : 1;
    }
    s = as + cs;
    e = ae + ce;
}

// lane_lower_bound for long keys (same result and eq); qt: q's tail words (load_qtail).  RP: probes
// per round inside a prefix run (more per round made k_seg_prep's few, latency-bound lookups slower
// at C4: 37.7 / 41.4 / 42.9 us at 3 / 5 / 7).
template <int RP = kRunProbes>
__device__ __forceinline__ int64_t lane_lower_bound_long(const Hist& h, const MaxLevels& m, int64_t n, const DKey& q,
                                                         const QTail& qt, const uint8_t* htail, const uint8_t* qtail,
                                                         bool& eq) {
    eq = false;
    if (n <= 0) return 0;
    int64_t c, b;
    lane_sample_range(m, n, q, c, b);
    int64_t lo, hh;
    lane_prefix_run(h, m, c > 0 ? kFan * (c - 1) + 1 : 0, min(n, kFan * b), q, lo, hh);
#if defined(__HIP_DEVICE_COMPILE__)
    // [lo, hh): boundaries sharing q's prefix, lower_bound among them by full compares.  dlo / dhi:
    // tail words known equal to q's in the boundaries just below lo and at hh (none at first: their
    // prefixes differ from q's).
    int dlo = 0, dhi = 0;
    bool eq_hh = false;  // the boundary at hh equals q (hh was set by a probe)
    const bool qlong = q.len > 16u;
    while (lo < hh) {
        const int64_t span = hh - lo;
        const int w0 = dlo < dhi ? dlo : dhi;  // tail words every boundary in [lo, hh) shares with q
        int64_t p[RP];
        bool v[RP];
        uint2 lt[RP];
#pragma unroll
        for (int j = 0; j < RP; j++) {
            p[j] = lo + (span * (j + 1)) / (RP + 1);
            v[j] = p[j] < hh && (j == 0 || p[j] != p[j - 1]);
            if (v[j]) lt[j] = h.lt[p[j]];
        }
        uint64_t x[RP][kQW];
        uint32_t nb[RP];
#pragma unroll
        for (int j = 0; j < RP; j++) {
            nb[j] = v[j] && qlong && lt[j].x > 16u ? (lt[j].x < q.len ? lt[j].x : q.len) - 16u : 0u;
            const uint64_t* ha = (const uint64_t*)hist_tail(htail, v[j] ? lt[j].y : 0u);
            const int nw = (int)((nb[j] + 7u) / 8u);
#pragma unroll
            for (int u = 0; u < kQW; u++)
                if (u >= w0 && u < nw) x[j][u] = ha[u];
        }
        int r[RP], d[RP];
#pragma unroll
        for (int j = 0; j < RP; j++) {
            r[j] = 1;
            d[j] = 0;
            if (!v[j]) continue;
            const int nw = (int)((nb[j] + 7u) / 8u);
            bool found = false;
#pragma unroll
            for (int u = 0; u < kQW; u++) {
                if (!found && u >= w0 && u < nw) {
                    const int vb = (int)nb[j] - 8 * u;
                    const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
                    const uint64_t hx = __builtin_bswap64(x[j][u]) & msk, qy = qt.w[u] & msk;
                    if (hx != qy) {
                        r[j] = hx < qy ? -1 : 1;
                        d[j] = u;
                        found = true;
                    }
                }
            }
            if (!found) {
                if (nw > kQW) {  // both tails run past the registers: the rest from memory
                    r[j] = tail_cmp(hist_tail(htail, lt[j].y) + 8 * kQW, lt[j].x - 8 * kQW, qtail + q.tail + 8 * kQW,
                                    q.len - 8 * kQW);
                    d[j] = kQW;
                } else {
                    r[j] = (lt[j].x > q.len) - (lt[j].x < q.len);
                    d[j] = (int)(nb[j] / 8u);
                }
            }
        }
        // the probes below q form a prefix of the valid ones
        int64_t nlo = lo, nhh = hh;
        int ndlo = dlo, ndhi = dhi;
        bool neq = eq_hh, hit = false;
#pragma unroll
        for (int j = 0; j < RP; j++) {
            if (!v[j] || hit) continue;
            if (r[j] < 0) {
                nlo = p[j] + 1;
                ndlo = d[j];
            } else {
                nhh = p[j];
                ndhi = d[j];
                neq = r[j] == 0;
                hit = true;
            }
        }
        lo = nlo;
        hh = nhh;
        dlo = ndlo;
        dhi = ndhi;
        eq_hh = neq;
    }
    eq = eq_hh;
#endif
    return lo;
}

// Does the read [kb, ke) (degenerate: [kb, kb)) meet a union segment of the previous batch, i.e.
// would the merge of that batch (SkipList.cpp:899-924: [B, E) set to its `now`, E keeping its old
// version) put a boundary the read counts at `now`?  Segments are disjoint and sorted, so the last
// one whose begin lies below the read's end decides (below its begin for a degenerate read, which
// looks at the greatest boundary < b): it meets the read iff its end lies past the read's begin (at
// or past it for a degenerate read).  Searched by the four lanes of one read (lanes 4i..4i+3 call
// with the same read): 16 probes per round, four per lane.
__device__ __forceinline__ bool prev_seg_hit_quad(const PrevSegs& ps, int64_t U, const DKey& kb, const DKey& ke,
                                                  bool degenerate, const uint8_t* qtail, bool active) {
    const DKey& target = degenerate ? kb : ke;
    const int ql = threadIdx.x & 3;
    int64_t lo = 0, hi = active ? U : 0;  // begins below the target: all of [0, lo), none of [hi, U)
    for (;;) {
        const bool more = lo < hi;
        // the quad's lanes share lo / hi: the loop runs while any read of the wave searches
        if (!__ballot(more)) break;
        int below = 0;
        if (more) {
            int64_t idx[4];
#pragma unroll
            for (int j = 0; j < 4; j++) idx[j] = lo + ((hi - lo) * (4 * ql + j + 1)) / 17;
            DKey d[4];
#pragma unroll
            for (int j = 0; j < 4; j++) d[j] = ps.segk[2 * idx[j]];
#pragma unroll
            for (int j = 0; j < 4; j++) below += dkey_cmp(d[j], ps.tail, target, qtail) < 0 ? 1 : 0;
        }
        // probes below the target form a prefix of the 16 (begins ascend with the index)
        below += __shfl_xor(below, 1, 64);
        below += __shfl_xor(below, 2, 64);
        if (more) {
            const int64_t nlo = below > 0 ? lo + ((hi - lo) * below) / 17 + 1 : lo;
            const int64_t nhi = below < 16 ? lo + ((hi - lo) * (below + 1)) / 17 : hi;
            lo = nlo;
            hi = nhi;
        }
    }
    if (!active || lo == 0) return false;
    const int cmp = dkey_cmp(ps.segk[2 * lo - 1], ps.tail, kb, qtail);  // end of segment lo - 1 vs b
    return degenerate ? cmp >= 0 : cmp > 0;
}

// D.CheckRead of one read by four lanes (both tiers): lane 4i + 0 / 1 locates its begin / end key
// in the base tier, 4i + 2 / 3 in the delta tier; the begin lanes take the end's position by a
// shuffle and decide their tier (tier_conflict); the previous batch's segments by the quad; the
// quad's verdict goes to the read's flags from lane 4i.  (Searching the segments in workgroups of
// their own, as the delta-tier launch does, made this launch 31-34 -> 28-30 us in the C2 pipeline
// but the line 1-2 % slower over three same-box A/Bs: the doubled grid crowds the kernels beside it.)
template <bool LONG>
__device__ __forceinline__ void check_read_lanes(const BatchDev& b, const Tier& base, const Tier& delta,
                                                 const uint8_t* htail, uint8_t* hist_conf, uint8_t* rconf,
                                                 const PrevSegs& ps) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = t >> 2;
    const int k = (int)(t & 3);
    const bool live = r < b.R;
    const int64_t rr = live ? r : 0;
    const DKey kb = b.keys[2 * rr], ke = b.keys[2 * rr + 1];
    const int64_t snap = b.snap[b.rowner[rr]];
    const bool degenerate = dkey_cmp(kb, b.tail, ke, b.tail) == 0;
    const bool is_delta = k >= 2;
    const Tier& tier = is_delta ? delta : base;
    const int64_t n = *tier.n;
    const bool active = live && (!is_delta || n > 0);
    int64_t lb = 0;
    bool eq = false;
    if (active && !((k & 1) && degenerate)) {
        const DKey& q = (k & 1) ? ke : kb;
        if constexpr (LONG) {
            QTail qt;
            load_qtail(qt, q, b.tail);
            lb = lane_lower_bound_long(tier.h, tier.m, n, q, qt, htail, b.tail, eq);
        } else {
            lb = lane_lower_bound(tier.h, tier.m, n, q, htail, b.tail, eq);
        }
    }
    const int64_t j = __shfl_xor(lb, 1, 64);  // the begin lane takes the end key's position
    bool conf = false;
    if (active && !(k & 1)) conf = tier_conflict(tier.h, tier.m, is_delta ? kHole : tier.hdr, lb, eq, j, degenerate, snap);
    if (ps.n) {  // the previous batch's union segments, not merged into the delta yet (every lane
                 // of the quad takes part in the search's shuffles)
        const int64_t U = *ps.n;
        const bool hit = prev_seg_hit_quad(ps, U, kb, ke, degenerate, b.tail, live && U > 0 && ps.version > snap);
        conf = conf || hit;
    }
    int c = conf ? 1 : 0;
    c |= __shfl_xor(c, 1, 64);
    c |= __shfl_xor(c, 2, 64);
    if (live && k == 0) {
        rconf[r] = (uint8_t)c;
        if (c) hist_conf[b.rowner[r]] = 1;
    }
}

// The previous batch's union segments (not merged into the delta the check reads) against read r
// by the four lanes of a quad, in workgroups of their own beside the delta-tier lookups'
// (k_check_lanes_tier): the two dependent chains run side by side instead of one after the other
// in the same lanes (C4: the delta-tier launch 72-78 -> 58-63 us in the pipeline, the line
// +2-6 %).  ORs into the same pre-zeroed flags.
__device__ __forceinline__ void check_read_segs(const BatchDev& b, const PrevSegs& ps, uint8_t* hist_conf,
                                                uint8_t* rconf, int64_t blk) {
    const int64_t t = blk * blockDim.x + threadIdx.x;
    const int64_t r = t >> 2;
    const bool live = r < b.R;
    const int64_t rr = live ? r : 0;
    const DKey kb = b.keys[2 * rr], ke = b.keys[2 * rr + 1];
    const int64_t snap = b.snap[b.rowner[rr]];
    const bool degenerate = dkey_cmp(kb, b.tail, ke, b.tail) == 0;
    const int64_t U = *ps.n;
    const bool hit = prev_seg_hit_quad(ps, U, kb, ke, degenerate, b.tail, live && U > 0 && ps.version > snap);
    int c = hit ? 1 : 0;
    c |= __shfl_xor(c, 1, 64);
    c |= __shfl_xor(c, 2, 64);
    if (live && (t & 3) == 0 && c) {
        rconf[r] = 1;
        hist_conf[b.rowner[r]] = 1;
    }
}

// One tier only (the split check) by two lanes per read: begin / end; a conflict sets the read's and
// its transaction's flags (zeroed beforehand by the epilogue that last used the workspace), so the
// base-tier launch (stage A, on its own stream) and the delta-tier launch (stage B) OR into the
// same flags.  is_base: the tier's header version applies below its first boundary (the delta's
// header is kHole: the base shows through).
template <bool LONG>
__device__ __forceinline__ void check_read_lanes_tier(const BatchDev& b, const Tier& tier, bool is_base,
                                                      const uint8_t* htail, uint8_t* hist_conf, uint8_t* rconf,
                                                      int64_t blk) {
    const int64_t t = blk * blockDim.x + threadIdx.x;
    const int64_t r = t >> 1;
    const int k = (int)(t & 1);
    const bool live = r < b.R;
    const int64_t rr = live ? r : 0;
    const DKey kb = b.keys[2 * rr], ke = b.keys[2 * rr + 1];
    const int64_t snap = b.snap[b.rowner[rr]];
    const bool degenerate = dkey_cmp(kb, b.tail, ke, b.tail) == 0;
    const int64_t n = *tier.n;
    const bool active = live && (is_base || n > 0);
    int64_t lb = 0;
    bool eq = false;
    if (active && !(k && degenerate)) {
        const DKey& q = k ? ke : kb;
        if constexpr (LONG) {
            QTail qt;
            load_qtail(qt, q, b.tail);
            lb = lane_lower_bound_long(tier.h, tier.m, n, q, qt, htail, b.tail, eq);
        } else {
            lb = lane_lower_bound(tier.h, tier.m, n, q, htail, b.tail, eq);
        }
    }
    const int64_t j = __shfl_xor(lb, 1, 64);
    bool conf = false;
    if (active && !k) conf = tier_conflict(tier.h, tier.m, is_base ? tier.hdr : kHole, lb, eq, j, degenerate, snap);
    int c = conf ? 1 : 0;
    c |= __shfl_xor(c, 1, 64);
    if (live && !k && c) {
        rconf[r] = 1;
        hist_conf[b.rowner[r]] = 1;
    }
}

// ------------------------------------------------------------------ D.Sort

// Endpoint item p of the batch (KeyInfo, SkipList.cpp:77-87): range g = p / 2, end = p & 1.
__device__ __forceinline__ SortItem make_item(const BatchDev& b, int p) {
    const int g = p >> 1, e = p & 1;
    const DKey k = b.keys[p];
    // extra_ordering (SkipList.cpp:89-91): begin*2 + (write ^ begin)
    const uint32_t cls = g < b.R ? (e ? kReadEnd : kReadBegin) : (e ? kWriteEnd : kWriteBegin);
    SortItem it;
    it.hi = k.hi;
    it.lo = k.lo;
    it.len = k.len;
    it.tail = k.tail;
    it.meta = ((uint32_t)g << 3) | ((uint32_t)e << 2) | cls;
    it.nx = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    if (k.len > 16u) {
        const uint32_t nb = k.len - 16u < 3u ? k.len - 16u : 3u;
        it.nx = (uint32_t)(tail_word(b.tail + k.tail) >> 40) & (0xffffffu << (8u * (3u - nb))) & 0xffffffu;
    }
#endif
    return it;
}

// The last (up to) 8 bytes of a tail of tl bytes, big-endian.
__device__ __forceinline__ uint64_t tail_last(const uint8_t* t, uint32_t tl) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (tl >= 8) return tail_word(t + tl - 8);
    return tl ? tail_word(t) & (~0ull << (64 - 8 * tl)) : 0ull;
#else
    (void)t;
    (void)tl;
    return 0;
#endif
}

// Total order used by the sort: KeyInfo::operator< (key, then class; SkipList.cpp:114-128) with the
// endpoint id as a final tie-break.  Endpoints equal in (key, class) are interchangeable for every
// later use, so the tie-break changes nothing observable; it makes every item distinct,
// which keeps sample-sort buckets balanced even when one hot key repeats thousands of times.
__device__ __forceinline__ bool item_less_tail(uint32_t alen, uint32_t atail, uint32_t ameta, uint32_t blen,
                                            uint32_t btail, uint32_t bmeta, const uint8_t* arena) {
    const int c = tail_cmp(arena + atail, alen, arena + btail, blen);
    if (c) return c < 0;
    const uint32_t ca = item_class(ameta), cb = item_class(bmeta);
    if (ca != cb) return ca < cb;
    return ameta < bmeta;
}

// Packed tie-break word after equal 16-byte prefixes: key bytes [16, 19), length capped at 20
// (20 stands for "longer than kSortNxLen"), class, endpoint id.  It decides every pair except two
// keys both longer than kSortNxLen with equal words (see item_tie).
__device__ __forceinline__ uint64_t item_aux(const SortItem& a) {
    const uint64_t l = a.len > kSortNxLen ? kSortNxLen + 1 : a.len;
    return ((uint64_t)(a.nx & 0xffffffu) << 37) | (l << 32) | ((uint64_t)item_class(a.meta) << 30) | (a.meta >> 2);
}
// Equal prefixes: does the order need the tail bytes?
__device__ __forceinline__ bool item_tie(const SortItem& a, const SortItem& b) {
    return a.len > kSortNxLen && b.len > kSortNxLen && (a.nx & 0xffffffu) == (b.nx & 0xffffffu);
}
__device__ __forceinline__ bool is_pad(const SortItem& a) { return a.meta == kPadMeta; }

// Branch-free on the common path; the tail comparison (both keys longer than 16 bytes with
// equal prefixes) is out of line.
__device__ __forceinline__ bool item_less_total(const SortItem& a, const SortItem& b, const uint8_t* arena) {
    const bool hi_eq = a.hi == b.hi, lo_eq = a.lo == b.lo;
    if (hi_eq && lo_eq && item_tie(a, b))
        return item_less_tail(a.len, a.tail, a.meta, b.len, b.tail, b.meta, arena);
    const bool aux_lt = item_aux(a) < item_aux(b);
    return (a.hi < b.hi) | (hi_eq & ((a.lo < b.lo) | (lo_eq & aux_lt)));
}

// Rank counting: rk[k] += number of items of sh[0, cnt) ordered before mine[k].  Branch-free on
// the 16-byte prefix and the (length, class, id) tie-break word, 8 LDS reads in flight; a
// comparison that needs the bytes beyond the prefix (both keys longer than 16 bytes, equal
// prefixes) only raises `tail`, and the caller recounts that item exactly.
template <int P>
__device__ __forceinline__ void rank_count(const SortItem* sh, int cnt, const SortItem (&mine)[P], int (&rk)[P],
                                           bool& tail) {
    uint64_t maux[P];
#pragma unroll
    for (int k = 0; k < P; k++) maux[k] = item_aux(mine[k]);
    auto one = [&](const SortItem& x) {
        const uint64_t xa = item_aux(x);
#pragma unroll
        for (int k = 0; k < P; k++) {
            const bool heq = x.hi == mine[k].hi, leq = x.lo == mine[k].lo;
            rk[k] += ((x.hi < mine[k].hi) | (heq & ((x.lo < mine[k].lo) | (leq & (xa < maux[k]))))) ? 1 : 0;
            tail |= heq && leq && item_tie(x, mine[k]) && x.meta != mine[k].meta;
        }
    };
    int j = 0;
    for (; j + 8 <= cnt; j += 8) {
        SortItem x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = sh[j + u];
#pragma unroll
        for (int u = 0; u < 8; u++) one(x[u]);
    }
    for (; j < cnt; j++) one(sh[j]);
}

// Exact rank of one item (tail comparisons included): the slow path of rank_count.
__device__ __noinline__ int rank_exact(const SortItem* sh, int cnt, SortItem mine, const uint8_t* arena) {
    int r = 0;
    for (int j = 0; j < cnt; j++) r += item_less_total(sh[j], mine, arena) ? 1 : 0;
    return r;
}

// ---- cold start of the sort: samples of the batch ranked against each other
constexpr int kSampleSlice = 64;

__device__ __forceinline__ int sample_pos(int i, int E, int S) { return (int)(((int64_t)i * E) / S); }

// Sample ranking (stage A, history-independent): workgroup (x, y) ranks samples [y*256, y*256+256)
// against the slice [x*64, x*64+64); partial ranks are added atomically.
struct SampleRank {
    int S, n_slice;
    int32_t* srank;  // [S] ranks (zeroed by the previous epilogue on this workspace)
    SortItem* samples;  // [S] the sample items, for k_bucket_count
    unsigned long long* trace;
};

__global__ __launch_bounds__(kBlock) void k_sample(BatchDev b, SampleRank c) {
    __shared__ SortItem sl[kSampleSlice];
    if (threadIdx.x == 0) trace_min(c.trace, kTrSampleBegin);
    const int E = 2 * (b.R + b.W), S = c.S;
    const int x = blockIdx.x % c.n_slice, y = blockIdx.x / c.n_slice;
    const int j0 = x * kSampleSlice;
    const int cj = min(kSampleSlice, S - j0);
    const int i = y * blockDim.x + threadIdx.x;
    // this thread's sample is loaded before the slice barrier (its loads overlap the slice's)
    SortItem mine[1];
    if (i < S) mine[0] = make_item(b, sample_pos(i, E, S));
    for (int t = threadIdx.x; t < cj; t += blockDim.x) sl[t] = make_item(b, sample_pos(j0 + t, E, S));
    __syncthreads();
    if (i < S) {
        if (x == 0) c.samples[i] = mine[0];
        int cnt[1] = {0};
        bool tail = false;
        rank_count<1>(sl, cj, mine, cnt, tail);
        if (tail) cnt[0] = rank_exact(sl, cj, mine[0], b.tail);
        if (cnt[0]) atomicAdd(&c.srank[i], cnt[0]);
    }
    if (threadIdx.x == 0) trace_max(c.trace, kTrSampleEnd);
}

// D.CheckRead (stage B: reads the history as the previous batch left it).
struct CheckReads {
    Tier base, delta;
    const uint8_t* htail;
    uint8_t *hist_conf, *rconf;
    unsigned long long* trace;
    PrevSegs ps;  // the previous batch's union segments, not merged yet
};

// Per-lane checks: both tiers, four lanes per read; one tier (the split check), two lanes per read;
// two instantiations of the tier launch so profiles tell the base and delta launches apart.
// LONG: the batch has keys over 24 bytes (lane_lower_bound_long).
template <bool LONG>
__global__ __launch_bounds__(kBlock) void k_check_lanes(BatchDev b, CheckReads c) {
    check_read_lanes<LONG>(b, c.base, c.delta, c.htail, c.hist_conf, c.rconf, c.ps);
}
template <bool BASE, bool LONG>
__global__ __launch_bounds__(kBlock) void k_check_lanes_tier(BatchDev b, Tier t, const uint8_t* htail,
                                                             uint8_t* hist_conf, uint8_t* rconf, PrevSegs ps,
                                                             int look_blocks) {
    // workgroups past look_blocks search the previous batch's segments (check_read_segs)
    if ((int)blockIdx.x < look_blocks)
        check_read_lanes_tier<LONG>(b, t, BASE, htail, hist_conf, rconf, blockIdx.x);
    else
        check_read_segs(b, ps, hist_conf, rconf, blockIdx.x - look_blocks);
}

void launch_check_tier(hipStream_t s, const BatchDev& b, const Work& w, const Tier& t, bool is_base,
                       const uint8_t* htail, bool long_keys, const PrevSegs& ps) {
    if (b.R == 0) return;
    const int grid = (int)(((int64_t)b.R * 2 + kBlock - 1) / kBlock);
    const int seg = !is_base && ps.n ? (int)(((int64_t)b.R * 4 + kBlock - 1) / kBlock) : 0;
    auto k = is_base ? (long_keys ? k_check_lanes_tier<true, true> : k_check_lanes_tier<true, false>)
                     : (long_keys ? k_check_lanes_tier<false, true> : k_check_lanes_tier<false, false>);
    fdb_launch(k, dim3(grid + seg), dim3(kBlock), 0, s, b, t, htail, w.hist_conf, w.rconf, seg ? ps : PrevSegs{}, grid);
}

void launch_check(hipStream_t s, const BatchDev& b, const Work& w, const Tier& base, const Tier& delta,
                  const uint8_t* htail, bool long_keys, const PrevSegs& ps) {
    if (b.R == 0) return;
    const CheckReads c{base, delta, htail, w.hist_conf, w.rconf, w.trace, ps};
    const int grid = (int)(((int64_t)b.R * 4 + kBlock - 1) / kBlock);
    fdb_launch(long_keys ? k_check_lanes<true> : k_check_lanes<false>, dim3(grid), dim3(kBlock), 0, s, b, c);
}

// ---- D.Sort (SkipList.cpp:161-208) and the sorted positions (KeyInfo::pIndex, SkipList.cpp:814)
//
// Two launches per batch (a cold start adds two small ones before them):
// 1. k_sort_partition: an endpoint's bucket is the number of splitters not above its projection
//    (SplitKey: binary search over the splitters' first two key words in LDS; ties there compare
//    the rest of the 64-byte windows in global memory).  One 64-bit atomic add per endpoint
//    reserves its slot in the bucket's slab and counts its class; past kSlab it joins the overflow
//    list.
// 2. k_sort_bucket: one wave per bucket.  The bucket counts give each bucket's offset and class
//    offsets (every workgroup reduces them itself: no scan launch).  Every key of a bucket shares
//    the bytes its two bounding splitters share, so the wave sorts by the 19 key bytes after that
//    common prefix (two words and a tie-break word, as the whole key's first 19 bytes before):
//    up to kSlab endpoints in registers, a bitonic network four per lane, cross-lane steps by
//    shuffles; runs tied on those 19 bytes are then ranked by their tails.  The wave writes each
//    position's meta, every endpoint's position, the class counts before every position and the
//    write-begin / read-begin position lists (what the position scan wrote before), and the
//    quantiles the next batch splits by.  A bucket past kSlab (skew the splitters did not
//    foresee) is ranked by its whole workgroup.
// Splitters are the projections of the quantiles of the last batch of at least kQuantMinE
// endpoints (a resolver's key distribution drifts slowly, and any splitters are exact: they only
// decide balance); at a cold start, of this batch's samples ranked by k_sample.

// Big-endian 8 key bytes from byte `off` (zero past the key's length): the first 16 bytes come
// from the prefix words, the rest from the tail bytes [16, len) at `tail`.
__device__ __forceinline__ uint64_t key_word(uint64_t hi, uint64_t lo, const uint8_t* tail, uint32_t len,
                                             uint32_t off) {
    if (off >= len) return 0;
    uint64_t v;
#if defined(__HIP_DEVICE_COMPILE__)
    if (off == 0) {
        v = hi;
    } else if (off < 8) {
        v = (hi << (8 * off)) | (lo >> (64 - 8 * off));
    } else if (off == 8) {
        v = lo;
    } else if (off < 16) {
        v = lo << (8 * (off - 8));
        if (len > 16) v |= tail_word(tail) >> (64 - 8 * (off - 8));
    } else {
        v = tail_word(tail + (off - 16));
    }
#else
    v = 0;
#endif
    const uint32_t valid = len - off;
    return valid >= 8 ? v : v & (~0ull << (8 * (8 - valid)));
}

// Tie-break word of an endpoint whose key bytes [0, c) are already known equal among the keys it
// is sorted with: key bytes [c + 16, c + kSortNxLen), length past c capped at kSortNxLen + 1,
// class, endpoint id (item_aux of the key with its first c bytes removed).
// Layout of the bucket sort's tie-break word: window bytes at bits 38-61, the capped length at
// 33-37, the range-end flag at 32 (kNxEndFlag, only for keys longer than the window: tied keys,
// whose run the tie ranking would otherwise order), class at 30-31, endpoint id at 0-29.
__device__ __forceinline__ uint64_t sort_aux(uint64_t nx24, uint32_t len_c, uint32_t meta, uint32_t nxf) {
    const uint64_t l = len_c > kSortNxLen ? kSortNxLen + 1 : len_c;
    const uint64_t f = len_c > kSortNxLen && (nxf & kNxEndFlag) ? 1ull : 0ull;
    return (nx24 << 38) | (l << 33) | (f << 32) | ((uint64_t)item_class(meta) << 30) | (meta >> 2);
}
__device__ __forceinline__ uint64_t aux_at(uint64_t w2, uint32_t len_c, uint32_t meta, uint32_t nxf) {
    return sort_aux(w2 >> 40, len_c, meta, nxf);
}
__device__ __forceinline__ bool key3_less(uint64_t ah, uint64_t al, uint64_t aa, uint64_t bh, uint64_t bl,
                                          uint64_t ba) {
    return ah < bh || (ah == bh && (al < bl || (al == bl && aa < ba)));
}
// Quantile-table entry of splitter k (of nb - 1).
__device__ __forceinline__ int split_index(int k, int nb) { return (int)(((int64_t)(k + 1) * kQuant) / nb); }
// Position of quantile q in a sorted batch of E endpoints.
__device__ __forceinline__ int64_t quant_pos(int q, int64_t E) { return ((int64_t)(q + 1) * E) / (kQuant + 1); }

// The splitter an endpoint projects to.
__device__ __forceinline__ SplitKey make_split(const SortItem& it, const uint8_t* arena) {
    SplitKey s;
    s.w[0] = it.hi;
    s.w[1] = it.lo;
#pragma unroll
    for (int i = 2; i < kSplitWords; i++) s.w[i] = key_word(it.hi, it.lo, arena + it.tail, it.len, 8 * i);
    s.len = it.len;
    s.meta = it.meta;
    return s;
}
// Projection order past the first two words: words 2.., min(len, kSplitBytes + 1), then class and
// id when both keys fit the window.  -1, 0, 1.
__device__ __forceinline__ int split_cmp_rest(const uint64_t (&a)[kSplitWords], uint32_t alen, uint32_t ameta,
                                              const SplitKey& b) {
#pragma unroll
    for (int i = 2; i < kSplitWords; i++)
        if (a[i] != b.w[i]) return a[i] < b.w[i] ? -1 : 1;
    const uint32_t la = alen > kSplitBytes ? kSplitBytes + 1 : alen, lb = b.len > kSplitBytes ? kSplitBytes + 1 : b.len;
    if (la != lb) return la < lb ? -1 : 1;
    if (la > kSplitBytes) return 0;  // tied on the window: one projection
    const uint32_t ca = item_class(ameta), cb = item_class(b.meta);
    if (ca != cb) return ca < cb ? -1 : 1;
    return (ameta >> 2) < (b.meta >> 2) ? -1 : ((ameta >> 2) > (b.meta >> 2) ? 1 : 0);
}

// Bucket k's counters: cnt[kCntStride k] = endpoints | write-begins << 32, cnt[kCntStride k + 1] =
// read-begins | write-ends << 32, one bucket per 128-byte line: the atomics of different buckets
// never share a line (device-scope atomics on one line serialize at the memory side).
struct SortArgs {
    uint8_t* btail;  // the workspace's copy of the batch tail region (see Work::btail)
    int64_t btail_n; // bytes of the batch tail region
    const SplitKey* quant;
    uint64_t* cnt;
    SortItem* slab;
    SortItem* ovf;
    int32_t* ovf_b;
    BatchScalars* bsc;
    int nb;
    unsigned long long* trace;
    int exp = 0;  // fdbcs_debug_kernel_time (FDBCS_SORT_EXP): 1 skips the tie ranking, 2 the position writes, 4 the network, 8 the count prologue
    int long_keys = 0;  // keys over kSortNxLen bytes: the partition marks the ends of non-empty ranges
};

__global__ __launch_bounds__(kBlock) void k_sort_partition(BatchDev b, SortArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_spl[];  // [2 (nb - 1)]: first two key words
    const int E = 2 * (b.R + b.W), nb = a.nb, ns = nb - 1;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (threadIdx.x == 0) trace_min(a.trace, kTrPartBegin);
    const unsigned long long tp0 = a.trace ? wall_clock64() : 0ull;
    SortItem it{};
    if (p < E) it = make_item(b, p);  // in flight during the splitter fill
    // the end of a range also loads its begin's key: is the range non-empty? (kNxEndFlag)
    const bool mark = a.long_keys && p < E && (p & 1);
    DKey pk{};
    if (mark) pk = b.keys[p ^ 1];
    for (int k = threadIdx.x; k < ns; k += blockDim.x) {
        const SplitKey* sk = &a.quant[split_index(k, nb)];
        s_spl[2 * k] = sk->w[0];
        s_spl[2 * k + 1] = sk->w[1];
    }
    __syncthreads();
    if (threadIdx.x == 0) trace_max(a.trace, kTrPartFill);
    const unsigned long long tp1 = a.trace ? wall_clock64() : 0ull;
    if (a.btail && p < E && (p >> 1) >= b.R && it.len > 16u) {
        // the tails of the write endpoints' keys into the workspace copy at the same offsets (the
        // union segments the next batch's check reads are made of write keys only): the aligned
        // words holding the tail; neighbouring keys' threads may write a shared word, always with
        // the same bytes
        const uint64_t* src = (const uint64_t*)b.tail;
        uint64_t* dst = (uint64_t*)a.btail;
        const int64_t w0 = it.tail / 8, w1 = ((int64_t)it.tail + (it.len - 16u) + 7) / 8;
        for (int64_t q = w0; q < w1; q++) dst[q] = src[q];
    }
    if (p >= E) {
        if (a.trace) trace_max(a.trace, kTrPartEnd);
        return;
    }
    unsigned long long tp2 = 0;
    if (a.trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tp2 = wall_clock64();
    }
    // splitters below my first two words: [0, lo); equal to them: [lo, up)
    int lo = 0, hi = ns;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint64_t h = s_spl[2 * mid], l = s_spl[2 * mid + 1];
        if (h < it.hi || (h == it.hi && l < it.lo)) lo = mid + 1; else hi = mid;
    }
    // the splitters equal to my first two words, [lo, up): searched only when the first one not
    // below me is equal (hot keys, shared prefixes), one LDS probe otherwise
    int up = lo;
    if (lo < ns && s_spl[2 * lo] == it.hi && s_spl[2 * lo + 1] == it.lo) {
        up = lo + 1;
        hi = ns;
        while (up < hi) {
            const int mid = (up + hi) >> 1;
            const uint64_t h = s_spl[2 * mid], l = s_spl[2 * mid + 1];
            if (h < it.hi || (h == it.hi && l <= it.lo)) up = mid + 1; else hi = mid;
        }
    }
    int bk = lo;
    if (up > lo) {  // ties on 16 bytes (hot keys, shared prefixes): the rest of the window
        uint64_t wv[kSplitWords];
        wv[0] = it.hi;
        wv[1] = it.lo;
#pragma unroll
        for (int i = 2; i < kSplitWords; i++) wv[i] = key_word(it.hi, it.lo, b.tail + it.tail, it.len, 8 * i);
        int l = lo, h = up;  // splitters in [lo, up) not above my projection
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (split_cmp_rest(wv, it.len, it.meta, a.quant[split_index(mid, nb)]) >= 0) l = mid + 1; else h = mid;
        }
        bk = l;
    }
    if (a.trace) trace_max(a.trace, kTrPartSearch);
    const unsigned long long tp3 = a.trace ? wall_clock64() : 0ull;
    if (mark && it.len > kSortNxLen) {  // (the flag matters only to keys the sort window cannot decide)
        bool ne = pk.hi != it.hi || pk.lo != it.lo || pk.len != it.len;
        if (!ne) {  // equal prefixes and lengths (> 19 bytes): last tail words first, then the tails
            const uint32_t tl = it.len - 16u;
            ne = tail_last(b.tail + it.tail, tl) != tail_last(b.tail + pk.tail, tl) ||
                 tail_cmp(b.tail + it.tail, it.len, b.tail + pk.tail, pk.len) != 0;
        }
        if (ne) it.nx |= kNxEndFlag;
    }
    const uint32_t cls = item_class(it.meta);
    const unsigned long long old =
        atomicAdd((unsigned long long*)&a.cnt[(size_t)kCntStride * bk], 1ull | (cls == kWriteBegin ? 1ull << 32 : 0ull));
    if (cls == kReadBegin || cls == kWriteEnd)
        atomicAdd((unsigned long long*)&a.cnt[(size_t)kCntStride * bk + 1], cls == kReadBegin ? 1ull : 1ull << 32);
    const uint32_t slot = (uint32_t)old;
    if (slot < (uint32_t)kSlab) {
        a.slab[(size_t)bk * kSlab + slot] = it;
    } else {
        const int o = atomicAdd(&a.bsc->ovf_n, 1);
        a.ovf[o] = it;
        a.ovf_b[o] = bk;
    }
    if (a.trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        trace_max(a.trace, kTrPartEnd);
        if ((threadIdx.x & 63) == 0) {
            const unsigned long long tp4 = wall_clock64();
            atomicAdd(&a.trace[kTrPartWaves], 1ull);
            atomicAdd(&a.trace[kTrPartSumFill], tp1 - tp0);
            atomicAdd(&a.trace[kTrPartSumCopy], tp2 - tp1);
            atomicAdd(&a.trace[kTrPartSumSearch], tp3 - tp2);
            atomicAdd(&a.trace[kTrPartSumPlace], tp4 - tp3);
        }
    }
}

// Outputs of k_sort_bucket: what the later kernels read by sorted position.
struct SortOut {
    int32_t* pos;      // [E] position of endpoint p
    uint32_t* pmeta;   // [E] meta at position P
    int32_t *cwb, *crb, *cwe;  // [E + 1] write-begins / read-begins / write-ends before position P
    int32_t *wbrange, *rbrange;  // ranges of the write-begins / read-begins in sorted order
    SortItem* items;   // [E] sorted items (FDBCS_VALIDATE) or null
    SplitKey* quant;   // quantiles of this batch for the next one, or null
    SortItem* big;     // [E] workgroup path: gathered endpoints of a big bucket
    int32_t* big_p;    // [E] workgroup path: its endpoint ids in sorted order
};

// Bitonic network over 64 S (hi, lo, aux) triples of one wave: element s * 64 + lane in slot s of
// the lane; partners closer than 64 by lane exchanges (lane_xor64), farther ones inside the lane's
// registers.
template <int S>
__device__ __forceinline__ void wave_bitonic(uint64_t (&kh)[4], uint64_t (&kl)[4], uint64_t (&ka)[4]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k <= 64 * S; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
                const int js = j >> 6;
#pragma unroll
                for (int s = 0; s < S; s++) {
                    if (s & js) continue;
                    const int t = s | js;
                    const bool up = ((s * 64 + lane) & k) == 0;
                    if (key3_less(kh[t], kl[t], ka[t], kh[s], kl[s], ka[s]) == up) {
                        uint64_t x = kh[s]; kh[s] = kh[t]; kh[t] = x;
                        x = kl[s]; kl[s] = kl[t]; kl[t] = x;
                        x = ka[s]; ka[s] = ka[t]; ka[t] = x;
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < S; s++) {
                    const uint64_t yh = lane_xor64_rt(kh[s], j), yl = lane_xor64_rt(kl[s], j),
                                   ya = lane_xor64_rt(ka[s], j);
                    const bool up = ((s * 64 + lane) & k) == 0, lower = (lane & j) == 0;
                    const bool y_less = key3_less(yh, yl, ya, kh[s], kl[s], ka[s]);
                    if (lower == up ? y_less : !y_less) {
                        kh[s] = yh;
                        kl[s] = yl;
                        ka[s] = ya;
                    }
                }
            }
        }
    }
}

// Meta of endpoint p (range p / 2, end p & 1; class as extra_ordering, SkipList.cpp:89-91).
__device__ __forceinline__ uint32_t endpoint_meta(const BatchDev& b, int p) {
    const int g = p >> 1, e = p & 1;
    const uint32_t cls = g < b.R ? (e ? kReadEnd : kReadBegin) : (e ? kWriteEnd : kWriteBegin);
    return ((uint32_t)g << 3) | ((uint32_t)e << 2) | cls;
}

// The quantiles of this batch at global position P (several when E < kQuant).
__device__ __forceinline__ void put_quantiles(const BatchDev& b, SplitKey* quant, int64_t P, int64_t E, int p) {
    int q = (int)((P * (kQuant + 1) + E - 1) / E) - 1;  // ceil(P (Q+1) / E) - 1
    if (q < 0) q = 0;
    if (q >= kQuant || quant_pos(q, E) > P) return;
    const SplitKey sk = make_split(make_item(b, p), b.tail);
    for (; q < kQuant && quant_pos(q, E) <= P; q++)
        if (quant_pos(q, E) == P) quant[q] = sk;
}

// Writes of sorted position P (endpoint p) given the class counts before it.
__device__ __forceinline__ void put_position(const BatchDev& b, const SortOut& o, int p, int64_t P, int32_t wb,
                                             int32_t rb, int32_t we) {
    const uint32_t meta = endpoint_meta(b, p);
    const uint32_t cls = item_class(meta);
    o.pmeta[P] = meta;
    o.pos[p] = (int32_t)P;
    o.cwb[P] = wb;
    o.crb[P] = rb;
    o.cwe[P] = we;
    if (cls == kWriteBegin) o.wbrange[wb] = p >> 1;  // (the edge scans want the range, not P)
    if (cls == kReadBegin) o.rbrange[rb] = p >> 1;
    if (o.items) o.items[P] = make_item(b, p);
}

// Bytes [0, c) shared by every key between splitters a and b (c <= both lengths, <= the window).
__device__ __forceinline__ uint32_t split_lcp(const SplitKey& a, const SplitKey& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < kSplitWords; i++) {
        const uint64_t x = a.w[i] ^ b.w[i];
        if (x) {
            c = 8 * i + (uint32_t)(__builtin_clzll(x) >> 3);
            break;
        }
        c = 8 * (i + 1);
    }
    c = c < a.len ? c : a.len;
    return c < b.len ? c : b.len;
}

template <bool LONG>
__global__ __launch_bounds__(kBlock) void k_sort_bucket(BatchDev b, SortArgs a, SortOut o) {
    constexpr int kWaves = kBlock / 64;
    __shared__ uint32_t s_red[8][kWaves];
    __shared__ uint32_t s_cnt[kWaves][4];   // per wave's bucket: endpoints, write-begins, read-begins, write-ends
    __shared__ uint32_t s_base[kWaves][4];  // the same counts over every bucket before it
    __shared__ int32_t s_p[kWaves][kSlab];  // tied runs: endpoint at each final position
    __shared__ uint8_t s_tie[kWaves][kSlab];
    __shared__ int s_big[kWaves];
    __shared__ SortItem s_tile[kBlock];     // workgroup path: a tile of the big bucket
    __shared__ int s_gather;
    const int E = 2 * (b.R + b.W), nb = a.nb;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int B0 = blockIdx.x * kWaves;
    if (threadIdx.x == 0) trace_min(a.trace, kTrBktBegin);
    // ---- this wave's bucket: its own counts first (one line), then every thread's share of the
    // counters the bucket offsets sum (all buckets before B0, and all), issued now and summed only
    // after the network so their latency hides behind the slab loads and the sort
    const int bk = B0 + wave;
    uint64_t own0 = 0, own1 = 0;
    if (bk < nb && !(a.exp & 8)) {
        own0 = a.cnt[(size_t)kCntStride * bk];
        own1 = a.cnt[(size_t)kCntStride * bk + 1];
    }
    if (a.exp & 8) own0 = bk < nb ? (64ull | 16ull << 32) : 0ull, own1 = bk < nb ? (16ull | 16ull << 32) : 0ull;
    // (the first kPreHeld chunks stay in registers across the sort, enough for nb <= 1536 buckets,
    // ~98k endpoints; larger batches load the rest after it)
    constexpr int kPreLoads = kSortMaxBuckets / kBlock, kPreHeld = 6;
    uint64_t c0[kPreHeld], c1[kPreHeld];
#pragma unroll
    for (int u = 0; u < kPreHeld; u++) {
        const int k = threadIdx.x + u * kBlock;
        const bool in = k < nb && !(a.exp & 8);  // (exp 8: cost breakdown only)
        c0[u] = in ? a.cnt[(size_t)kCntStride * k] : 0;
        c1[u] = in ? a.cnt[(size_t)kCntStride * k + 1] : 0;
    }
    const int n = (int)(uint32_t)own0;
    const bool small = bk < nb && n > 0 && n <= kSlab;
    int ps[4] = {0, 0, 0, 0};  // endpoint at each position of the wave's bucket (after the sort)
    int S = 1;
    unsigned long long tt[3] = {0, 0, 0};  // FDBCS_TRACE section stamps
    if (small) {
        const unsigned long long tw0 = a.trace ? wall_clock64() : 0ull;
        unsigned long long tw1 = 0, tw2 = 0;
        // bytes every key of the bucket shares: those its bounding splitters share (none at the ends)
        // (batches of keys up to kSortNxLen bytes sort exactly on their first 19 bytes: no strip)
        uint32_t c = 0;
        if (LONG && bk > 0 && bk < nb - 1)
            c = split_lcp(a.quant[split_index(bk - 1, nb)], a.quant[split_index(bk, nb)]);
        uint64_t kh[4], kl[4], ka[4];
        S = n <= 64 ? 1 : (n <= 128 ? 2 : 4);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int k = s * 64 + lane;
            kh[s] = kl[s] = ka[s] = ~0ull;  // padding sorts after every endpoint
            if (s < S && k < n) {
                const SortItem it = a.slab[(size_t)bk * kSlab + k];
                if (c == 0) {
                    kh[s] = it.hi;
                    kl[s] = it.lo;
                    ka[s] = sort_aux(it.nx & 0xffffffu, it.len, it.meta, it.nx);
                } else {  // the key with its first c bytes removed
                    const uint8_t* t = b.tail + it.tail;
                    kh[s] = key_word(it.hi, it.lo, t, it.len, c);
                    kl[s] = key_word(it.hi, it.lo, t, it.len, c + 8);
                    ka[s] = aux_at(key_word(it.hi, it.lo, t, it.len, c + 16), it.len - c, it.meta, it.nx);
                }
            }
        }
        if (a.trace) tw1 = wall_clock64();
        if (a.exp & 4) {  // cost breakdown only: no network
        } else if (S == 1) wave_bitonic<1>(kh, kl, ka);
        else if (S == 2) wave_bitonic<2>(kh, kl, ka);
        else wave_bitonic<4>(kh, kl, ka);
        if (lane == 0) trace_max(a.trace, kTrBktSorted);
        if (a.trace) tw2 = wall_clock64();
#pragma unroll
        for (int s = 0; s < 4; s++) ps[s] = (int)(ka[s] & 0x3fffffffull);
        if ((LONG || c > 0) && !(a.exp & 1)) {  // exp: fdbcs_debug_kernel_time's cost breakdown only
            // positions k, k+1 tied: same two words, both keys longer than kSortNxLen past c with
            // equal bytes up to there: their order needs the tails
            bool any = false;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                if (s >= S) break;
                uint64_t nh = __shfl_down(kh[s], 1, 64), nl = __shfl_down(kl[s], 1, 64),
                         na = __shfl_down(ka[s], 1, 64);
                const int s1 = s + 1 < 4 ? s + 1 : 3;
                const uint64_t h2 = __shfl(kh[s1], 0, 64), l2 = __shfl(kl[s1], 0, 64), a2 = __shfl(ka[s1], 0, 64);
                if (lane == 63) {  // the next slot's lane 0
                    nh = h2;
                    nl = l2;
                    na = a2;
                }
                const int k = s * 64 + lane;
                const bool tie = k + 1 < n && nh == kh[s] && nl == kl[s] && (na >> 33) == (ka[s] >> 33) &&
                                 ((ka[s] >> 33) & 31u) == kSortNxLen + 1;
                s_tie[wave][k] = tie ? 1 : 0;
                s_p[wave][k] = ps[s];
                any |= tie;
            }
            if (__ballot(any)) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                int fin[4];
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int k = s * 64 + lane;
                    fin[s] = k;
                    if (s >= S) break;  // uniform
                    const bool in_run = k < n && (s_tie[wave][k] || (k > 0 && s_tie[wave][k - 1]));
                    int st = k, en = k;
                    if (in_run) {
                        while (st > 0 && s_tie[wave][st - 1]) st--;
                        while (s_tie[wave][en]) en++;
                    }
                    // a run of just the two ends of one range is in order already: the sort word
                    // holds the range-end flag (begin first when the keys differ, else class order)
                    const bool pair = in_run && en == st + 1 && (s_p[wave][k == st ? en : st] >> 1) == (ps[s] >> 1);
                    bool todo = in_run && !pair;
                    // Runs inside this slot's 64 positions: every member loads its own key's tail
                    // words once (two dependent loads) and takes the others' by shuffles, so a
                    // member's rank costs no load per other member.  Tied keys share their first
                    // c + 19 > 16 bytes: the order is the tails, then the length, class and id.
                    const bool simple = todo && st >= s * 64 && en < s * 64 + 64 && en - st < 16;
                    DKey kme{};
                    QTail tw;
                    if (simple) {
                        kme = b.keys[ps[s]];
                        load_qtail(tw, kme, b.tail);
                    }
                    bool fallback = simple && kme.len > 16u + 8u * kQW;  // past the words held
                    int mr = simple ? en - st + 1 : 0;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int y = __shfl_xor(mr, o, 64);
                        mr = y > mr ? y : mr;
                    }
                    int rank = 0;
                    const uint32_t mcls = item_class(endpoint_meta(b, ps[s]));
                    for (int r = 0; r < mr; r++) {  // uniform: every lane shuffles
                        const int j = simple ? st + r : k;
                        const int pl = (j - s * 64) & 63;
                        const uint32_t plen = (uint32_t)__shfl((int)kme.len, pl, 64);
                        const int pid = __shfl(ps[s], pl, 64);
                        const int pfall = __shfl((int)fallback, pl, 64);
                        const uint32_t nbytes = (plen < kme.len ? plen : kme.len) - 16u;
                        int cmpv = 0;  // partner against me
#pragma unroll
                        for (int u = 0; u < kQW; u++) {
                            const uint64_t pw = (uint64_t)__shfl((long long)tw.w[u], pl, 64);
                            const int vb = (int)nbytes - 8 * u;
                            if (cmpv == 0 && vb > 0) {
                                const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
                                const uint64_t x = pw & msk, y = tw.w[u] & msk;
                                if (x != y) cmpv = x < y ? -1 : 1;
                            }
                        }
                        if (simple && j <= en && j != k) {
                            if (pfall) {
                                fallback = true;
                            } else {
                                if (cmpv == 0) cmpv = plen < kme.len ? -1 : (plen > kme.len ? 1 : 0);
                                if (cmpv == 0) {
                                    const uint32_t pc = item_class(endpoint_meta(b, pid));
                                    cmpv = pc < mcls ? -1 : (pc > mcls ? 1 : (pid < ps[s] ? -1 : 1));
                                }
                                rank += cmpv < 0 ? 1 : 0;
                            }
                        }
                    }
                    if (simple && !fallback) {
                        fin[s] = st + rank;
                        todo = false;
                    }
                    if (a.trace && in_run) {
                        atomicAdd(&a.trace[kTrBktRuns], 1ull);
                        if (simple && !fallback) atomicAdd(&a.trace[kTrBktSimple], 1ull);
                        if (todo) atomicAdd(&a.trace[kTrBktSlow], 1ull);
                        atomicMax(&a.trace[kTrBktMaxRun], (unsigned long long)(en - st + 1));
                    }
                    if (!todo) continue;
                    // Runs the register ranking above cannot take (crossing a 64-position slot, longer
                    // than 16, or keys past the tail words held): every partner's key and tail words
                    // are loaded, two partners at a time with all their loads in flight, and compared
                    // against this lane's in registers (C4: ~50 lanes a batch, whose serial loads of
                    // one partner after another set the launch's length).  Keys past the held words
                    // compare whole (item_less_total).
                    const int pm = ps[s];
                    kme = b.keys[pm];
                    QTail tme;
                    load_qtail(tme, kme, b.tail);
                    const bool mlong = kme.len > 16u + 8u * kQW;
                    rank = 0;
                    for (int j0 = st; j0 <= en; j0 += 2) {
                        int po[2];
                        DKey ko[2];
                        QTail tq[2];
#pragma unroll
                        for (int u = 0; u < 2; u++) po[u] = (j0 + u <= en && j0 + u != k) ? s_p[wave][j0 + u] : -1;
#pragma unroll
                        for (int u = 0; u < 2; u++)
                            if (po[u] >= 0) ko[u] = b.keys[po[u]];
#pragma unroll
                        for (int u = 0; u < 2; u++)
                            if (po[u] >= 0) load_qtail(tq[u], ko[u], b.tail);
#pragma unroll
                        for (int u = 0; u < 2; u++) {
                            if (po[u] < 0) continue;
                            if (mlong || ko[u].len > 16u + 8u * kQW) {
                                rank += item_less_total(make_item(b, po[u]), make_item(b, pm), b.tail) ? 1 : 0;
                                continue;
                            }
                            // tied keys share bytes [0, c + 19 > 16): tails from byte 16, then
                            // length, class, endpoint id (item_less_total's order)
                            const uint32_t nbytes = (ko[u].len < kme.len ? ko[u].len : kme.len) - 16u;
                            int cmpv = 0;
#pragma unroll
                            for (int w = 0; w < kQW; w++) {
                                const int vb = (int)nbytes - 8 * w;
                                if (cmpv == 0 && vb > 0) {
                                    const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
                                    const uint64_t x = tq[u].w[w] & msk, y = tme.w[w] & msk;
                                    if (x != y) cmpv = x < y ? -1 : 1;
                                }
                            }
                            if (cmpv == 0) cmpv = ko[u].len < kme.len ? -1 : (ko[u].len > kme.len ? 1 : 0);
                            if (cmpv == 0) {
                                const uint32_t pc = item_class(endpoint_meta(b, po[u]));
                                cmpv = pc < mcls ? -1 : (pc > mcls ? 1 : (po[u] < pm ? -1 : 1));
                            }
                            rank += cmpv < 0 ? 1 : 0;
                        }
                    }
                    fin[s] = st + rank;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int k = s * 64 + lane;
                    if (s < S && k < n) s_p[wave][fin[s]] = ps[s];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int k = s * 64 + lane;
                    if (s < S && k < n) ps[s] = s_p[wave][k];
                }
            }
        }
        if (lane == 0) trace_max(a.trace, kTrBktTies);
        tt[0] = tw0;
        tt[1] = tw1;
        tt[2] = tw2;
    }
    // ---- bucket offsets: the counts of every bucket before B0 and of all buckets (loaded above)
    {
        uint32_t pre[4] = {0, 0, 0, 0}, tot[4] = {0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < kPreLoads; u++) {
            const int k = threadIdx.x + u * kBlock;
            if (u >= kPreHeld && (k >= nb || (a.exp & 8))) continue;
            const uint64_t x0 = u < kPreHeld ? c0[u < kPreHeld ? u : 0] : a.cnt[(size_t)kCntStride * k];
            const uint64_t x1 = u < kPreHeld ? c1[u < kPreHeld ? u : 0] : a.cnt[(size_t)kCntStride * k + 1];
            const uint32_t v[4] = {(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                tot[c] += v[c];
                pre[c] += k < B0 ? v[c] : 0u;
            }
        }
        if (a.exp & 8) {  // cost breakdown: 64 endpoints per bucket
            const uint32_t per[4] = {64, 16, 16, 16};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                pre[c] = threadIdx.x == 0 ? per[c] * (uint32_t)B0 : 0u;
                tot[c] = threadIdx.x == 0 ? per[c] * (uint32_t)nb : 0u;
            }
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                pre[c] += __shfl_xor(pre[c], off, 64);
                tot[c] += __shfl_xor(tot[c], off, 64);
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                s_red[c][wave] = pre[c];
                s_red[4 + c][wave] = tot[c];
            }
            const uint32_t v[4] = {(uint32_t)own0, (uint32_t)(own0 >> 32), (uint32_t)own1, (uint32_t)(own1 >> 32)};
#pragma unroll
            for (int c = 0; c < 4; c++) s_cnt[wave][c] = v[c];
            s_big[wave] = n > kSlab ? 1 : 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run[4] = {0, 0, 0, 0};
            for (int q = 0; q < kWaves; q++)
#pragma unroll
                for (int c = 0; c < 4; c++) run[c] += s_red[c][q];
            for (int q = 0; q < kWaves; q++)
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    s_base[q][c] = run[c];
                    run[c] += s_cnt[q][c];
                }
            if (blockIdx.x == 0) {  // class totals after the last position
                uint32_t t4[4] = {0, 0, 0, 0};
                for (int q = 0; q < kWaves; q++)
#pragma unroll
                    for (int c = 0; c < 4; c++) t4[c] += s_red[4 + c][q];
                o.cwb[E] = (int32_t)t4[1];
                o.crb[E] = (int32_t)t4[2];
                o.cwe[E] = (int32_t)t4[3];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) trace_max(a.trace, kTrBktPrologue);
    }
    if (small) {
        const int64_t base = s_base[wave][0];
        const unsigned long long tw3 = a.trace ? wall_clock64() : 0ull;
        // positions, class counts before them, begin lists; quantiles for the next batch
        uint32_t carry[3] = {s_base[wave][1], s_base[wave][2], s_base[wave][3]};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            if (s >= S) break;
            const int k = s * 64 + lane;
            const bool live = k < n;
            const uint32_t cls = live ? item_class(endpoint_meta(b, ps[s])) : 4u;
            const uint32_t f[3] = {cls == kWriteBegin, cls == kReadBegin, cls == kWriteEnd};
            uint32_t ex[3];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                uint32_t x = f[q];
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t y = __shfl_up(x, off, 64);
                    if (lane >= off) x += y;
                }
                ex[q] = carry[q] + x - f[q];
                carry[q] += __shfl(x, 63, 64);
            }
            if (live && !(a.exp & 2)) {
                put_position(b, o, ps[s], base + k, (int32_t)ex[0], (int32_t)ex[1], (int32_t)ex[2]);
                if (o.quant) put_quantiles(b, o.quant, base + k, E, ps[s]);
            } else if (live && ex[0] == 0x7fffffff) {
                o.pos[0] = 0;
            }
        }
        if (a.trace && lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long tw4 = wall_clock64();
            atomicAdd(&a.trace[kTrBktWaves], 1ull);
            atomicAdd(&a.trace[kTrBktSumLoad], tt[1] - tt[0]);
            atomicAdd(&a.trace[kTrBktSumSort], tt[2] - tt[1]);
            atomicAdd(&a.trace[kTrBktSumTies], tw3 - tt[2]);
            atomicAdd(&a.trace[kTrBktSumPut], tw4 - tw3);
        }
    }
    // ---- buckets past kSlab: ranked by the whole workgroup, one after another
    __syncthreads();
    for (int wv = 0; wv < kWaves; wv++) {
        if (!s_big[wv] || B0 + wv >= nb) continue;  // uniform: LDS after the barrier
        const int bb = B0 + wv;
        const int m = (int)s_cnt[wv][0];
        const int64_t bbase = s_base[wv][0];
        if (threadIdx.x == 0) {
            s_gather = 0;
            atomicAdd(&a.bsc->sort_big, 1);
        }
        for (int i = threadIdx.x; i < kSlab; i += kBlock) o.big[bbase + i] = a.slab[(size_t)bb * kSlab + i];
        __syncthreads();
        const int novf = a.bsc->ovf_n;
        for (int i = threadIdx.x; i < novf; i += kBlock)
            if (a.ovf_b[i] == bb) o.big[bbase + kSlab + atomicAdd(&s_gather, 1)] = a.ovf[i];
        __syncthreads();
        // rank of every endpoint among the bucket's (exact order, tails included)
        for (int i0 = 0; i0 < m; i0 += kBlock) {
            const int i = i0 + threadIdx.x;
            SortItem me{};
            if (i < m) me = o.big[bbase + i];
            int rank = 0;
            for (int j0 = 0; j0 < m; j0 += kBlock) {
                __syncthreads();
                if (j0 + (int)threadIdx.x < m) s_tile[threadIdx.x] = o.big[bbase + j0 + threadIdx.x];
                __syncthreads();
                const int cnt = min(kBlock, m - j0);
                if (i < m)
                    for (int j = 0; j < cnt; j++) rank += item_less_total(s_tile[j], me, b.tail) ? 1 : 0;
            }
            if (i < m) o.big_p[bbase + rank] = (int32_t)(me.meta >> 2);  // ranks are distinct
        }
        __syncthreads();
        uint32_t carry[3] = {s_base[wv][1], s_base[wv][2], s_base[wv][3]};
        for (int k0 = 0; k0 < m; k0 += kBlock) {
            const int k = k0 + threadIdx.x;
            const bool live = k < m;
            const int p = live ? o.big_p[bbase + k] : 0;
            const uint32_t cls = live ? item_class(endpoint_meta(b, p)) : 4u;
            uint32_t ex[3];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const uint32_t f = cls == (q == 0 ? (uint32_t)kWriteBegin : q == 1 ? (uint32_t)kReadBegin
                                                                                     : (uint32_t)kWriteEnd);
                uint32_t total;
                ex[q] = carry[q] + block_excl_sum<uint32_t>(f, &s_red[q][0], &total);
                carry[q] += total;
            }
            if (live) {
                put_position(b, o, p, bbase + k, (int32_t)ex[0], (int32_t)ex[1], (int32_t)ex[2]);
                if (o.quant) put_quantiles(b, o.quant, bbase + k, E, p);
            }
        }
        __syncthreads();
    }
    if (a.trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) trace_max(a.trace, kTrBktEnd);
    }
}

// Cold start: the quantile table from this batch's samples ranked by k_sample (one workgroup).
__global__ __launch_bounds__(kWG) void k_quant_cold(BatchDev b, const SortItem* samples, const int32_t* srank, int S,
                                                    SplitKey* quant) {
    __shared__ int32_t inv[kMaxSample];
    for (int i = threadIdx.x; i < S; i += blockDim.x) inv[srank[i]] = i;
    __syncthreads();
    for (int q = threadIdx.x; q < kQuant; q += blockDim.x) {
        const int r = (int)(((int64_t)(q + 1) * S) / (kQuant + 1));
        quant[q] = make_split(samples[inv[r]], b.tail);
    }
}

int sort_cold_samples(int64_t E, int nb) { return (int)std::min<int64_t>(E, std::min(kMaxSample, std::max(1024, 4 * nb))); }

int sort_bucket_count(int64_t E, int target, int slab_buckets) {
    if (target <= 0) target = kSortTarget;
    int64_t nb = (E + target - 1) / target;
    const int64_t cap = std::min<int64_t>(kSortMaxBuckets, std::max(1, slab_buckets));
    return (int)std::max<int64_t>(1, std::min(nb, cap));
}

static SortArgs sort_args(const Work& w, const SplitKey* quant, int nb, int64_t btail_n, bool long_keys) {
    SortArgs a{w.btail, btail_n, quant, w.scnt, w.slab, w.ovf, w.ovf_b, w.bsc, nb, w.trace};
    a.long_keys = long_keys ? 1 : 0;
    return a;
}

void launch_sort(hipStream_t s, const BatchDev& b, const Work& w, SplitKey* quant, SplitKey* quant_out, bool cold,
                 int bucket_target, bool long_keys, bool validate, hipEvent_t sort_begin, hipEvent_t sort_end) {
    const int E = 2 * (b.R + b.W);
    if (E == 0) return;
    const int nb = sort_bucket_count(E, bucket_target, w.slab_buckets);
    fdb_event(LaunchList::kTimingRecord, sort_begin, s);
    if (cold && nb > 1) {  // splitters from this batch's ranked samples
        SampleRank c{};
        c.S = sort_cold_samples(E, nb);
        c.n_slice = (c.S + kSampleSlice - 1) / kSampleSlice;
        c.srank = w.srank;
        c.samples = w.samples;
        c.trace = w.trace;
        fdb_launch(k_sample, dim3(c.n_slice * ((c.S + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, b, c);
        fdb_launch(k_quant_cold, dim3(1), dim3(kWG), 0, s, b, (const SortItem*)w.samples, (const int32_t*)w.srank,
                   c.S, quant);
    }
    const SortArgs a = sort_args(w, quant, nb, b.tail_n, long_keys);
    fdb_launch(k_sort_partition, dim3((E + kBlock - 1) / kBlock), dim3(kBlock), (uint32_t)(16 * (nb - 1)), s, b, a);
    SortOut o{w.pos, w.pmeta, w.cwb, w.crb, w.cwe, w.wbrange, w.rbrange, validate ? w.items : nullptr,
              quant_out, w.big, w.big_p};
    const int grid = (nb + kBlock / 64 - 1) / (kBlock / 64);
    if (long_keys)
        fdb_launch(k_sort_bucket<true>, dim3(grid), dim3(kBlock), 0, s, b, a, o);
    else
        fdb_launch(k_sort_bucket<false>, dim3(grid), dim3(kBlock), 0, s, b, a, o);
    fdb_event(LaunchList::kTimingRecord, sort_end, s);
}

// Diagnostics (fdbcs_debug_kernel_time, which 1-2): isolated device time of k_sort_partition or
// k_sort_bucket (warm splitters) over `reps` runs of the sort on an idle stream; the zeroed
// scratch is reset before each run, outside the timing.
hipError_t debug_time_sort(hipStream_t s, const BatchDev& b, const Work& w, SplitKey* quant, int bucket_target,
                           bool long_keys, int which, int reps, double* us) {
    const int E = 2 * (b.R + b.W);
    if (E == 0) return hipErrorInvalidValue;
    const int nb = sort_bucket_count(E, bucket_target, w.slab_buckets);
    hipEvent_t e0, e1;
    hipError_t err;
    if ((err = hipEventCreate(&e0)) || (err = hipEventCreate(&e1))) return err;
    SortArgs a = sort_args(w, quant, nb, b.tail_n, long_keys);
    if (const char* v = getenv("FDBCS_SORT_EXP")) a.exp = atoi(v);  // cost breakdown (results unused)
    SortOut o{w.pos, w.pmeta, w.cwb, w.crb, w.cwe, w.wbrange, w.rbrange, nullptr, nullptr, w.big, w.big_p};
    const int grid = (nb + kBlock / 64 - 1) / (kBlock / 64);
    double total = 0;
    for (int r = 0; r < reps && err == hipSuccess; r++) {
        (void)hipMemsetAsync(w.scnt, 0, 8 * kCntStride * (size_t)kSortMaxBuckets, s);
        (void)hipMemsetAsync(&w.bsc->ovf_n, 0, 4, s);
        if (which == 1) (void)hipEventRecord(e0, s);
        fdb_launch(k_sort_partition, dim3((E + kBlock - 1) / kBlock), dim3(kBlock), (uint32_t)(16 * (nb - 1)), s, b, a);
        if (which == 1) (void)hipEventRecord(e1, s);
        if (which == 2) (void)hipEventRecord(e0, s);
        if (long_keys)
            fdb_launch(k_sort_bucket<true>, dim3(grid), dim3(kBlock), 0, s, b, a, o);
        else
            fdb_launch(k_sort_bucket<false>, dim3(grid), dim3(kBlock), 0, s, b, a, o);
        if (which == 2) (void)hipEventRecord(e1, s);
        if ((err = hipEventSynchronize(e1))) break;
        float ms = 0;
        if ((err = hipEventElapsedTime(&ms, e0, e1))) break;
        total += ms;
    }
    (void)hipMemsetAsync(w.scnt, 0, 8 * kCntStride * (size_t)kSortMaxBuckets, s);
    (void)hipMemsetAsync(w.bsc, 0, sizeof(BatchScalars), s);
    (void)hipStreamSynchronize(s);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *us = total * 1000.0 / reps;
    return err;
}

// FDBCS_VALIDATE=1: check the endpoint order and that positions invert the permutation.
__global__ __launch_bounds__(kBlock) void k_validate_sort(const SortItem* sorted, const int32_t* pos,
                                                          const uint32_t* pmeta, int E, const uint8_t* arena,
                                                          BatchScalars* sc) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= E) return;
    bool bad = p > 0 && !item_less_total(sorted[p - 1], sorted[p], arena);
    bad |= sorted[p].meta != pmeta[p];
    const int q = pos[p];  // slot p -> position
    bad |= q < 0 || q >= E || (2 * item_range(pmeta[q]) + item_is_end(pmeta[q])) != (uint32_t)p;
    if (bad) atomicOr(&sc->debug_error, 1);
}

void launch_validate_sort(hipStream_t s, const BatchDev& b, const Work& w) {
    const int E = 2 * (b.R + b.W);
    if (E == 0) return;
    fdb_launch(k_validate_sort, dim3((E + kBlock - 1) / kBlock), dim3(kBlock), 0, s, (const SortItem*)w.items,
               (const int32_t*)w.pos, (const uint32_t*)w.pmeta, E, (const uint8_t*)b.tail, w.bsc);
}

// ------------------------------------------------------------------ D.CheckIntraBatch: candidate edges
//
// Read r of txn t and write w of txn t' < t overlap iff (index space, SkipList.cpp:812-834)
// wb < re and rb < we with both intervals non-empty.  Either w begins inside (rb, re)
// (found from the read) or r begins inside (wb, we) (found from the write).  Each such
// pair is one candidate edge t' -> t: t aborts iff some candidate writer commits.

//
// Every (range, candidate) pair is enumerated in parallel, so a hot key written by hundreds of
// transactions and read by thousands (Zipf, C3) costs no serial per-range loop:
//   * read r owns the write-begins inside (rb, re): wbrange[cwb[rb] .. cwb[re]) ("a" pairs);
//   * write w owns the read-begins inside (wb, we): rbrange[crb[wb] .. crb[we]) ("b" pairs).
// Read r owns eoff[r+1] - eoff[r] slots: its a pairs plus one per write covering rb, a count that
// is #(write-begins before rb) - #(write-ends before rb), known without enumerating (an empty write
// has its end before its begin and no read-begin between them, so it counts 0).  Only pairs that
// pass the filter (earlier writer, both ranges non-empty) take a slot, so read r's edges are
// edges[eoff[r] .. eoff[r] + ecur[r]).

__device__ __forceinline__ bool range_nonempty(const Work& w, int g) { return w.pos[2 * g] < w.pos[2 * g + 1]; }

// Per range g: slots (reads only) and pairs; exclusive prefixes give each read's first slot and
// each range's first pair.
// The read-begins a write contains, as an interval of read-begin indices (empty: none).
__device__ __forceinline__ uint2 write_rb_interval(const Work& w, int g) {
    const int b = w.pos[2 * g], e = w.pos[2 * g + 1];
    if (b >= e) return make_uint2(0, 0);
    const int lo = w.crb[b], hi = w.crb[e];
    return hi > lo ? make_uint2((uint32_t)lo, (uint32_t)hi) : make_uint2(0, 0);
}

// Elements per thread of the scans whose visits are chains of dependent gathers (scan.h): one,
// so every chain has its own lane and the small batch-sized scans still span many workgroups.
constexpr int kEdgeScanP = 1;
constexpr int kCombineP = 1;
constexpr int kCombineTile = kScanThreads * kCombineP;
constexpr int kRouteScanP = 1;

struct EdgePairScan {
    Work w;
    int32_t R, G;
    const int32_t* wowner;
    const DKey* keys;
    const int32_t* rowner;
    int32_t T;
    __device__ void counts(int64_t g, uint32_t& slots, uint32_t& pairs, uint32_t& a) const {
        slots = pairs = a = 0;
        if (g >= R) {
            // the write's two entries in the sorted list of write endpoints (index = write
            // endpoints before its position), read by D.Combine at the end of k_resolve
            const int pb = w.pos[2 * g], pe = w.pos[2 * g + 1];
            const int code = pb < pe ? 2 * wowner[g - R] : -1;
            const int ib = w.cwb[pb] + w.cwe[pb], ie = w.cwb[pe] + w.cwe[pe];
            w.wends[ib] = make_int2(pb, code);
            w.wends[ie] = make_int2(pe, code < 0 ? -1 : code + 1);
            w.wkeys[ib] = keys[2 * g];
            w.wkeys[ie] = keys[2 * g + 1];
        }
        if (g >= R && w.groups) {
            // write-begin index j of this write; it leads a group unless the write before it in
            // sorted order contains the same read-begins (then that group's edges cover it)
            const int j = w.cwb[w.pos[2 * g]];
            const uint2 iv = write_rb_interval(w, (int)g);
            int lead = 0;
            if (iv.y > iv.x) {
                lead = 2;
                if (j > 0) {
                    const int gp = w.wbrange[j - 1];
                    const uint2 ip = write_rb_interval(w, gp);
                    if (ip.x == iv.x && ip.y == iv.y) lead = 1;
                }
            }
            w.wlead[j] = lead;
            w.wtxn[j] = wowner[g - R];
            if (lead == 2) pairs = iv.y - iv.x;
            return;
        }
        if (!range_nonempty(w, (int)g)) return;
        const int b = w.pos[2 * g], e = w.pos[2 * g + 1];
        if (g < R) {
            a = (uint32_t)(w.cwb[e] - w.cwb[b]);
            const int cover = w.cwb[b] - w.cwe[b];  // < 0 only with an inverted write (invalid input)
            slots = a + (uint32_t)(cover > 0 ? cover : 0);
            pairs = a;
        } else {
            pairs = (uint32_t)(w.crb[e] - w.crb[b]);
        }
    }
    static constexpr bool kOwn = true;
    // counts: edge slots, candidate pairs, has pairs (the compacted index k_edge_fill searches)
    __device__ void load(int64_t g, uint32_t (&v)[3]) const {
        uint32_t a;
        counts(g, v[0], v[1], a);
        v[2] = v[1] > 0 ? 1u : 0u;
    }
    __device__ void store(int64_t g, const uint32_t (&ex)[3], const uint32_t (&own)[3]) const {
        if (g < R) w.eoff[g] = (int32_t)ex[0];
        w.poff[g] = (int32_t)ex[1];
        if (own[2]) {
            w.pcg[ex[2]] = (int32_t)g;
            w.pcoff[ex[2]] = (int32_t)ex[1];
            // k_edge_fill's per-range operands (its staging then takes one load, not three): the
            // base of the partner list (cwb / crb at the range's begin) and the range's side of the
            // edge test (the read's owner; the write's owner, or its group's edge T + j)
            const int p0 = w.pos[2 * g];
            if (g < R) {
                w.pcbase[ex[2]] = w.cwb[p0];
                w.pca[ex[2]] = rowner[g];
            } else {
                w.pcbase[ex[2]] = w.crb[p0];
                w.pca[ex[2]] = w.groups ? T + w.cwb[p0] : wowner[g - R];
            }
        }
    }
    __device__ void finish(const uint32_t (&tot)[3]) const {
        w.eoff[R] = (int32_t)tot[0];
        w.poff[G] = (int32_t)tot[1];
        w.pcg[tot[2]] = G;
        w.pcoff[tot[2]] = (int32_t)tot[1];
        w.bsc->n_pranges = tot[2];
        w.bsc->n_edges = tot[0];
        w.bsc->edge_overflow = (int64_t)tot[0] > w.edge_cap || tot[0] > 0x7fffffffu || tot[1] > 0x7fffffffu ? 1 : 0;
        // to the host (mapped memory): does this batch have candidate edges?  Read once the
        // batch's stage A event completed, tagged with the batch's sequence number
        if (w.hedge) {
            w.hedge[1] = tot[0] != 0 ? 1u : 0u;
            __threadfence_system();
            w.hedge[0] = w.hseq;
        }
    }
};

constexpr int kPairsPerThread = 4;
constexpr int kFillPairs = kBlock * kPairsPerThread;  // pairs per workgroup step of k_edge_fill

// Last index c in [lo, hi) with a[c] <= x, given a[lo] <= x < a[hi] (a non-decreasing), by one
// whole wave: 64 probes per step, so ~3 dependent loads for 10^5 entries instead of ~17.
__device__ __forceinline__ int wave_last_le(const int32_t* a, int lo, int hi, int x) {
    const int lane = threadIdx.x & 63;
    while (hi - lo > 1) {
        const int idx = lo + 1 + (int)(((int64_t)lane * (hi - lo - 1)) / 64);  // inside (lo, hi)
        const uint64_t le = __ballot(a[idx] <= x);  // a prefix of the lanes
        const int c = __popcll(le);
        const int nlo = c > 0 ? __shfl(idx, c - 1, 64) : lo;
        const int nhi = c < 64 ? __shfl(idx, c, 64) : hi;
        lo = nlo;
        hi = nhi;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void k_edge_fill(BatchDev b, Work w) {
    // per compacted range of the step: first pair, range id, the base of its partner list
    // (cwb / crb at its begin) and its side of the edge test (the read's owner, or the write's
    // edge target), staged once so each pair's chain starts at the partner list
    __shared__ int32_t s_off[kFillPairs + 2], s_g[kFillPairs + 1], s_b[kFillPairs + 1], s_a[kFillPairs + 1];
    __shared__ int s_c[2];
    if (w.bsc->edge_overflow) return;
    const int R = b.R;
    const int M = (int)w.bsc->n_pranges;  // ranges with pairs: pcg / pcoff[0, M), pcoff[M] = P
    const int P = w.pcoff[M];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    for (int Q0 = blockIdx.x * kFillPairs; Q0 < P; Q0 += gridDim.x * kFillPairs) {
        // the compacted ranges holding this step's first and last pair (each range there has at
        // least one pair, so at most kFillPairs of them), found by waves 0 and 1 side by side,
        // then their first pairs and range ids staged in LDS
        const int Q1 = min(P, Q0 + kFillPairs) - 1;
        if (wave < 2) {
            const int c = wave_last_le(w.pcoff, 0, M, wave == 0 ? Q0 : Q1);
            if (lane == 0) s_c[wave] = c;
        }
        __syncthreads();
        const int c0 = s_c[0], nc = s_c[1] - s_c[0] + 1;
        for (int i = threadIdx.x; i <= nc; i += blockDim.x) {
            s_off[i] = w.pcoff[c0 + i];
            if (i < nc) {
                // read gg: its k-th write-begin's range is wbrange[base + k]; write gg: its k-th
                // read-begin's range is rbrange[base + k].  A write leading a group gets one edge
                // T + j for the group (its members' transactions are compared with the reader's
                // in the resolution rounds).  (EdgePairScan::store)
                s_g[i] = w.pcg[c0 + i];
                s_b[i] = w.pcbase[c0 + i];
                s_a[i] = w.pca[c0 + i];
            }
        }
        __syncthreads();
        // each dependent step of the pair filter for the thread's four pairs at once: four chains
        // of gathers in flight per thread instead of one after another (C3: 1.85M pairs per batch)
        int gq[kPairsPerThread], part[kPairsPerThread], aq[kPairsPerThread];
#pragma unroll
        for (int u = 0; u < kPairsPerThread; u++) {
            const int q = Q0 + threadIdx.x * kPairsPerThread + u;
            gq[u] = -1;
            part[u] = aq[u] = 0;
            if (q >= P) continue;
            int lo = 0, hi = nc;  // s_off[lo] <= q < s_off[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_off[mid] <= q) lo = mid; else hi = mid;
            }
            const int gg = s_g[lo];
            gq[u] = gg;
            aq[u] = s_a[lo];
            // partner range: read g's k-th write-begin inside it, or write g's k-th read-begin
            part[u] = (gg < R ? w.wbrange : w.rbrange)[s_b[lo] + q - s_off[lo]];
        }
        int rd[kPairsPerThread], tw[kPairsPerThread];
        bool ok[kPairsPerThread];
#pragma unroll
        for (int u = 0; u < kPairsPerThread; u++) {
            const int gg = gq[u];
            ok[u] = false;
            rd[u] = tw[u] = 0;
            if (gg < 0) continue;
            const int other = part[u];
            const bool ne = range_nonempty(w, other);  // the pair's own range is: it has pairs
            if (gg < R) {  // read gg, write other: an earlier writer
                rd[u] = gg;
                tw[u] = b.wowner[other - R];
                ok[u] = tw[u] < aq[u] && ne;
            } else {       // write gg, read other
                rd[u] = other;
                tw[u] = aq[u];
                ok[u] = ne && (w.groups || aq[u] < b.rowner[other]);
            }
        }
        // edge slots: one atomic per run of lanes filing under the same read (a read's own pairs
        // are consecutive, so its lanes form one run per wave instead of one atomic each)
#pragma unroll
        for (int u = 0; u < kPairsPerThread; u++) {
            const int key = ok[u] ? rd[u] : -1;
            const int prev = __shfl_up(key, 1, 64);
            const bool head = ok[u] && (lane == 0 || prev != key);
            const uint64_t hm = __ballot(head), om = __ballot(ok[u]);
            const uint64_t brk = (hm | ~om) & ~((2ull << lane) - 1);  // run breaks above this lane
            const int start = ok[u] ? 63 - __builtin_clzll(hm & ((2ull << lane) - 1)) : lane;
            int base = 0;
            if (head) base = atomicAdd(&w.ecur[key], (brk ? __builtin_ctzll(brk) : 64) - lane);
            base = __shfl(base, start, 64);
            if (ok[u]) {
                const int slot = w.eoff[key] + base + lane - start;
                if (slot < w.eoff[key + 1]) w.edges[slot] = tw[u];
            }
        }
        __syncthreads();  // the next step restages s_c / s_off / s_g
    }
}

void launch_edges(hipStream_t s, const BatchDev& b, const Work& w) {
    const int G = b.R + b.W;
    launch_scan<3, kEdgeScanP>(s, EdgePairScan{w, b.R, G, b.wowner, b.keys, b.rowner, b.T}, nullptr, G, w.scan[kScanEdges]);
    if (G) {
        const int blocks = G / 16 < 64 ? 64 : (G / 16 > 4096 ? 4096 : G / 16);
        fdb_launch(k_edge_fill, dim3(blocks), dim3(kBlock), 0, s, b, w);
    }
}

// ------------------------------------------------------------------ D.CheckIntraBatch: resolution
//
// Batch order (SkipList.cpp:817-833): commit(t) = !hist(t) && !tooOld(t) && no earlier committed
// candidate writer.  Rounds in one workgroup: an undecided t commits once every candidate writer
// is aborted and aborts as soon as one commits; the lowest undecided t always decides, so the
// rounds terminate.  If the candidate edges overflowed, the workgroup replays MiniConflictSet
// sequentially over point indices instead (exact, slower).

// vout: the batch's host-mapped verdict bytes (ConflictSet.h:40-44 encoding), written here as soon
// as each status is final so the epilogue only publishes scalars and the completion flag.
__device__ __forceinline__ uint8_t verdict_byte(const BatchDev& b, int t, uint8_t status) {
    if (b.flags[t] & kFlagTooOld) return 1;  // TransactionTooOld
    return status == kCommitted ? 2 : 0;     // TransactionCommitted : TransactionConflict
}

// D.Combine (combineWriteConflictRanges, SkipList.cpp:926-939): +1 at the begin and -1 at the end
// of every committed non-empty write, summed over the write endpoints in sorted order (wends, from
// stage A), gives the coverage before each; a union segment [key(begin), key(end)) starts where
// coverage leaves 0 and ends where it returns (CoverScan / SegNumScan below).
__global__ void k_set_i64(int64_t* p, int64_t v) {
    if (threadIdx.x == 0) *p = v;
}


// D.Combine across the pre-pass workgroups when no transaction has a candidate writer (a
// transaction commits iff it has no history conflict and is not TooOld, so every status is known
// from the check's flags): the coverage of committed writes over the sorted write endpoints by one
// look-back scan, the union segments numbered by a second one chained in the same tile (k_scan2's
// scheme), instead of one workgroup walking all 2W endpoints after the statuses.
struct CoverScan {
    Work w;
    BatchDev b;
    int use_status;  // 1: the resolution's final statuses (candidate edges existed); 0: the check's flags
    __device__ int delta(int64_t i) const {
        const int2 e = w.wends[i];
        if (e.y < 0) return 0;
        const int t = e.y >> 1;
        const bool committed = use_status ? w.status[t] == kCommitted
                                          : (!w.hist_conf[t] && !(b.flags[t] & kFlagTooOld));
        return committed ? ((e.y & 1) ? -1 : 1) : 0;
    }
    __device__ void load(int64_t i, uint32_t (&v)[1]) const { v[0] = (uint32_t)delta(i); }
    __device__ void store(int64_t i, const uint32_t (&ex)[1]) const {
        const int d = delta(i), c = (int)ex[0];  // coverage before endpoint i
        w.cflag[i] = (d == 1 && c == 0) ? 1 : ((d == -1 && c == 1) ? 2 : 0);
    }
    __device__ void finish(const uint32_t (&)[1]) const {}
};
struct SegNumScan {
    Work w;
    __device__ void load(int64_t i, uint32_t (&v)[1]) const { v[0] = w.cflag[i] == 1 ? 1u : 0u; }
    __device__ void store(int64_t i, const uint32_t (&ex)[1]) const {
        const uint8_t f = w.cflag[i];
        if (!f) return;
        const int x = w.wends[i].x;
        if (f == 1) {  // segment ex opens here
            w.seg_b[ex[0]] = x;
            w.segk[2 * ex[0]] = w.wkeys[i];
        } else {       // the segment opened last (ex - 1) closes here
            w.seg_e[ex[0] - 1] = x;
            w.segk[2 * ex[0] - 1] = w.wkeys[i];
        }
    }
    __device__ void finish(const uint32_t (&tot)[1]) const { w.bsc->n_segments = tot[0]; }
};

// Pre-pass of the resolution, one wave per transaction across the chip (k_resolve_pre), then the
// batch-order rounds and D.Combine in one workgroup (k_resolve).  Two launches: the rounds keep the
// status bytes, group minima and members in up to 159 KiB of LDS, and a single kernel would ask
// that of every pre-pass workgroup too (one per CU, blocked by whatever else holds LDS there).
__global__ __launch_bounds__(kBlock) void k_resolve_pre(BatchDev b, Work w, uint8_t* vout) {
    const BatchScalars* sc = w.bsc;
    const int T = b.T;
    if (blockIdx.x == 0 && threadIdx.x == 0) trace_min(w.trace, kTrResBegin);
    if (sc->n_edges == 0 && !sc->edge_overflow) {
        // no candidate writer anywhere: every admitted transaction without a history conflict
        // commits (SkipList.cpp:817-833 with an empty MiniConflictSet).  No rounds (k_resolve, which
        // a replay may leave out, would set the same).
        if (blockIdx.x == 0 && threadIdx.x == 0) w.bsc->rounds = 0;
        for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < T; t += gridDim.x * blockDim.x) {
            const uint8_t st = (w.hist_conf[t] || (b.flags[t] & kFlagTooOld)) ? kAborted : kCommitted;
            w.status[t] = st;
            w.first_conf[t] = INT_MAX;
            vout[t] = verdict_byte(b, t, st);
            if (w.vdev) w.vdev[t] = vout[t];
        }
        // D.Combine: tiles of kCombineTile write endpoints, ids in launch order.  Only the first
        // ntiles workgroups take an id: the grid is sized for the waves of the edge case, and
        // every id taken is one more atomic on the same counter word
        __shared__ uint32_t sv[1][scan_pad(kCombineP)];
        __shared__ uint32_t swave[1][kScanThreads / 64];
        __shared__ uint32_t sbase[1];
        __shared__ int s_tile;
        const int64_t n = 2 * (int64_t)b.W;
        const int64_t ntiles = n > 0 ? (n + kCombineTile - 1) / kCombineTile : 1;
        if (blockIdx.x >= ntiles) {
            if (threadIdx.x == 0) trace_max(w.trace, kTrResPre);
            return;
        }
        if (threadIdx.x == 0) s_tile = atomicAdd(w.scan[kScanCover].counter, 1);
        __syncthreads();
        if (s_tile < ntiles) {
            scan_tile<1, CoverScan, kCombineP>(CoverScan{w, b, 0}, n, s_tile, ntiles, w.scan[kScanCover], sv, swave,
                                               sbase);
            scan_tile<1, SegNumScan, kCombineP>(SegNumScan{w}, n, s_tile, ntiles, w.scan[kScanSegNum], sv, swave,
                                                sbase);
        }
        if (threadIdx.x == 0) trace_max(w.trace, kTrResPre);
        return;
    }
    if (sc->edge_overflow || w.no_prepass) return;
    // The write groups' members packed for k_resolve (one word per write-begin index): members
    // the pre-pass knows aborted (history conflict or TooOld) never count in a group's minima and
    // carry only their lead bits.
    if (w.groups) {
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < b.W; j += gridDim.x * blockDim.x) {
            const uint32_t lead = (uint32_t)w.wlead[j];
            const int tx = w.wtxn[j];
            const bool dead = lead == 0 || w.hist_conf[tx] || (b.flags[tx] & kFlagTooOld);
            w.wpk[j] = lead << 30 | (dead ? 0u : (uint32_t)tx + 1u);
        }
    }
    // Skip the candidate writers already known aborted (history conflict or TooOld), 64 edges per
    // step with one ballot, and commit the transactions left with none; the rest keep a resume
    // pointer at their first writer not known aborted.  These are exactly the decisions round one
    // would make, but a hot key's reader (hundreds of aborted writers, C3) costs a few ballots
    // instead of a serial walk, and every transaction's chain of dependent loads runs on its own
    // wave across the chip.
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * (blockDim.x >> 6);
    for (int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < T; t += nwaves) {
        uint8_t s0 = (w.hist_conf[t] || (b.flags[t] & kFlagTooOld)) ? kAborted : kUndecided;
        const int r0 = b.roff[t], r1 = b.roff[t + 1];
        // t's slots are contiguous over its reads: its live writers are packed at their start
        const int tbase = r0 < r1 ? w.eoff[r0] : 0;
        int cnt = 0;
        int first[4] = {-1, -1, -1, -1};  // t's first four live writers (uniform over the wave)
        if (s0 == kUndecided) {
            // t's reads 64 at a time, their edge runs flattened into one index space so the loads
            // of every read's edges go out together (per-read chains no longer add up); 256 edges
            // per step: four 64-edge loads, then their writers' flags
            for (int rb = r0; rb < r1; rb += 64) {
                const int nr = min(64, r1 - rb);
                const int myq = lane < nr ? w.eoff[rb + lane] : 0;
                const int myn = lane < nr ? w.ecur[rb + lane] : 0;
                int incl = myn;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += y;
                }
                const int excl = incl - myn;  // lanes >= nr hold the total
                const int total = __shfl(incl, 63, 64);
                for (int f0 = 0; f0 < total; f0 += 4 * 64) {
                    int e[4];
                    bool live[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int f = f0 + 64 * u + lane;
                        const int fc = f < total ? f : total - 1;
                        // the read holding flattened edge fc: the last lane with excl <= fc (binary
                        // lifting, every lane shuffling in step)
                        int lo = 0;
#pragma unroll
                        for (int step = 32; step > 0; step >>= 1) {
                            const int cand = lo + step;
                            const int ex = __shfl(excl, cand < 64 ? cand : 63, 64);
                            if (cand < 64 && ex <= fc) lo = cand;
                        }
                        const int q = __shfl(myq, lo, 64) + fc - __shfl(excl, lo, 64);
                        e[u] = f < total ? w.edges[q] : -1;
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const bool in = (unsigned)e[u] < (unsigned)T;
                        const int ee = in ? e[u] : 0;
                        const uint8_t hc = w.hist_conf[ee], fl = b.flags[ee];
                        live[u] = in ? (!hc && !(fl & kFlagTooOld)) : e[u] >= T;  // group edges stay
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        uint64_t m = __ballot(live[u]);
                        if (live[u]) w.tedges[tbase + cnt + __popcll(m & ((1ull << lane) - 1))] = e[u];
                        for (int j = cnt; j < 4 && m; j++) {  // the first ones, by shuffles
                            first[j] = __shfl(e[u], __ffsll((unsigned long long)m) - 1, 64);
                            m &= m - 1;
                        }
                        cnt += __popcll(__ballot(live[u]));
                    }
                }
            }
            if (cnt == 0) s0 = kCommitted;
        }
        if (lane == 0) {
            w.pre_st[t] = s0;
            w.pre_ep[t] = tbase;
            w.pre_end[t] = tbase + cnt;
            w.first_conf[t] = INT_MAX;  // (k_resolve's reports)
            if (s0 != kUndecided) {  // final: k_resolve's register rounds see only the undecided
                w.status[t] = s0;
                vout[t] = verdict_byte(b, t, s0);
                if (w.vdev) w.vdev[t] = verdict_byte(b, t, s0);
            } else {
                const int u = atomicAdd(&w.bsc->n_undec, 1);
                w.ulist[2 * u] = make_int4(t, tbase, tbase + cnt, 0);
                w.ulist[2 * u + 1] = make_int4(first[0], first[1], first[2], first[3]);
            }
        }
    }
    if (threadIdx.x == 0) trace_max(w.trace, kTrResPre);
}

// TPER: transactions per thread held in registers on the register path (T <= TPER * kWG); two
// instantiations so the common batch sizes keep every register-resident value without spills.
template <int TPER>
__global__ __launch_bounds__(kWG) void k_resolve(BatchDev b, Work w, uint8_t* vout, Scalars* hs) {
    const unsigned long long t_start = wall_clock64();
    if ((threadIdx.x & 63) == 0 && w.trace) {
        atomicMin(&w.trace[kTrResW0min], t_start);
        atomicMax(&w.trace[kTrResW0max], t_start);
    }
    BatchScalars* sc = w.bsc;
    extern __shared__ __attribute__((aligned(16))) uint8_t st[];
    __shared__ int s_more;
    const int T = b.T;
    if (threadIdx.x == 0) trace_max(w.trace, kTrResWait);
    constexpr int kTPer = TPER;
    // One workgroup pays ~2 us per dependent round trip to data another XCD's kernel wrote, and its
    // loads are bounded by one CU's outstanding misses: the rounds load as little as possible, in
    // two round trips.  First: the edge counters, the number of transactions the pre-pass left
    // undecided, every status byte (four per load) and this thread's packed group members.
    const int64_t n_edges = sc->n_edges;
    const int32_t overflow = sc->edge_overflow;
    const int U = w.no_prepass ? 0 : sc->n_undec;
    const int NW = w.groups ? b.W : 0;
    constexpr int kPer = (kMaxGroupWrites + kWG - 1) / kWG;
    const int per = (NW + blockDim.x - 1) / blockDim.x, x0 = threadIdx.x * per;
    uint32_t pk[kPer];  // lead << 30 | transaction + 1 (0: none, or known aborted)
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const bool in = k < per && x0 + k < NW;
        pk[k] = !in ? 0u
                : !w.no_prepass ? w.wpk[x0 + k]
                                : (uint32_t)w.wlead[x0 + k] << 30 | ((uint32_t)w.wtxn[x0 + k] + 1u);
    }
    const int nsw = (T + 3) / 4;  // status words
    const uint32_t* pre_w = (const uint32_t*)w.pre_st;
    uint32_t sw[4];
    if (!w.no_prepass) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = threadIdx.x + u * blockDim.x;
            sw[u] = i < nsw ? pre_w[i] : 0u;
        }
    }
    if (n_edges == 0 && !overflow) {  // k_resolve_pre decided everything and combined
        if (threadIdx.x == 0) {
            sc->rounds = 0;
            trace_max(w.trace, kTrResEnd);
        }
        return;
    }
    const bool use_pre = !overflow && !w.no_prepass;
    const bool in_regs = use_pre && U <= kTPer * (int)blockDim.x;
    // Second: this thread's undecided transactions (the pre-pass's list): transaction, resume
    // pointer, end and its first four live writers.  The rounds see only them; every other
    // transaction's verdict is final and already written by the pre-pass.
    int tt[kTPer], ep[kTPer], en[kTPer], cur[kTPer];
    int4 f4[kTPer];
    if (in_regs) {
#pragma unroll
        for (int k = 0; k < kTPer; k++) {
            const int i = threadIdx.x + k * blockDim.x;
            int4 r = make_int4(-1, 0, 0, 0);
            f4[k] = make_int4(-1, -1, -1, -1);
            if (i < U) {
                r = w.ulist[2 * i];
                f4[k] = w.ulist[2 * i + 1];
            }
            tt[k] = r.x;
            ep[k] = r.y;
            en[k] = r.z;
        }
    }
    // the status bytes into LDS: the pre-pass's (in words), or from the flags without a pre-pass
    if (use_pre) {
        uint32_t* stw = (uint32_t*)st;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = threadIdx.x + u * blockDim.x;
            if (i < nsw) stw[i] = sw[u];
        }
        for (int i = threadIdx.x + 4 * blockDim.x; i < nsw; i += blockDim.x) stw[i] = pre_w[i];  // T > 16K
    } else {
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            st[t] = (w.hist_conf[t] || (b.flags[t] & kFlagTooOld)) ? kAborted : kUndecided;
            w.first_conf[t] = INT_MAX;
        }
    }
    int ep0[kTPer];
#pragma unroll
    for (int k = 0; k < kTPer; k++) {
        ep0[k] = ep[k];
        cur[k] = in_regs && ep[k] < en[k] ? f4[k].x : -1;
    }
    __syncthreads();
    int rounds = 0;
    // write groups: per group j (its first write-begin index), the least transaction among its
    // members not aborted (minLive) and among its committed members (minComm), recomputed from the
    // statuses at the start of every round, in LDS after the status bytes
    int32_t* minLive = (int32_t*)(st + ((T + 15) & ~15));
    int32_t* minComm = minLive + NW;
    __shared__ int s_wred[kWG / 64];
    // The group members stay in registers for the whole launch: each thread holds the members
    // among its contiguous run of <= kPer write-begin indices (W <= kMaxGroupWrites), as
    // (transaction, group = nearest group start at or before it); members the pre-pass knows
    // aborted never count and are left out.
    static_assert(kMaxTxnLds <= 65536 && kMaxGroupWrites < 65535, "member packing");
    uint32_t mem[kPer];  // transaction | group << 16; group 0xffff: none
#pragma unroll
    for (int k = 0; k < kPer; k++) mem[k] = 0xffff0000u;
    // A thread's members of one group are consecutive: each run is min-reduced in registers and
    // takes one pair of LDS atomics (a hot key's writers fill whole runs of one group).
    auto group_minima = [&](const volatile uint8_t* sv) {
        for (int j = threadIdx.x; j < NW; j += blockDim.x) minLive[j] = minComm[j] = INT_MAX;
        uint8_t sx[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) sx[k] = (mem[k] >> 16) != 0xffffu ? sv[mem[k] & 0xffffu] : kAborted;
        __syncthreads();
        int g = -1, lv = INT_MAX, cm = INT_MAX;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int mg = (int)(mem[k] >> 16), mt = (int)(mem[k] & 0xffffu);
            if (mg == 0xffff) continue;
            if (mg != g) {
                if (g >= 0) {
                    if (lv != INT_MAX) atomicMin(&minLive[g], lv);
                    if (cm != INT_MAX) atomicMin(&minComm[g], cm);
                }
                g = mg;
                lv = cm = INT_MAX;
            }
            if (sx[k] != kAborted) lv = mt < lv ? mt : lv;
            if (sx[k] == kCommitted) cm = mt < cm ? mt : cm;
        }
        if (g >= 0) {
            if (lv != INT_MAX) atomicMin(&minLive[g], lv);
            if (cm != INT_MAX) atomicMin(&minComm[g], cm);
        }
        __syncthreads();
    };
    if (NW && !overflow) {
        // a block max-scan carries the group start into each thread's run
        int last = -1;
#pragma unroll
        for (int k = 0; k < kPer; k++)
            if ((pk[k] >> 30) == 2u) last = x0 + k;
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        int v = last;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(v, o, 64);
            if (lane >= o) v = y > v ? y : v;
        }
        if (lane == 63) s_wred[wid] = v;
        __syncthreads();
        int carry = -1;
        for (int q = 0; q < wid; q++) carry = s_wred[q] > carry ? s_wred[q] : carry;
        const int prev_in_wave = __shfl_up(v, 1, 64);
        if (lane > 0) carry = prev_in_wave > carry ? prev_in_wave : carry;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t lead = pk[k] >> 30, txp = pk[k] & 0x3fffffffu;
            if (lead == 2u) carry = x0 + k;
            if (lead != 0u && txp != 0u) mem[k] = (txp - 1u) | (uint32_t)carry << 16;
        }
    }
    // the group rule for reader t and group edge e = T + j: a committed member before t aborts t,
    // an undecided one before t makes it wait, otherwise the group is no obstacle
    auto group_status = [&](int e, int t) -> uint8_t {
        const int j = e - T;
        if (minComm[j] < t) return kCommitted;
        if (minLive[j] < t) return kUndecided;
        return kAborted;
    };
    __syncthreads();
    if (threadIdx.x == 0) trace_max(w.trace, kTrResSetup);
    if (in_regs) {
        // Rounds with each thread's transactions' resume pointers and current writers in
        // registers: a round reads only LDS unless a walk steps past writers aborted since (the
        // rare case), so the rounds run at LDS and barrier speed.
        volatile uint8_t* vst = st;
        // "more" flags of alternate rounds: round r's is set during r and read after its closing
        // barrier; the other one, read last after round r-1's closing barrier, is reset during r
        // (past at least one barrier since that read), so a round needs two barriers, not three
        __shared__ int s_more2[2];
        if (threadIdx.x == 0) s_more2[0] = s_more2[1] = 0;
        __syncthreads();
        for (;;) {
            // a barrier between the last round's reads of its "more" flag and the reset below:
            // group_minima ends with one
            if (NW)
                group_minima(vst);
            else
                __syncthreads();
            if (rounds == 0 && threadIdx.x == 0) trace_max(w.trace, kTrResMin1);
            if (threadIdx.x == 0) s_more2[(rounds + 1) & 1] = 0;
            int more = 0;
#pragma unroll
            for (int k = 0; k < kTPer; k++) {
                const int t = tt[k];
                if (t < 0 || vst[t] != kUndecided) continue;
                int p = ep[k];
                const int end = en[k];
                uint8_t res = kUndecided;
                int e = cur[k];
                while (p < end) {
                    const uint8_t sp = e >= T ? group_status(e, t) : vst[e];
                    if (sp != kAborted) {
                        if (sp == kCommitted) res = kAborted;
                        break;
                    }
                    // e aborted since: the next four writers, their loads issued together (one
                    // global round trip per four writers aborted in earlier rounds, not per writer)
                    int nx[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int q = p + 1 + u, d = q - ep0[k];  // d < 4: held in f4
                        nx[u] = q >= end ? 0
                                : d < 4  ? (d == 0 ? f4[k].x : d == 1 ? f4[k].y : d == 2 ? f4[k].z : f4[k].w)
                                         : w.tedges[q];
                    }
                    int adv = 0, ne = 0;
                    bool stop = false;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (!stop && p + 1 + u < end) {
                            const int x = nx[u];
                            if ((x >= T ? group_status(x, t) : vst[x]) != kAborted) {
                                stop = true;
                                ne = x;
                            } else {
                                adv++;
                            }
                        }
                    }
                    p += 1 + adv;
                    if (p < end) e = stop ? ne : (p - ep0[k] < 4 ? f4[k].w : w.tedges[p]);
                }
                if (p == end) res = kCommitted;
                ep[k] = p;
                cur[k] = e;
                if (res != kUndecided)
                    vst[t] = res;
                else
                    more = 1;
            }
            if (more) s_more2[rounds & 1] = 1;
            __syncthreads();
            if (rounds == 0 && threadIdx.x == 0) trace_max(w.trace, kTrResRound1);
            const int again = s_more2[rounds & 1];
            rounds++;
            if (!again) break;
        }
    } else if (!overflow) {
        for (int t = threadIdx.x; t < T; t += blockDim.x)
            w.eptr[t] = use_pre ? w.pre_ep[t] : (b.roff[t] < b.roff[t + 1] ? w.eoff[b.roff[t]] : 0);
        volatile uint8_t* vst = st;
        for (;;) {
            if (threadIdx.x == 0) s_more = 0;
            if (NW) group_minima(vst);
            __syncthreads();
            int more = 0;
            for (int t = threadIdx.x; t < T; t += blockDim.x) {
                if (vst[t] != kUndecided) continue;
                // resume at edge p: skip aborted writers, stop at the first undecided or committed
                int p = w.eptr[t];
                uint8_t res = kUndecided;
                if (use_pre) {
                    // the pre-pass packed t's writers not known aborted: one contiguous list
                    const int end = w.pre_end[t];
                    while (p < end) {
                        const int e = w.tedges[p];
                        const uint8_t sp = e >= T ? group_status(e, t) : vst[e];
                        if (sp == kAborted) {
                            p++;
                            continue;
                        }
                        if (sp == kCommitted) res = kAborted;
                        break;
                    }
                    if (p == end) res = kCommitted;
                    w.eptr[t] = p;
                    if (res != kUndecided)
                        vst[t] = res;
                    else
                        more = 1;
                    continue;
                }
                int r = b.roff[t];
                const int rend = b.roff[t + 1];
                for (; r < rend; r++) {
                    const int s0 = w.eoff[r], s1 = s0 + w.ecur[r];
                    if (p < s0) p = s0;
                    // four edges per step, loads issued together: a hot key's reader skips hundreds
                    // of aborted writers
                    while (p < s1) {
                        int e[4];
#pragma unroll
                        for (int u = 0; u < 4; u++) e[u] = p + u < s1 ? w.edges[p + u] : -1;
                        int u = 0;
                        uint8_t sp = kAborted;
                        for (; u < 4 && p + u < s1; u++) {
                            sp = (unsigned)e[u] < (unsigned)T ? vst[e[u]] : (e[u] >= T && NW ? group_status(e[u], t) : kAborted);
                            if (sp != kAborted) break;
                        }
                        p += u;
                        if (sp != kAborted) {
                            if (sp == kCommitted) res = kAborted;
                            break;
                        }
                    }
                    if (p < s1) break;
                }
                if (r == rend) res = kCommitted;
                w.eptr[t] = p;
                if (res != kUndecided)
                    vst[t] = res;
                else
                    more = 1;
            }
            if (more) s_more = 1;
            __syncthreads();
            rounds++;
            if (!s_more) break;
            __syncthreads();
        }
    } else {
        // Sequential MiniConflictSet replay (SkipList.cpp:797-834) over E point indices.
        const int E = 2 * (b.R + b.W);
        for (int i = threadIdx.x; i <= E / 64; i += blockDim.x) w.mcs_bits[i] = 0;
        __syncthreads();
        for (int t = 0; t < T; t++) {
            if (st[t] != kUndecided) continue;  // uniform: st read after a barrier
            int conflict_at = INT_MAX;
            for (int r = b.roff[t]; r < b.roff[t + 1]; r++) {
                const int a = w.pos[2 * r], e = w.pos[2 * r + 1];
                int hit = 0;
                if (a < e) {
                    for (int word = (a >> 6) + threadIdx.x; word <= ((e - 1) >> 6); word += blockDim.x) {
                        uint64_t m = ((volatile uint64_t*)w.mcs_bits)[word];
                        const int lo = word << 6;
                        if (a > lo) m &= ~0ull << (a - lo);
                        if (e < lo + 64) m &= (e - lo >= 64) ? ~0ull : ((1ull << (e - lo)) - 1);
                        if (m) hit = 1;
                    }
                }
                if (__syncthreads_or(hit)) {
                    conflict_at = r - b.roff[t];
                    break;
                }
            }
            if (conflict_at == INT_MAX) {
                for (int x = b.woff[t]; x < b.woff[t + 1]; x++) {
                    const int g = b.R + x;
                    const int a = w.pos[2 * g], e = w.pos[2 * g + 1];
                    if (a < e) {
                        for (int word = (a >> 6) + threadIdx.x; word <= ((e - 1) >> 6); word += blockDim.x) {
                            uint64_t m = ~0ull;
                            const int lo = word << 6;
                            if (a > lo) m &= ~0ull << (a - lo);
                            if (e < lo + 64) m &= (e - lo >= 64) ? ~0ull : ((1ull << (e - lo)) - 1);
                            atomicOr((unsigned long long*)&w.mcs_bits[word], (unsigned long long)m);
                        }
                    }
                    __syncthreads();
                }
            }
            if (threadIdx.x == 0) {
                st[t] = conflict_at == INT_MAX ? kCommitted : kAborted;
                if (conflict_at != INT_MAX) w.first_conf[t] = conflict_at;
            }
            __syncthreads();
        }
        rounds = -1;
    }
    __syncthreads();
    if (threadIdx.x == 0) trace_max(w.trace, kTrResRounds);
    if (NW && !overflow && w.report) {  // final committed minima per group (conflicting-key reports)
        group_minima(st);
        for (int j = threadIdx.x; j < NW; j += blockDim.x) w.gminc[j] = minComm[j];
    }
    if (in_regs) {  // the undecided ones (never TooOld: the pre-pass aborted those)
#pragma unroll
        for (int k = 0; k < kTPer; k++) {
            const int t = tt[k];
            if (t >= 0) {
                const uint8_t x = st[t];
                w.status[t] = x;
                vout[t] = x == kCommitted ? 2 : 0;  // verdict_byte
                if (w.vdev) w.vdev[t] = x == kCommitted ? 2 : 0;
            }
        }
    } else {
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            w.status[t] = st[t];
            vout[t] = verdict_byte(b, t, st[t]);
            if (w.vdev) w.vdev[t] = verdict_byte(b, t, st[t]);
        }
    }
    if (threadIdx.x == 0) sc->rounds = rounds;
    (void)hs;  // D.Combine: k_combine, across workgroups, after this launch
    if (threadIdx.x == 0) trace_max(w.trace, kTrResEnd);
}

// D.Combine after batch-order rounds (candidate edges existed): the same two chained look-back
// scans as the no-edge case, over the final statuses; exits at once when k_resolve_pre combined.
__global__ __launch_bounds__(kScanThreads) void k_combine(BatchDev b, Work w) {
    __shared__ uint32_t sv[1][scan_pad(kCombineP)];
    __shared__ uint32_t swave[1][kScanThreads / 64];
    __shared__ uint32_t sbase[1];
    __shared__ int s_tile;
    if (w.bsc->n_edges == 0 && !w.bsc->edge_overflow) return;
    if (threadIdx.x == 0) s_tile = atomicAdd(w.scan[kScanCover].counter, 1);
    __syncthreads();
    const int64_t n = 2 * (int64_t)b.W;
    const int64_t ntiles = n > 0 ? (n + kCombineTile - 1) / kCombineTile : 1;
    if (s_tile >= ntiles) return;
    scan_tile<1, CoverScan, kCombineP>(CoverScan{w, b, 1}, n, s_tile, ntiles, w.scan[kScanCover], sv, swave, sbase);
    scan_tile<1, SegNumScan, kCombineP>(SegNumScan{w}, n, s_tile, ntiles, w.scan[kScanSegNum], sv, swave, sbase);
}

// First conflicting read index of intra-batch aborts that report conflicting keys
// (SkipList.cpp:821-828).
__global__ __launch_bounds__(kBlock) void k_intra_report(BatchDev b, Work w) {
    const BatchScalars* sc = w.bsc;
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= b.R || sc->edge_overflow) return;
    const int t = b.rowner[r];
    if (!(b.flags[t] & kFlagReport) || w.hist_conf[t] || w.status[t] != kAborted) return;
    for (int p = w.eoff[r]; p < w.eoff[r] + w.ecur[r]; p++) {
        const int e = w.edges[p];
        if (((unsigned)e < (unsigned)b.T && w.status[e] == kCommitted) ||
            (w.groups && e >= b.T && w.gminc[e - b.T] < t)) {
            atomicMin(&w.first_conf[t], r - b.roff[t]);
            return;
        }
    }
}

constexpr size_t kResolveLdsMax = 160 * 1024 - 1024;  // dynamic LDS of k_resolve (static uses < 1 KiB)

void init_kernel_attributes() {
    // status bytes (<= kMaxTxnLds) + write-group minima (<= 8 kMaxGroupWrites) + the members that
    // fit, within kResolveLdsMax (the rest of the 160 KiB is the kernel's static LDS)
    (void)hipFuncSetAttribute((const void*)k_resolve<5>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResolveLdsMax);
    (void)hipFuncSetAttribute((const void*)k_resolve<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResolveLdsMax);
}

void launch_resolve(hipStream_t s, const BatchDev& b, const Work& w, bool report, uint8_t* verdict_out, Scalars* sc) {
    if (b.T == 0) {  // no transactions, no writes: no union segments
        fdb_launch(k_set_i64, dim3(1), dim3(64), 0, s, &w.bsc->n_segments, (int64_t)0);
        return;
    }
    // one wave per transaction for the pre-pass, then the rounds in one workgroup
    // (at least one workgroup per D.Combine tile of the no-edge case)
    const int64_t pre_grid = std::max<int64_t>(((int64_t)b.T * 64 + kBlock - 1) / kBlock,
                                               (2 * (int64_t)b.W + kCombineTile - 1) / kCombineTile);
    fdb_launch(k_resolve_pre, dim3((unsigned)pre_grid), dim3(kBlock), 0, s, b, w, verdict_out);
    // LDS: the status bytes and the write groups' minima (the members stay in registers)
    const size_t lds = ((size_t)b.T + 15) / 16 * 16 + (w.groups ? 8 * (size_t)b.W : 0);
    Work wr = w;
    wr.report = report ? 1 : 0;
    // Without candidate edges (k_resolve_pre decided, combined and set the rounds to 0) these
    // three have nothing to do: a replay leaves them out once stage A's edge count reached the host
    t_group = kGroupEdges;
    fdb_launch(b.T <= 5 * kWG ? k_resolve<5> : k_resolve<8>, dim3(1), dim3(kWG), (uint32_t)lds, s, b, wr, verdict_out,
               sc);
    fdb_launch(k_combine, dim3((unsigned)std::max<int64_t>(1, (2 * (int64_t)b.W + kCombineTile - 1) / kCombineTile)),
               dim3(kScanThreads), 0, s, b, w);
    if (b.R && report) fdb_launch(k_intra_report, dim3((b.R + kBlock - 1) / kBlock), dim3(kBlock), 0, s, b, w);
    t_group = 0;
}

// Epilogue work of a batch (k_epilogue, or fused into the merge copy when the batch does not
// compact): device verdict copy, scratch zeroing, scalars and the completion flag.
struct Epilogue {
    uint8_t* verdict_out;  // [T] verdicts, then Scalars at kVerdictScalarsOffset(T) (host-mapped)
    uint32_t* flag;        // host-mapped completion word, set to `seq` last
    uint32_t seq;
    unsigned long long* trace;
    int32_t T;
    int compacted, gc_ran;
    // Scratch the next batch on this workspace expects zeroed: exactly what this batch dirtied
    // (everything else is still zero from the allocation or an earlier epilogue), not the
    // workspace's capacity.
    uint8_t* zero8;  // hist_conf [T]
    int64_t zero8_n;
    uint8_t* zero8r;  // rconf [R]
    int64_t zero8r_n;
    int32_t* zero32b;  // ecur [R]
    int64_t zero32_n;
    uint64_t* zero64[kNumScans + 1];  // scan arena: the tile counters, then each scan's granules used
    int64_t zero64_n[kNumScans + 1];
    uint64_t* zero_bc;  // sort bucket counters of the batch's buckets (two words of each line used)
    int64_t zero_bc_n;
    int32_t* zero_rank;  // cold-start sample ranks
    int64_t zero_rank_n;
    BatchScalars* bsc;   // the batch workspace's scalars (error bits reported, then cleared)
    int64_t* nd_out;     // Scalars::ndb of the delta buffer the batch leaves current
};

// ------------------------------------------------------------------ D.MergeWrite
//
// mergeWriteConflictRanges (SkipList.cpp:899-924, 414-424): for each union segment [B, E):
// boundaries in [B, E) are removed, B is written at `now`, and E keeps the version it had
// (SkipList.cpp:419) unless a boundary at E already exists or the next segment starts at E.
// The batch merges into the delta tier, whose header is kHole: an E that inherits kHole lets the
// base tier show through from E on, exactly as the reference's E keeps the old version.

__device__ __forceinline__ const DKey& seg_key(const BatchDev& b, const Work& w, int pos, int end) {
    const int g = (int)item_range(w.pmeta[pos]);
    return b.keys[2 * g + end];
}

constexpr int kDeltaTile = 256;   // copy tile of the (small) delta tier: ~4 workgroups per CU at C2
constexpr int kBaseTile = 4096;   // copy tile of the base tier during compaction

// tile_first[t] = first segment whose lo lies in copy tile t or later (segment j's share).
__device__ __forceinline__ void fill_tile_first(int32_t* tile_first, const int64_t* lo, int64_t j, int tile) {
    const int64_t t0 = j > 0 ? lo[j - 1] / tile + 1 : 0;
    for (int64_t t = t0; t <= lo[j] / tile; t++) tile_first[t] = (int32_t)j;
}
__device__ __forceinline__ void fill_tile_first_tail(int32_t* tile_first, const int64_t* lo, int64_t U, int64_t n,
                                                     int tile) {
    const int64_t t0 = U > 0 ? lo[U - 1] / tile + 1 : 0;
    for (int64_t t = t0; t <= n / tile + 1; t++) tile_first[t] = (int32_t)U;
}

// Per union segment (mergeWriteConflictRanges' insertion points, SkipList.cpp:899-924): lo / hi =
// the delta boundaries [lo, hi) the segment removes (lower bounds of B and E), whether E needs a
// boundary of its own (no exact match, not glued to the next segment's B) and the version it
// inherits, then the exclusive prefixes of removed boundaries, inserted boundaries and tail units
// with one decoupled look-back across tiles, and tile_first for the copy.  One workgroup per tile
// of seg_per segments: 2 lookups each (B and E) plus one for the B of the segment before the tile,
// whose lo bounds the tile's first copy tiles.  Three layouts:
//   short keys, W < kSegWideMinW: 1024-thread workgroups, 63 segments per tile, kArity cooperating
//     lanes per lookup (group_lower_bound): many waves in flight for a small batch (C3 17.2 us per
//     launch against 24.6 with the wide layout, C2 17.7 against 19.2);
//   short keys, larger batches (WIDE): 256 threads, 127 segments, one lane per lookup
//     (lane_lower_bound).  The tiles' look-back chain sets the pace once tiles number in the
//     hundreds: at 32768-txn C2 batches 1040 narrow tiles took 116 us per launch, 516 wide ones 46
//     (255 segments per tile: 53, 511: 67, too few lookups in flight);
//   long keys (always WIDE): 128 threads, 63 segments, one lane per lookup (lane_lower_bound_long
//     holds the query's tail words in registers; kArity lanes per lookup measured 56 against 39 us
//     at C4).
constexpr int kSegWideMinW = 24576;
constexpr int seg_per(bool long_keys, bool wide) { return long_keys || !wide ? 63 : 127; }
constexpr int seg_lanes(bool, bool wide) { return wide ? 1 : kArity; }
constexpr int seg_threads(bool long_keys, bool wide) {
    return 2 * seg_lanes(long_keys, wide) * (seg_per(long_keys, wide) + 1);
}
inline bool seg_wide(int64_t W, bool long_keys) { return long_keys || W >= kSegWideMinW; }
inline int64_t seg_tiles(int64_t W, bool long_keys, bool wide) { return (W > 0 ? W : 1) / seg_per(long_keys, wide) + 1; }
// an upper bound over the layouts (workspace look-back granules)
inline int64_t seg_prep_tiles(int64_t W) { return (W > 0 ? W : 1) / 63 + 1; }

template <bool LONG, bool WIDE>
__global__ __launch_bounds__(seg_threads(LONG, WIDE)) void k_seg_prep(BatchDev b, Work w, Hist h, MaxLevels hm,
                                                                      const uint8_t* htail, Scalars* sc, TierIO io,
                                                                      int64_t* lvl3, int64_t lvl3_n, int64_t* lvl2,
                                                                      int64_t lvl2_n) {
    constexpr int SP = seg_per(LONG, WIDE);
    constexpr int LL = seg_lanes(LONG, WIDE);
    constexpr int NSW = (SP + 1 + 63) / 64;     // waves over the tile's SP + 1 scan entries
    __shared__ int64_t s_lo[SP + 1];            // lo of the segment before the tile, then the tile's
    __shared__ uint32_t s_val[3][SP + 1];       // removed, inserted, tail units per segment
    __shared__ uint32_t s_wsum[3][NSW];
    __shared__ uint32_t s_base[3];
    __shared__ int s_tile;
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the destination tier's top two levels, reset for the epilogue's atomicMax build (their
    // previous contents belonged to the history two batches back, which no check reads any more)
    for (int64_t i = gt; i < lvl3_n * kL3Rep; i += (int64_t)gridDim.x * blockDim.x) lvl3[i * kL3Pad] = LLONG_MIN;
    for (int64_t i = gt; i < lvl2_n; i += (int64_t)gridDim.x * blockDim.x) lvl2[i] = LLONG_MIN;
    if (threadIdx.x == 0) s_tile = atomicAdd(w.scan[kScanSegSum].counter, 1);
    __syncthreads();
    const int tile = s_tile;
    const int U = (int)w.bsc->n_segments;
    const int ntiles = U > 0 ? (U + SP - 1) / SP : 1;
    if (tile >= ntiles) return;  // spare workgroup: nobody waits on it
    const int64_t n = *io.n_in;
    const int q = threadIdx.x / (2 * LL), role = (threadIdx.x / LL) & 1;
    const int sg = tile * SP + (q < SP ? q : -1);  // slot SP: the segment before
    const bool live = sg >= 0 && sg < U && (q < SP || role == 0);
    int64_t pos = 0;
    bool eq = false;
    DKey kb{}, ke{};
    if (live) {
        kb = seg_key(b, w, w.seg_b[sg], 0);
        ke = seg_key(b, w, w.seg_e[sg], 1);
        const DKey& key = role ? ke : kb;
        if constexpr (LONG) {
            static_assert(WIDE, "long-key batches take the one-lane layout");
            QTail qt;
            load_qtail(qt, key, b.tail);
            pos = lane_lower_bound_long(h, hm, n, key, qt, htail, b.tail, eq);
        } else if constexpr (WIDE) {
            pos = lane_lower_bound(h, hm, n, key, htail, b.tail, eq);
        } else {  // the group's kArity lanes search together (live is uniform per group)
            pos = group_lower_bound<false>(h, hm, n, key, htail, b.tail, eq);
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t hi = __shfl(pos, (lane + LL) & 63, 64);
    const int exact = __shfl((int)eq, (lane + LL) & 63, 64);
    if (threadIdx.x % (2 * LL) == 0) {
        if (q == SP) {
            s_lo[0] = live ? pos : 0;
        } else if (live) {
            const int64_t lo = pos;
            const bool glue = sg + 1 < U && dkey_cmp(seg_key(b, w, w.seg_b[sg + 1], 0), b.tail, ke, b.tail) == 0;
            const bool endins = !exact && !glue;
            w.seg_lo[sg] = lo;
            w.seg_hi[sg] = hi;
            w.seg_endins[sg] = endins ? 1 : 0;
            w.seg_vend[sg] = hi > 0 ? h.ver[hi - 1] : kHole;
            s_lo[q + 1] = lo;
            s_val[0][q] = (uint32_t)(hi - lo);
            s_val[1][q] = endins ? 2 : 1;
            s_val[2][q] = tail_units(kb.len) + (endins ? tail_units(ke.len) : 0u);  // 8-byte units
        } else {
            s_val[0][q] = s_val[1][q] = s_val[2][q] = 0;
        }
    }
    __syncthreads();
    // exclusive prefixes inside the tile (entry k: segment tile * SP + k, entry SP: past the tile)
    uint32_t ex[3] = {0, 0, 0};
    if (wid < NSW) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const uint32_t v = threadIdx.x < SP ? s_val[c][threadIdx.x] : 0u;
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            ex[c] = x - v;
            if (lane == 63) s_wsum[c][wid] = x;
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        uint32_t btot[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint32_t t = 0;
#pragma unroll
            for (int k = 0; k < NSW; k++) t += s_wsum[c][k];
            btot[c] = t;
        }
        tile_lookback<3>(w.scan[kScanSegSum], tile, btot, s_base);
    }
    __syncthreads();
    if (wid < NSW) {  // entries 0..SP: the tile's segments, then the one after it
        const int k = threadIdx.x;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint32_t before = s_base[c];
            for (int v = 0; v < wid; v++) before += s_wsum[c][v];
            ex[c] += before;
        }
        const int j = tile * SP + k;
        if (k < SP && j < U) {
            w.seg_rem[j] = ex[0];
            w.seg_ins[j] = ex[1];
            w.seg_tlen[j] = ex[2];
            // tile_first[t] = j for the copy tiles t in (lo[j-1] / tile, lo[j] / tile]
            const int64_t t0 = j > 0 ? s_lo[k] / kDeltaTile + 1 : 0;
            for (int64_t t = t0; t <= s_lo[k + 1] / kDeltaTile; t++) w.tile_first[t] = j;
        }
        if (tile == ntiles - 1 && j == U && k <= SP) {
            // sentinel entries at U (totals, for elements after every segment), the remaining copy
            // tiles and the tier's new size
            const uint32_t r = ex[0], in = ex[1], tl = ex[2];
            w.seg_rem[U] = r;
            w.seg_ins[U] = in;
            w.seg_tlen[U] = tl;
            const int64_t t0 = U > 0 ? s_lo[k] / kDeltaTile + 1 : 0;
            for (int64_t t = t0; t <= n / kDeltaTile + 1; t++) w.tile_first[t] = U;
            *io.before = n;
            *io.removed = r;
            *io.n_out = n - (int64_t)r + (int64_t)in;
            sc->tail_next = sc->tail_used + 8 * (int64_t)tl;
        }
    }
}

constexpr int kSegLds = 1024;

// Streaming (non-temporal) moves for the compaction's whole-base copy: gigabytes read once and
// written once, kept out of the caches the concurrent read checks use (FDBCS_COPY_NT A/B).
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
template <bool NT, class T>
__device__ __forceinline__ T stream_load(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void stream_store(T* p, const T& v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Copy surviving old boundaries to their new positions and write each segment's inserts.  Per
// tile, the segments that can affect it are staged in LDS; element i is removed iff
// lo_j <= i < hi_j for the last segment j with lo_j <= i, else it moves to i - rem_before +
// ins_before.  `Ins` writes segment s's new boundaries starting at output position o; the inserts
// are spread over the whole grid (grid-stride over the segments), not over the copy tiles that own
// their positions: right after a compaction the delta is nearly empty and one copy tile owns every
// segment of the batch (at the reference's 32768-transaction cap, ~60k inserts by one workgroup).
template <class Ins, int TILE, bool NT = false>
__global__ __launch_bounds__(kBlock) void k_merge_copy(Segs g, Hist src, Hist dst, const int64_t* n_in,
                                                       const int64_t* U_ptr, Ins ins) {
    __shared__ int64_t s_lo[kSegLds + 1], s_hi[kSegLds + 1], s_shift[kSegLds + 1];
    __shared__ int s_j0, s_cnt;
    const int64_t n = *n_in;
    const int64_t U = *U_ptr;
    __shared__ int s_ins0, s_ins1;
    // tiles cover positions [0, n]: position n only owns the inserts of segments past every boundary
    for (int64_t i0 = (int64_t)blockIdx.x * TILE; i0 <= n; i0 += (int64_t)gridDim.x * TILE) {
        const int64_t i1 = min(n, i0 + TILE);
        if (threadIdx.x == 0) {
            const int64_t t = i0 / TILE;
            s_ins0 = g.tile_first[t];
            s_ins1 = g.tile_first[t + 1];
            s_j0 = s_ins0;  // slots: segment ja-1 (last with lo < i0), then the tile's own segments
            s_cnt = s_ins1 - s_ins0;
        }
        __syncthreads();
        const int ja = s_j0, cnt = s_cnt;
        int top = 0;  // the largest power of two <= cnt (0 for none): the lifting's first step
        if (cnt > 0 && cnt <= kSegLds)
            for (top = 1; 2 * top <= cnt;) top *= 2;
        if (cnt <= kSegLds) {
            // slot k <-> segment ja-1+k for k in [0, cnt]; slot holds lo/hi of that segment and the
            // shift applying to elements after it (= shift of segment index ja+k as prefix)
            for (int k = threadIdx.x; k <= cnt; k += blockDim.x) {
                const int j = ja - 1 + k;
                s_lo[k] = j >= 0 ? g.lo[j] : LLONG_MIN;
                s_hi[k] = j >= 0 ? g.hi[j] : LLONG_MIN;
                s_shift[k] = g.ins[j + 1] - g.rem[j + 1];  // exclusive prefixes at j+1
            }
        }
        __syncthreads();
        if (cnt <= kSegLds) {
            // 8 elements per thread per chunk: resolve every destination first (branch-free binary
            // lifting over the staged segments), then issue all loads, then all stores, so each
            // thread keeps 8 independent HBM requests in flight.
            constexpr int kPer = TILE / kBlock < 8 ? TILE / kBlock : 8;
            for (int64_t c0 = i0; c0 < i1; c0 += kPer * kBlock) {
                int64_t dsto[kPer];
#pragma unroll
                for (int k = 0; k < kPer; k++) {
                    const int64_t i = c0 + k * kBlock + threadIdx.x;
                    int sl = 0;  // last slot with s_lo <= i (slot 0 always qualifies)
#pragma unroll
                    for (int step = kSegLds; step > 0; step >>= 1) {
                        if (step > top) continue;
                        const int mid = sl + step;
                        if (mid <= cnt && s_lo[mid] <= i) sl = mid;
                    }
                    const bool keep = i < i1 && !(i >= s_lo[sl] && i < s_hi[sl]);  // else inside a written span
                    dsto[k] = keep ? i + s_shift[sl] : -1;
                }
                u64x2 kk[kPer];
                uint64_t lt[kPer], vv[kPer];
#pragma unroll
                for (int k = 0; k < kPer; k++) {
                    const int64_t i = c0 + k * kBlock + threadIdx.x;
                    const int64_t j = dsto[k] >= 0 ? i : i0;  // always-valid address, loads stay unconditional
                    kk[k] = stream_load<NT>(reinterpret_cast<const u64x2*>(src.key) + j);
                    lt[k] = stream_load<NT>(reinterpret_cast<const uint64_t*>(src.lt) + j);
                    vv[k] = stream_load<NT>(reinterpret_cast<const uint64_t*>(src.ver) + j);
                }
#pragma unroll
                for (int k = 0; k < kPer; k++) {
                    if (dsto[k] >= 0) {
                        stream_store<NT>(reinterpret_cast<u64x2*>(dst.key) + dsto[k], kk[k]);
                        stream_store<NT>(reinterpret_cast<uint64_t*>(dst.lt) + dsto[k], lt[k]);
                        stream_store<NT>(reinterpret_cast<uint64_t*>(dst.ver) + dsto[k], vv[k]);
                    }
                }
            }
        } else {
            for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
                int64_t lo = 0, hi = U;
                while (lo < hi) {
                    int64_t mid = (lo + hi) >> 1;
                    if (g.lo[mid] <= i) lo = mid + 1; else hi = mid;
                }
                const int64_t j = lo - 1;
                if (j >= 0 && i >= g.lo[j] && i < g.hi[j]) continue;
                const int64_t o = i + g.ins[j + 1] - g.rem[j + 1];
                dst.key[o] = src.key[i];
                dst.lt[o] = src.lt[i];
                dst.ver[o] = src.ver[i];
            }
        }
        __syncthreads();
    }
    for (int64_t sg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sg < U; sg += (int64_t)gridDim.x * blockDim.x)
        ins((int)sg, dst, g.lo[sg] - g.rem[sg] + g.ins[sg]);
}

// Inserts of a union segment: B at `now`, E (when needed) at the version it had.
struct BatchIns {
    BatchDev b;
    const uint32_t* pmeta;
    const int32_t *seg_b, *seg_e;
    const int64_t *tlen, *vend;
    const uint8_t* endins;
    uint8_t* htail;
    const Scalars* sc;
    int64_t now;
    __device__ const DKey& key(int pos, int end) const {
        return b.keys[2 * (int)item_range(pmeta[pos]) + end];
    }
    __device__ void operator()(int s, Hist dst, int64_t o) const {
        int64_t tu = sc->tail_used / 8 + tlen[s];  // 8-byte unit of this segment's first tail
        const DKey kb = key(seg_b[s], 0);
        uint32_t tb = 0;
        if (kb.len > 16) {
            tb = (uint32_t)tu;
            copy_tail_words(htail + 8 * tu, b.tail + kb.tail, kb.len - 16);
            tu += tail_units(kb.len);
        }
        dst.key[o] = make_ulonglong2(kb.hi, kb.lo);
        dst.lt[o] = make_uint2(kb.len, tb);
        dst.ver[o] = now;
        if (endins[s]) {
            const DKey ke = key(seg_e[s], 1);
            uint32_t te = 0;
            if (ke.len > 16) {
                te = (uint32_t)tu;
                copy_tail_words(htail + 8 * tu, b.tail + ke.tail, ke.len - 16);
            }
            dst.key[o + 1] = make_ulonglong2(ke.hi, ke.lo);
            dst.lt[o + 1] = make_uint2(ke.len, te);
            dst.ver[o + 1] = vend[s];
        }
    }
};

static Segs batch_segs(const Work& w) { return Segs{w.seg_lo, w.seg_hi, w.seg_rem, w.seg_ins, w.tile_first}; }

// Workgroups of a merge copy: the copy tiles of a source of about grid_hint_n boundaries, and at
// least one thread per insert of up to max_inserts segments.
static unsigned copy_tiles(int64_t grid_hint_n, int tile, int64_t max_inserts = 0) {
    int64_t tiles = (grid_hint_n + 1 + tile - 1) / tile;
    tiles = std::max<int64_t>(tiles, (max_inserts + kBlock - 1) / kBlock);
    if (tiles < 1) tiles = 1;
    if (tiles > 8192) tiles = 8192;
    return (unsigned)tiles;
}

static Epilogue make_epilogue(const BatchDev& b, const Work& w, int compacted, int gc_ran, uint8_t* verdict_out,
                              uint32_t* flag, uint32_t seq, int sort_nb, int sort_samples) {
    Epilogue ep{};
    ep.flag = flag;
    ep.seq = seq;
    ep.trace = w.trace;
    ep.verdict_out = verdict_out;
    ep.T = b.T;
    ep.compacted = compacted;
    ep.gc_ran = gc_ran;
    ep.zero8 = w.hist_conf;
    ep.zero8_n = b.T;
    ep.zero8r = w.rconf;
    ep.zero8r_n = b.R;
    ep.zero32b = w.ecur;
    ep.zero32_n = b.R;
    // the scans' tile counters, then the granules of the tiles each scan of this batch ran
    const int64_t G = (int64_t)b.R + b.W;
    const int64_t used[kNumScans] = {scan_granules(G, 3, kEdgeScanP), 3 * seg_prep_tiles(b.W),
                                     compacted ? w.scan_gran[kScanCompact] : 0, gc_ran ? w.scan_gran[kScanGc] : 0,
                                     scan_granules(2 * (int64_t)b.W, 1, kCombineP),
                                     scan_granules(2 * (int64_t)b.W, 1, kCombineP)};
    ep.zero64[0] = w.scan_arena;
    ep.zero64_n[0] = kNumScans;
    for (int k = 0; k < kNumScans; k++) {
        ep.zero64[k + 1] = w.scan[k].granules;
        ep.zero64_n[k + 1] = std::min<int64_t>(used[k], w.scan_gran[k]);
    }
    ep.zero_bc = w.scnt;
    ep.zero_bc_n = sort_nb;
    ep.zero_rank = w.srank;
    ep.zero_rank_n = sort_samples;
    ep.bsc = w.bsc;
    return ep;
}

void launch_merge(hipStream_t s, const BatchDev& b, const Work& w, const Hist& src, const MaxLevels& srcm,
                  const Hist& dst, const MaxLevels& dstm, const int64_t* nd_src, uint8_t* htail, Scalars* sc,
                  int64_t now, int64_t lvl3_n, int64_t lvl2_n, int64_t grid_hint_n, hipEvent_t copy_begin,
                  hipEvent_t copy_end, bool long_keys) {
    const TierIO io{nd_src, &sc->nd_next, &sc->d_before, &sc->d_rem};
    // the destination's top level is reset for the epilogue's atomicMax build (the source's levels
    // stay intact: the next batch's read check may still search them)
    const bool wide = seg_wide(b.W, long_keys);
    fdb_launch(long_keys ? k_seg_prep<true, true> : (wide ? k_seg_prep<false, true> : k_seg_prep<false, false>),
               dim3((unsigned)seg_tiles(b.W, long_keys, wide)), dim3(seg_threads(long_keys, wide)), 0, s, b, w, src, srcm, htail, sc, io, dstm.lvl[3], lvl3_n,
               dstm.lvl[2], lvl2_n);
    fdb_event(LaunchList::kTimingRecord, copy_begin, s);
    BatchIns ins{};
    ins.b = b;
    ins.pmeta = w.pmeta;
    ins.seg_b = w.seg_b;
    ins.seg_e = w.seg_e;
    ins.tlen = w.seg_tlen;
    ins.vend = w.seg_vend;
    ins.endins = w.seg_endins;
    ins.htail = htail;
    ins.sc = sc;
    ins.now = now;
    fdb_launch((k_merge_copy<BatchIns, kDeltaTile>), dim3(copy_tiles(grid_hint_n, kDeltaTile, b.W)), dim3(kBlock), 0,
               s, batch_segs(w), src, dst, nd_src, &w.bsc->n_segments, ins);
    fdb_event(LaunchList::kTimingRecord, copy_end, s);
}

// ------------------------------------------------------------------ compaction
//
// Overlay the delta tier onto the base: delta boundary j with a version overwrites the base over
// [d_j, d_{j+1}) (base boundaries there are removed, d_j is inserted); a kHole boundary j is the E
// of an earlier merge and becomes a real boundary carrying the base version at d_j, unless the
// base already has a boundary at d_j.  The result is the boundary set the reference would hold.

// One lane per delta boundary.  MODE 1: lane_lower_bound; 2: the long-key form
// (lane_lower_bound_long: tuple keys sharing 16-byte prefixes), after long-key batches.  (kArity
// lanes per boundary, round 4's search, measured 1321 against 535 us at C4.)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_compact_search(Hist base, MaxLevels basem, Hist delta,
                                                           const uint8_t* htail, const int64_t* nb_ptr,
                                                           const int64_t* nd_ptr, int64_t hdr, Work w, int64_t* lvl3,
                                                           int64_t lvl3_n, int64_t* lvl2, int64_t lvl2_n) {
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = gt; i < lvl3_n * kL3Rep; i += (int64_t)gridDim.x * blockDim.x) lvl3[i * kL3Pad] = LLONG_MIN;
    for (int64_t i = gt; i < lvl2_n; i += (int64_t)gridDim.x * blockDim.x) lvl2[i] = LLONG_MIN;
    const int64_t j = gt;
    const int64_t nd = *nd_ptr;
    if (j >= nd) return;
    const int64_t nb = *nb_ptr;
    const ulonglong2 k = delta.key[j];
    const uint2 lt = delta.lt[j];
    DKey q;
    q.hi = k.x;
    q.lo = k.y;
    q.len = lt.x;
    q.tail = 0;  // the query's tail arena below starts at its own tail
    bool exact;
    const uint8_t* qtail = hist_tail(htail, lt.y);
    int64_t lo;
    if constexpr (MODE == 1) {
        lo = lane_lower_bound(base, basem, nb, q, htail, qtail, exact);
    } else {
        QTail qt;
        load_qtail(qt, q, qtail);
        lo = lane_lower_bound_long(base, basem, nb, q, qt, htail, qtail, exact);
    }
    const int64_t dv = delta.ver[j];
    w.c_lo[j] = lo;
    w.c_exact[j] = exact ? 1 : 0;
    w.c_val[j] = dv != kHole ? dv : (lo > 0 ? base.ver[lo - 1] : hdr);
}

// Per delta boundary: removed range [lo_j, hi_j) (hi_j = lo_{j+1} for a written segment, empty for
// a hole) and 0/1 inserts, as exclusive prefixes.
struct CompactSumScan {
    Segs g;
    const int64_t* dver;
    const uint8_t* exact;
    TierIO io;
    const int64_t* nd_ptr;
    int tile;  // the copy tile of k_merge_copy<CompactIns, tile>
    __device__ int64_t hi_of(int64_t j) const {
        if (dver[j] == kHole) return g.lo[j];
        return j + 1 < *nd_ptr ? g.lo[j + 1] : *io.n_in;
    }
    __device__ void load(int64_t j, uint32_t (&v)[2]) const {
        v[0] = (uint32_t)(hi_of(j) - g.lo[j]);
        v[1] = (dver[j] != kHole || !exact[j]) ? 1u : 0u;
    }
    __device__ void store(int64_t j, const uint32_t (&ex)[2]) const {
        g.hi[j] = hi_of(j);
        g.rem[j] = ex[0];
        g.ins[j] = ex[1];
        fill_tile_first(g.tile_first, g.lo, j, tile);
    }
    __device__ void finish(const uint32_t (&tot)[2]) const {
        const int64_t U = *nd_ptr, n = *io.n_in;
        g.rem[U] = tot[0];
        g.ins[U] = tot[1];
        fill_tile_first_tail(g.tile_first, g.lo, U, n, tile);
        *io.before = n;
        *io.removed = tot[0];
        *io.n_out = n - (int64_t)tot[0] + (int64_t)tot[1];
    }
};

struct CompactIns {
    Hist delta;
    const int64_t *val, *ins;
    __device__ void operator()(int s, Hist dst, int64_t o) const {
        if (ins[s + 1] == ins[s]) return;  // hole over an existing base boundary
        dst.key[o] = delta.key[s];
        dst.lt[o] = delta.lt[s];
        dst.ver[o] = val[s];
    }
};

void launch_compact(hipStream_t s, const Work& w, const Hist& base, const MaxLevels& basem, const Hist& delta,
                    const Hist& dst, const uint8_t* htail, Scalars* sc, int64_t header_version, int64_t lvl3_n,
                    int64_t lvl2_n, int64_t delta_hint_n, int64_t grid_hint_n, hipEvent_t copy_begin,
                    hipEvent_t copy_end, int mode, int base_tile, bool nt) {
    int64_t blocks = (delta_hint_n + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (mode == 1)
        fdb_launch(k_compact_search<1>, dim3((unsigned)blocks), dim3(kBlock), 0, s, base, basem, delta, htail,
                   &sc->n, &sc->nd_next, header_version, w, basem.lvl[3], lvl3_n, basem.lvl[2], lvl2_n);
    else
        fdb_launch(k_compact_search<2>, dim3((unsigned)blocks), dim3(kBlock), 0, s, base, basem, delta, htail,
                   &sc->n, &sc->nd_next, header_version, w, basem.lvl[3], lvl3_n, basem.lvl[2], lvl2_n);
    const Segs g{w.c_lo, w.c_hi, w.c_rem, w.c_ins, w.tile_first};
    const TierIO io{&sc->n, &sc->n_next, &sc->c_before, &sc->c_rem};
    const int tile = base_tile == 1024 || base_tile == 2048 ? base_tile : kBaseTile;
    launch_scan<2>(s, CompactSumScan{g, delta.ver, w.c_exact, io, &sc->nd_next, tile}, &sc->nd_next,
                   delta_hint_n + 1, w.scan[kScanCompact]);
    fdb_event(LaunchList::kTimingRecord, copy_begin, s);
    const dim3 grid(copy_tiles(grid_hint_n, tile, delta_hint_n + 1));
    const CompactIns ins{delta, w.c_val, w.c_ins};
    auto k = tile == 1024 ? (nt ? k_merge_copy<CompactIns, 1024, true> : k_merge_copy<CompactIns, 1024>)
             : tile == 2048 ? (nt ? k_merge_copy<CompactIns, 2048, true> : k_merge_copy<CompactIns, 2048>)
                            : (nt ? k_merge_copy<CompactIns, kBaseTile, true> : k_merge_copy<CompactIns, kBaseTile>);
    fdb_launch(k, grid, dim3(kBlock), 0, s, g, base, dst, &sc->n, &sc->nd_next, ins);
    fdb_event(LaunchList::kTimingRecord, copy_end, s);
}

// ------------------------------------------------------------------ D.RemoveBefore
//
// removeBefore (SkipList.cpp:542-571) over the whole history: boundary i is dropped when its
// version and its predecessor's are both below oldestVersion (verdict-neutral).

__device__ __forceinline__ bool gc_keep(const Hist& h, int64_t i, int64_t v, int64_t hdr) {
    const int64_t pv = i ? h.ver[i - 1] : hdr;
    return h.ver[i] >= v || pv >= v;
}

struct GcScan {
    Hist src, dst;
    const uint8_t* tsrc;
    uint8_t* tdst;
    int64_t v, hdr;
    Scalars* sc;
    // [0] kept boundaries, [1] tail units of the kept boundaries (their offsets in the new arena)
    __device__ void load(int64_t i, uint32_t (&x)[2]) const {
        const bool keep = gc_keep(src, i, v, hdr);
        x[0] = keep ? 1u : 0u;
        x[1] = keep ? tail_units(src.lt[i].x) : 0u;
    }
    __device__ void store(int64_t i, const uint32_t (&ex)[2]) const {
        if (!gc_keep(src, i, v, hdr)) return;
        const int64_t o = ex[0];
        uint2 lt = src.lt[i];
        if (lt.x > 16u) {
            const uint64_t* a = (const uint64_t*)hist_tail(tsrc, lt.y);
            uint64_t* d = (uint64_t*)hist_tail(tdst, ex[1]);
            for (uint32_t k = 0; k < tail_units(lt.x); k++) d[k] = a[k];
            lt.y = ex[1];
        }
        dst.key[o] = src.key[i];
        dst.lt[o] = lt;
        dst.ver[o] = src.ver[i];
    }
    __device__ void finish(const uint32_t (&tot)[2]) const {
        sc->n_gc = tot[0];
        sc->tail_gc = 8 * (int64_t)tot[1];
    }
};

void launch_gc(hipStream_t s, const Work& w, const Hist& src, const Hist& dst, const uint8_t* tsrc, uint8_t* tdst,
               Scalars* sc, int64_t oldest, int64_t header_version, int64_t grid_hint_n) {
    launch_scan<2>(s, GcScan{src, dst, tsrc, tdst, oldest, header_version, sc}, &sc->n_next, grid_hint_n,
                   w.scan[kScanGc]);
}

int64_t scan_arena_words(int64_t T, int64_t R, int64_t W, int64_t hist_cap, int64_t delta_cap) {
    (void)T;
    const int64_t E = 2 * (R + W);
    (void)E;
    return kNumScans + scan_granules(R + W, 3, kEdgeScanP) + 3 * seg_prep_tiles(W) + scan_granules(delta_cap + 1, 2) +
           scan_granules(hist_cap, 2) + 2 * scan_granules(2 * W, 1, kCombineP);
}

void carve_scans(Work& w, int64_t T, int64_t R, int64_t W, int64_t hist_cap, int64_t delta_cap) {
    (void)T;
    const int64_t E = 2 * (R + W);
    uint64_t* a = w.scan_arena;
    (void)E;
    const int64_t gran[kNumScans] = {scan_granules(R + W, 3, kEdgeScanP), 3 * seg_prep_tiles(W),
                                     scan_granules(delta_cap + 1, 2), scan_granules(hist_cap, 2),
                                     scan_granules(2 * W, 1, kCombineP), scan_granules(2 * W, 1, kCombineP)};
    uint64_t* g = a + kNumScans;
    for (int k = 0; k < kNumScans; k++) {
        w.scan[k].counter = (int*)(a + k);
        w.scan[k].granules = g;
        w.scan_gran[k] = gran[k];
        g += gran[k];
    }
    w.scan_words = g - a;
}

// ------------------------------------------------------------------ multi-resolver routing
//
// The commit proxy's split of a batch across resolvers (CommitProxyServer.actor.cpp:118-187,
// static keyResolvers): a read range goes, unclipped, to every resolver whose key range it meets
// (intersectingRanges = [rangeContaining(begin), lower_bound(end)), fdbrpc/RangeMap.h:126-129; an
// empty range to rangeContaining(begin)), a write range to every owner it meets; a transaction
// gets a sub-transaction only on resolvers that received one of its ranges (:107-116), with its
// snapshot and report flag (:181-186).  Here every resolver routes the all-gathered shares for
// itself: one scan over the global transactions (one element each, its ranges visited by its
// thread) counts what this resolver keeps and its store places it.  TooOld (SkipList.cpp:770) is
// decided when the batch is detected (k_route_too_old), against the oldest version every earlier
// detect left: routing runs ahead of the previous batch's detect, and the Resolver adds a batch only
// after the previous one is resolved (Resolver.actor.cpp:139-150, 179-194).

__device__ __forceinline__ const ShareHeader* share_at(const RouteArgs& a, int p) {
    return (const ShareHeader*)(a.shares + (int64_t)p * a.stride);
}

// The shares are written by another HIP runtime (torch's collectives load their own), whose
// streams this engine cannot wait on: the caller's stream sets a device word once the all-gather
// is complete, and one wave here polls it (agent scope, bounded) before the routing kernels.
// The wait is bounded by `timeout_ticks` of the 100 MHz constant clock (wall_clock64): never hang
// the GPU, but outlast a slow all-gather (the communicator's first call, a straggler rank).
__global__ void k_route_wait(const uint32_t* ready, uint32_t value, uint32_t* err, uint64_t timeout_ticks) {
    if (threadIdx.x != 0) return;
    if (ready) {
        const uint64_t t0 = wall_clock64();
        for (;;) {
            if (__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == value) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                *err = 0;
                return;
            }
            if (wall_clock64() - t0 > timeout_ticks) break;
            __builtin_amdgcn_s_sleep(16);
        }
        *err = 1;
        return;
    }
    *err = 0;
}

// Per range of every share (one thread each): does it meet this resolver's [lo, hi)?  info =
// kept | an endpoint longer than 19 bytes << 1 | longer than 24 << 2 | tail bytes of both
// endpoints << 8.
__global__ __launch_bounds__(kBlock) void k_route_mark(RouteArgs a) {
    if (*a.wait_err) return;
    const int p = blockIdx.y;
    const ShareHeader* h = share_at(a, p);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= h->R + h->W || j >= a.rstride) return;
    const uint8_t* base = (const uint8_t*)h;
    const DKey* keys = (const DKey*)(base + h->off_keys);
    const uint8_t* tb = base + h->off_tail;
    const DKey kb = keys[2 * j], ke = keys[2 * j + 1];
    bool in = !a.has_hi || dkey_cmp(kb, tb, a.hi, a.btail) < 0;
    if (in && a.has_lo) in = dkey_cmp(ke, tb, a.lo, a.btail) > 0 || dkey_cmp(kb, tb, a.lo, a.btail) >= 0;
    const uint32_t tl = (kb.len > 16u ? kb.len - 16u : 0u) + (ke.len > 16u ? ke.len - 16u : 0u);
    a.info[(int64_t)p * a.rstride + j] =
        (in ? 1u : 0u) | ((kb.len > 19u || ke.len > 19u) ? 2u : 0u) | ((kb.len > 24u || ke.len > 24u) ? 4u : 0u) | (tl << 8);
}

// One element per transaction of every share (element i = share i / tcap, transaction i % tcap;
// past the share's T: padding): what this resolver keeps of it, as counts; the store places the
// sub-transaction and leaves its prefixes for k_route_write.
struct RouteScan {
    RouteArgs a;
    __device__ const ShareHeader* at(int64_t i, int& p, int& t, int64_t& gid) const {
        p = (int)(i / a.tcap);
        t = (int)(i - (int64_t)p * a.tcap);
        if (*a.wait_err) return nullptr;  // the shares never arrived: read nothing of them
        const ShareHeader* h = share_at(a, p);
        if (t >= h->T) return nullptr;
        gid = t;
        for (int q = 0; q < p; q++) gid += share_at(a, q)->T;
        return h;
    }
    // counts: sub-transaction, kept reads, kept writes, kept tail bytes, ranges with a key > 19 / > 24 bytes
    __device__ bool visit(int64_t i, uint32_t (&v)[6], bool& any, int& p, int& t, int64_t& gid,
                          const ShareHeader*& h) const {
        h = at(i, p, t, gid);
        if (!h) return false;
        const uint8_t* base = (const uint8_t*)h;
        const int32_t* roff = (const int32_t*)(base + h->off_roff);
        const int32_t* woff = (const int32_t*)(base + h->off_woff);
        const uint32_t* info = a.info + (int64_t)p * a.rstride;
        uint32_t nr = 0, nw = 0, tl = 0, g19 = 0, g24 = 0;
        const int r0 = roff[t], r1 = roff[t + 1], w0 = h->R + woff[t], w1 = h->R + woff[t + 1];
        for (int j = r0; j < r1; j++) {
            const uint32_t x = info[j];
            if (!(x & 1u)) continue;
            nr++;
            tl += x >> 8;
            g19 += (x >> 1) & 1u;
            g24 += (x >> 2) & 1u;
        }
        for (int j = w0; j < w1; j++) {
            const uint32_t x = info[j];
            if (!(x & 1u)) continue;
            nw++;
            tl += x >> 8;
            g19 += (x >> 1) & 1u;
            g24 += (x >> 2) & 1u;
        }
        any = nr + nw > 0;
        if (!any) return true;
        v[0] = 1;
        v[1] = nr;
        v[2] = nw;
        v[3] = tl;
        v[4] = g19;
        v[5] = g24;
        return true;
    }
    __device__ void load(int64_t i, uint32_t (&v)[6]) const {
        bool any;
        int p, t;
        int64_t gid;
        const ShareHeader* h;
        visit(i, v, any, p, t, gid, h);
    }
    __device__ void store(int64_t i, const uint32_t (&ex)[6]) const {
        uint32_t v[6] = {0, 0, 0, 0, 0, 0};
        bool any;
        int p, t;
        int64_t gid;
        const ShareHeader* h;
        if (!visit(i, v, any, p, t, gid, h)) return;
        if (a.out_zero && gid < a.out_n) a.out_zero[gid] = 0;
        const int lt = (int)ex[0];
        const bool fits = any && lt < a.cap_T;
        if (gid < a.inv_n) a.inv[gid] = fits ? lt : -1;
        a.txpre[i] = make_int4(fits ? lt : -1, (int)ex[1], (int)ex[2], (int)ex[3]);
        if (!fits) return;
        const uint8_t* base = (const uint8_t*)h;
        a.snap[lt] = ((const int64_t*)(base + h->off_snap))[t];
        a.flags[lt] = 0;  // TooOld is decided when the batch is detected (k_route_too_old)
        a.roff[lt] = (int32_t)ex[1];
        a.woff[lt] = (int32_t)ex[2];
    }
    __device__ void finish(const uint32_t (&tot)[6]) const {
        RouteResult r{};
        if (!*a.wait_err)
            for (int q = 0; q < a.n_shares; q++) r.global_T += share_at(a, q)->T;
        r.T = (int32_t)tot[0];
        r.R = (int32_t)tot[1];
        r.W = (int32_t)tot[2];
        r.tail_bytes = tot[3];
        r.n_gt19 = (int32_t)tot[4];
        r.n_gt24 = (int32_t)tot[5];
        r.error = (r.T > a.cap_T || r.R > a.cap_R || r.W > a.cap_W || (int64_t)tot[3] > a.cap_tail) ? 1 : 0;
        if (*a.wait_err) r.error = 2;
        if (!r.error && a.out_zero && r.global_T != a.out_n) r.error = 3;  // conflict bytes for every global txn
        if (!r.error) {
            a.roff[r.T] = r.R;
            a.woff[r.T] = r.W;
        }
        *a.dres = r;
        *a.res = r;
    }
};

// Per range of every share again: a kept range of a sub-transaction that is not TooOld goes to
// its place (the transaction's prefix plus the kept ranges before it in the transaction; reads
// before writes, as addTransaction registers them, SkipList.cpp:779-789), its tails appended.
__global__ __launch_bounds__(kBlock) void k_route_write(RouteArgs a) {
    const RouteResult res = *a.dres;
    if (res.error) return;
    const int p = blockIdx.y;
    const ShareHeader* h = share_at(a, p);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= h->R + h->W) return;
    const uint32_t* info = a.info + (int64_t)p * a.rstride;
    const uint32_t x = info[j];
    if (!(x & 1u)) return;
    const uint8_t* base = (const uint8_t*)h;
    const int t = ((const int32_t*)(base + h->off_owner))[j];
    const int4 pre = a.txpre[(int64_t)p * a.tcap + t];
    if (pre.x < 0) return;  // not placed
    const int32_t* roff = (const int32_t*)(base + h->off_roff);
    const int32_t* woff = (const int32_t*)(base + h->off_woff);
    const bool is_read = j < h->R;
    const int first = is_read ? roff[t] : h->R + woff[t];
    // kept ranges of the transaction before this one (its kept reads all precede a write's tails)
    uint32_t rank = 0, tail = (uint32_t)pre.w;
    if (!is_read)
        for (int q = roff[t]; q < roff[t + 1]; q++) tail += (info[q] & 1u) ? info[q] >> 8 : 0u;
    for (int q = first; q < j; q++) {
        const uint32_t y = info[q];
        if (!(y & 1u)) continue;
        rank++;
        tail += y >> 8;
    }
    const DKey* keys = (const DKey*)(base + h->off_keys);
    const uint8_t* tb = base + h->off_tail;
    const int64_t slot = is_read ? (int64_t)pre.y + rank : (int64_t)res.R + pre.z + rank;
    if (is_read) {
        a.rown[pre.y + rank] = pre.x;
        if (a.read_ids) a.read_ids[pre.y + rank] = j - roff[t];
    } else {
        a.wown[pre.z + rank] = pre.x;
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
        DKey k = keys[2 * j + e];
        const uint32_t n = k.len > 16u ? k.len - 16u : 0u;
        if (n) {
            const uint8_t* src = tb + k.tail;
            for (uint32_t q = 0; q < n; q++) a.tail[tail + q] = src[q];
            k.tail = tail;
            tail += n;
        } else {
            k.tail = 0;
        }
        a.keys[2 * slot + e] = k;
    }
}

// TooOld of a routed batch's sub-transactions (SkipList.cpp:770: snapshot below the oldest version
// with at least one read), decided at detect time in stage A; every kernel that reads the flags
// runs in stage B.  A TooOld sub-transaction keeps its ranges here, unlike addTransaction's: its
// status is aborted from the start, so its writes never enter the MiniConflictSet or the history,
// and its endpoints do not change any other range's answer (overlap is a key-order question).
__global__ __launch_bounds__(kBlock) void k_route_too_old(BatchDev b, int64_t oldest) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.T) return;
    if (b.roff[t + 1] > b.roff[t] && b.snap[t] < oldest) b.flags[t] |= kFlagTooOld;
}

void launch_route_too_old(hipStream_t s, const BatchDev& b, int64_t oldest) {
    if (b.T <= 0) return;
    fdb_launch(k_route_too_old, dim3((unsigned)((b.T + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, b, oldest);
}

int64_t route_scan_words(int64_t n_elems) { return 8 + scan_granules(n_elems, 6, kRouteScanP); }

void launch_route(hipStream_t s, const RouteArgs& a, ScanState st) {
    const dim3 grid((unsigned)std::max<int64_t>(1, (a.rstride + kBlock - 1) / kBlock), (unsigned)a.n_shares);
    fdb_launch(k_route_wait, dim3(1), dim3(64), 0, s, a.ready, a.ready_value, a.wait_err, a.wait_ticks);
    fdb_launch(k_route_mark, grid, dim3(kBlock), 0, s, a);
    launch_scan<6, kRouteScanP>(s, RouteScan{a}, nullptr, (int64_t)a.n_shares * a.tcap, st);
    fdb_launch(k_route_write, grid, dim3(kBlock), 0, s, a);
}

// ------------------------------------------------------------------ range-max hierarchy + epilogue
//
// Each wave reduces kEpiBlocks blocks of 64 versions to level 1 on its own (no barrier, no LDS);
// levels 2 and 3 are built by atomicMax (both reset beforehand).  With a batch attached the same
// launch writes the device copy of the verdicts (k_resolve already wrote the host-mapped bytes),
// publishes the scalars after them and then the completion flag, and zeroes the scratch the next
// batch on the workspace expects zeroed.

// Range-max levels over lvl[0][0, n0) (lvl[2] and lvl[3] reset beforehand); with a batch attached,
// also the verdicts and the scalar roll-over.  n0 comes from `n_levels` or, for a batch, from the
// tier that changed.
// Round 3 gave each workgroup 4096 boundaries, its waves 16 blocks each and wave 0 the level-2
// reduce behind a barrier: at C2 (~150k delta boundaries) ~40 workgroups, each wave issuing ~40
// dependent-free loads one after another, 10 us for the levels (device trace).  Here a wave owns 4
// blocks, so the same tier spreads over 4x the waves, and level 2 takes one atomic per wave (16 per
// word).  (16 waves per 4096-boundary workgroup with the barrier: slower, 22.6 vs 18.6 us per
// launch at C2 on one box.)
constexpr int kEpiWaves = 4;
constexpr int kEpiThreads = 64 * kEpiWaves;
constexpr int kEpiBlocks = 4;  // level-1 blocks (64 boundaries each) per wave
constexpr int64_t kEpiSpan = (int64_t)kEpiWaves * kEpiBlocks * kFan;  // boundaries per workgroup step
static_assert(kFan % kEpiBlocks == 0, "a wave's blocks share one level-2 entry");

// Words of Scalars / BatchScalars, prefetched by the publishing wave at the start of the launch.
constexpr int kScWords = (int)(sizeof(Scalars) / 8);
constexpr int kBscWords = (int)(sizeof(BatchScalars) / 8);
static_assert(sizeof(Scalars) % 8 == 0 && sizeof(BatchScalars) % 8 == 0, "scalars move in 8-byte words");
static_assert(kScWords <= 32 && kBscWords <= 32, "one lane per word, Scalars in lanes 0-31, BatchScalars in 32-63");
constexpr int sc_word(size_t off) { return (int)(off / 8); }

// BASE: the launch rebuilds a whole tier (after a compaction, or a history load), not the delta a
// merge left: the same code, named apart so per-kernel times separate the per-batch work from the
// occasional full rebuild.
template <bool BASE>
__global__ __launch_bounds__(kEpiThreads) void k_epilogue(MaxLevels m, Scalars* sc, const int64_t* n_levels, Epilogue ep) {
    if (threadIdx.x == 0) trace_min(ep.trace, kTrEpiBegin);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // the publishing wave loads the scalars it will publish now, while the levels are built: this
    // launch is the only writer of them until it publishes (every kernel that sets them ran
    // earlier on this stream)
    uint64_t pre = 0;
    if (ep.verdict_out && blockIdx.x == 0 && wid == 0) {
        if (lane < kScWords)
            pre = reinterpret_cast<const uint64_t*>(sc)[lane];
        else if (lane >= 32 && lane < 32 + kBscWords)
            pre = reinterpret_cast<const uint64_t*>(ep.bsc)[lane - 32];
    }
    int64_t n0;
    if (n_levels)
        n0 = *n_levels;
    else if (ep.compacted)
        n0 = ep.gc_ran ? sc->n_gc : sc->n_next;
    else
        n0 = sc->nd_next;
    const int64_t n1 = (n0 + kFan - 1) / kFan, nwv = (n1 + kEpiBlocks - 1) / kEpiBlocks;
    for (int64_t wv = (int64_t)blockIdx.x * kEpiWaves + wid; wv < nwv; wv += (int64_t)gridDim.x * kEpiWaves) {
        // the wave's kEpiBlocks blocks of 64 versions: all loads first, then the reductions
        const int64_t b1_0 = wv * kEpiBlocks;
        int64_t v[kEpiBlocks];
#pragma unroll
        for (int q = 0; q < kEpiBlocks; q++) {
            const int64_t i = (b1_0 + q) * kFan + lane;
            v[q] = i < n0 ? m.lvl[0][i] : LLONG_MIN;
        }
        const int64_t b1l = b1_0 + lane;  // lane q < kEpiBlocks owns block b1_0 + q
        ulonglong2 sk = make_ulonglong2(0, 0);
        if (lane < kEpiBlocks && b1l < n1) sk = m.keys[b1l * kFan];  // sampled key of the block
        // every 8th boundary of the wave's blocks (8 entries of skey8 per block), one per lane
        constexpr int kE8 = kEpiBlocks * kFan / 8;
        static_assert(kE8 <= 64, "one skey8 entry per lane");
        const int64_t n8 = (n0 + 7) / 8, e8_0 = b1_0 * (kFan / 8);
        ulonglong2 k8 = make_ulonglong2(0, 0);
        ulonglong2 prev_k = make_ulonglong2(0, 0);  // the previous wave's last group start (delta directory fill)
        if (lane < kE8 && e8_0 + lane < n8) {
            k8 = m.keys[(e8_0 + lane) * 8];
            m.skey8[e8_0 + lane] = k8;
        }
        if (m.edir_epoch && lane == 0 && e8_0 > 0 && e8_0 < n8) prev_k = m.keys[(e8_0 - 1) * 8];
        int64_t mine = LLONG_MIN;
#pragma unroll
        for (int q = 0; q < kEpiBlocks; q++) {
            int64_t x = v[q];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const int64_t y = __shfl_xor(x, o, 64);
                x = y > x ? y : x;
            }
            if (lane == q) mine = x;
        }
        if (lane < kEpiBlocks && b1l < n1) {
            m.lvl[1][b1l] = mine;
            m.skey[0][b1l] = sk;
            // search-tree levels above: block b1l is entry b1l / A^L of level L when divisible
            // (arithmetic level offsets: a dynamic index into skey[] would spill the argument)
            int64_t d = b1l, off = 0;
            for (int L = 1; L < kIdxLevels && d % kArity == 0; L++) {
                off += idx_level_cap(m.idx_cap, L - 1);
                d /= kArity;
                m.skey[0][off + d] = sk;
            }
        }
        if (m.edir_epoch) {
            // delta directory (group starts, as the base's): slots (dir_slot(previous start),
            // dir_slot(this start)] hold this start's skey8 index (the first start not below
            // them); the last start also fills the slots above it with the entry count.  At most
            // kDirRun slots per run: slots left over keep an older epoch and send their lookups
            // down the tree.  Most runs are short (C2's delta: ~0.4 slots per start) and each lane
            // writes its own; runs over 4 slots (keys crowding a few slots, as C3's hot range, and
            // the last start's run to the top) are written by the whole wave, 64 slots per store.
            const int64_t e = e8_0 + lane;
            const bool live = lane < kE8 && e < n8;
            const int64_t c_l = live ? (int64_t)dir_slot(m, k8.x, k8.y) : -1;
            int64_t a = __shfl_up(c_l, 1, 64);
            if (lane == 0) a = e8_0 > 0 && live ? (int64_t)dir_slot(m, prev_k.x, prev_k.y) : -1;
            const uint64_t tag = (uint64_t)m.edir_epoch << 32;
            const int64_t z = live ? (c_l < a + kDirRun ? c_l : a + kDirRun) : a;
            const bool wide = live && z - a > 4;
            if (live && !wide)
                for (int64_t v = a + 1; v <= z; v++) m.edir[v] = tag | (uint64_t)e;
            for (uint64_t wm = __ballot(wide); wm; wm &= wm - 1) {
                const int q = __builtin_ctzll(wm);
                const int64_t aq = __shfl(a, q, 64), zq = __shfl(z, q, 64);
                for (int64_t v = aq + 1 + lane; v <= zq; v += 64) m.edir[v] = tag | (uint64_t)(e8_0 + q);
            }
            const uint64_t lm = __ballot(live && e == n8 - 1);  // the last start: slots above it
            if (lm) {
                const int q = __builtin_ctzll(lm);
                const int64_t cq = __shfl(c_l, q, 64);
                const int64_t top = (int64_t)m.dir_top + 1, z2 = cq + kDirRun < top ? cq + kDirRun : top;
                for (int64_t v = cq + 1 + lane; v <= z2; v += 64) m.edir[v] = tag | (uint64_t)n8;
            }
        }
        // the wave's maximum into levels 2 and 3; level 3 only when above what it already holds
        // (up to 1024 waves share a level-3 word, and one word takes ~90 atomics per us)
        int64_t x = lane < kEpiBlocks ? mine : LLONG_MIN;
#pragma unroll
        for (int o = 1; o < kEpiBlocks; o <<= 1) {
            const int64_t y = __shfl_xor(x, o, 64);
            x = y > x ? y : x;
        }
#ifndef FDBCS_EPI_EXP
#define FDBCS_EPI_EXP 0
#endif
        if (lane == 0 && b1_0 < n1) {
            if (!(FDBCS_EPI_EXP & 1)) atomicMax((long long*)&m.lvl[2][b1_0 / kFan], (long long)x);
            int64_t* l3 = &m.lvl[3][((b1_0 / ((int64_t)kFan * kFan)) * kL3Rep + (int64_t)(blockIdx.x % kL3Rep)) * kL3Pad];
            if (!(FDBCS_EPI_EXP & 2) && x > __hip_atomic_load(l3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                atomicMax((long long*)l3, (long long)x);
        }
    }
    if (!ep.verdict_out) return;
    if (threadIdx.x == 0) trace_max(ep.trace, kTrEpiLevels);
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    // (the device verdicts are written by the resolution next to the host-mapped ones: this launch
    // reads nothing of the batch's slot, so a destroyed batch's slot may return to the pool once
    // the flag was seen)
    for (int64_t i = tid; i < ep.zero8_n; i += stride) ep.zero8[i] = 0;
    for (int64_t i = tid; i < ep.zero8r_n; i += stride) ep.zero8r[i] = 0;
    for (int64_t i = tid; i < ep.zero32_n; i += stride) ep.zero32b[i] = 0;
#pragma unroll
    for (int k = 0; k <= kNumScans; k++)
        for (int64_t i = tid; i < ep.zero64_n[k]; i += stride) ep.zero64[k][i] = 0;
    for (int64_t i = tid; i < ep.zero_bc_n; i += stride) {
        ep.zero_bc[(size_t)kCntStride * i] = 0;
        ep.zero_bc[(size_t)kCntStride * i + 1] = 0;
    }
    for (int64_t i = tid; i < ep.zero_rank_n; i += stride) ep.zero_rank[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0) trace_max(ep.trace, kTrEpiZero);
    if (blockIdx.x != 0) return;
    // Workgroup 0 writes the scalars the host reads next to the verdicts (which k_resolve already
    // wrote to the host-mapped buffer), then publishes the batch's sequence number.  Other
    // workgroups may still be writing levels, index and zeroed scratch when the flag lands: the
    // flag tells the host the batch's results are final, never that this launch is over (the
    // engine's cross-stream dependency checks query the ev_b event for that).  Wave 0 holds the
    // prefetched words (lane i: Scalars word i, lane 32 + i: BatchScalars word i) and writes the
    // host copy one word per lane, with the roll-over applied.
    if (wid == 0) {
        auto scw = [&](size_t off) -> int64_t { return (int64_t)__shfl(pre, sc_word(off), 64); };
        auto bsw = [&](size_t off) -> uint64_t { return __shfl(pre, 32 + sc_word(off), 64); };
        auto bs32 = [&](size_t off) -> uint32_t { return (uint32_t)(bsw(off) >> (8 * (off % 8))); };
        const int64_t n_new = !ep.compacted ? scw(offsetof(Scalars, n))
                                            : (ep.gc_ran ? scw(offsetof(Scalars, n_gc)) : scw(offsetof(Scalars, n_next)));
        const int64_t nd_new = ep.compacted ? 0 : scw(offsetof(Scalars, nd_next));
        const int64_t tail_new = ep.gc_ran ? scw(offsetof(Scalars, tail_gc)) : scw(offsetof(Scalars, tail_next));
        const int64_t edges = bs32(offsetof(BatchScalars, edge_overflow)) ? -1 : (int64_t)bsw(offsetof(BatchScalars, n_edges));
        const uint32_t dbg = bs32(offsetof(BatchScalars, debug_error)), rounds = bs32(offsetof(BatchScalars, rounds));
        const uint32_t big = bs32(offsetof(BatchScalars, sort_big));
        const int64_t nseg = (int64_t)bsw(offsetof(BatchScalars, n_segments));
        // the delta buffer the batch leaves current: one of Scalars::ndb
        const int64_t nd_slot = ep.nd_out ? ep.nd_out - sc->ndb : -1;
        static_assert(offsetof(Scalars, debug_error) % 8 == 0 &&
                          offsetof(Scalars, intra_rounds) == offsetof(Scalars, debug_error) + 4 &&
                          offsetof(Scalars, sort_big) % 8 == 0 && offsetof(Scalars, intra_edges) % 8 == 0,
                      "Scalars word packing the host copy assumes");
        if (lane < kScWords) {
            uint64_t x = pre;
            if (lane == sc_word(offsetof(Scalars, n))) x = (uint64_t)n_new;
            if (lane == sc_word(offsetof(Scalars, nd))) x = (uint64_t)nd_new;
            if (lane == sc_word(offsetof(Scalars, tail_used))) x = (uint64_t)tail_new;
            if (nd_slot >= 0 && nd_slot < 2 && lane == sc_word(offsetof(Scalars, ndb)) + nd_slot) x = (uint64_t)nd_new;
            if (lane == sc_word(offsetof(Scalars, debug_error))) x = (uint64_t)dbg | (uint64_t)rounds << 32;
            if (lane == sc_word(offsetof(Scalars, intra_edges))) x = (uint64_t)edges;
            if (lane == sc_word(offsetof(Scalars, sort_big))) x = (x & ~0xffffffffull) | big;
            if (lane == sc_word(offsetof(Scalars, n_segments))) x = (uint64_t)nseg;
            reinterpret_cast<uint64_t*>(ep.verdict_out + verdict_scalars_offset(ep.T))[lane] = x;
        }
        if (lane == 0) {
            sc->n = n_new;
            sc->nd = nd_new;
            if (ep.nd_out) *ep.nd_out = nd_new;
            sc->tail_used = tail_new;
            ep.bsc->debug_error = 0;
            ep.bsc->ovf_n = 0;  // the sort's overflow list and big-bucket count (this batch's sort is done)
            ep.bsc->n_undec = 0;  // the resolution's undecided list
            ep.bsc->sort_big = 0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) trace_max(ep.trace, kTrEpiHost);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        trace_max(ep.trace, kTrEpiFence);
        __hip_atomic_store(ep.flag, ep.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Report side outputs (rconf, hist_conf, first_conf) into the batch's host-mapped result buffer:
// a kernel rather than a DMA copy, in stream order on the batch's X stream without a copy-engine
// hand-off.
__global__ __launch_bounds__(kBlock) void k_copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                       int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

void launch_copy_bytes(hipStream_t s, void* dst, const void* src, int64_t n) {
    if (n <= 0) return;
    int64_t blocks = (n + kBlock - 1) / kBlock;
    blocks = blocks > 256 ? 256 : blocks;
    fdb_launch(k_copy_bytes, dim3((unsigned)blocks), dim3(kBlock), 0, s, (uint8_t*)dst, (const uint8_t*)src, n);
}

// Multi-resolver combine input (fdbcs_batch_set_conflict_output): out[g] = 2 - verdict of the
// batch transaction inv[g] (0 where the global transaction was not routed here); an element-wise
// MAX all-reduce over resolvers then holds 2 - min(verdict) (CommitProxyServer.actor.cpp:764-780).
// inv is host-mapped (n_global int32 over PCIe, read once).  Runs after k_resolve on the
// batch-order stream, so it is complete before the epilogue publishes the completion flag.
__global__ __launch_bounds__(kBlock) void k_conflict_output(BatchDev b, const uint8_t* __restrict__ status,
                                                            const int32_t* __restrict__ inv, int64_t n,
                                                            uint8_t* __restrict__ out) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
        const int t = inv[g];
        uint8_t c = 0;
        if (t >= 0) c = (uint8_t)(2 - verdict_byte(b, t, status[t]));
        out[g] = c;
    }
}

void launch_conflict_output(hipStream_t s, const BatchDev& b, const Work& w, const int32_t* inv, int64_t n,
                            uint8_t* out) {
    if (n <= 0) return;
    int64_t blocks = (n + kBlock - 1) / kBlock;
    blocks = blocks > 1024 ? 1024 : blocks;
    fdb_launch(k_conflict_output, dim3((unsigned)blocks), dim3(kBlock), 0, s, b, (const uint8_t*)w.status, inv, n,
               out);
}

// fdbcs_debug_hold: holds a stream until the host writes the release word (host-mapped), so batches
// queued behind it then run back to back at the device's own rate.  Bounded (a few seconds): never a hang.
__global__ void k_hold(const volatile uint32_t* release) {
    if (threadIdx.x != 0) return;
    for (int64_t spin = 0; spin < ((int64_t)1 << 22) && *release == 0u; spin++) __builtin_amdgcn_s_sleep(64);
}

void launch_hold(hipStream_t s, const uint32_t* release) {
    fdb_launch(k_hold, dim3(1), dim3(64), 0, s, (const volatile uint32_t*)release);
}

__global__ void k_lvl3_reset(int64_t* lvl3, int64_t n, int64_t* lvl2, int64_t n2) {
    for (int64_t i = threadIdx.x; i < n * kL3Rep; i += blockDim.x) lvl3[i * kL3Pad] = LLONG_MIN;
    for (int64_t i = threadIdx.x; i < n2; i += blockDim.x) lvl2[i] = LLONG_MIN;
}

static int64_t epilogue_grid(int64_t hint_n, int64_t extra) {
    int64_t g = (hint_n + kEpiSpan - 1) / kEpiSpan;
    const int64_t ge = (extra + kEpiThreads - 1) / kEpiThreads;
    g = g > ge ? g : ge;
    g = g < 1 ? 1 : g;
    return g > 4096 ? 4096 : g;
}

// Radix directory of the base tier (D.CheckRead): dir[v] = number of group starts (keys[8 j], the
// skey8 entries, j < ceil(n / 8)) whose directory slot (dir_slot) is below v, v in [0, dir_top + 1].
// A lookup whose slot holds at most kLaneProbe group starts probes them at once (lane_lower_bound:
// one directory load, one round over the slot's group starts, one over a group); a wider slot
// starts at level 0 (its samples are every 8th entry) or, crowded by shared key prefixes
// (subspaces, hot ranges), part-way down the tree.  Rebuilt with the base tier's index
// (compaction, GC, load), one binary search per slot.
__global__ __launch_bounds__(kBlock) void k_directory(MaxLevels m, const int64_t* np) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v > (int)m.dir_top + 1) return;
    const ulonglong2* keys = m.keys;
    int32_t* dir = const_cast<int32_t*>(m.dir);
    const int64_t S = (*np + 7) / 8;
    int64_t lo = 0, hi = S;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const ulonglong2 k = keys[mid * 8];
        if ((int64_t)dir_slot(m, k.x, k.y) < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    dir[v] = (int32_t)lo;
}

static void launch_directory(hipStream_t s, const MaxLevels& m, const int64_t* n) {
    if (!m.dir) return;
    fdb_launch(k_directory, dim3((m.dir_top + 1 + kBlock) / kBlock), dim3(kBlock), 0, s, m, n);
}

void launch_rangemax(hipStream_t s, const MaxLevels& m, Scalars* sc, const int64_t* n, int64_t lvl3_n,
                     int64_t lvl2_n, int64_t grid_hint_n) {
    launch_directory(s, m, n);
    fdb_launch(k_lvl3_reset, dim3(1), dim3(kBlock), 0, s, m.lvl[3], lvl3_n, m.lvl[2], lvl2_n);
    Epilogue ep{};
    ep.trace = nullptr;
    fdb_launch(k_epilogue<true>, dim3((unsigned)epilogue_grid(grid_hint_n, 0)), dim3(kEpiThreads), 0, s, m, sc, n, ep);
}

void launch_epilogue(hipStream_t s, const BatchDev& b, const Work& w, const MaxLevels& m, Scalars* sc,
                     int compacted, int gc_ran, uint8_t* verdict_out, uint32_t* flag,
                     uint32_t seq, int64_t grid_hint_n, int64_t* nd_out, int sort_nb, int sort_samples) {
    Epilogue ep = make_epilogue(b, w, compacted, gc_ran, verdict_out, flag, seq, sort_nb, sort_samples);
    ep.nd_out = nd_out;
    if (compacted) launch_directory(s, m, gc_ran ? &sc->n_gc : &sc->n_next);  // the k_epilogue's n0
    int64_t extra = std::max<int64_t>(b.R, b.T);
    for (int k = 0; k <= kNumScans; k++) extra = std::max(extra, ep.zero64_n[k]);
    if (compacted)
        fdb_launch(k_epilogue<true>, dim3((unsigned)epilogue_grid(grid_hint_n, extra)), dim3(kEpiThreads), 0, s, m, sc,
                   (const int64_t*)nullptr, ep);
    else
        fdb_launch(k_epilogue<false>, dim3((unsigned)epilogue_grid(grid_hint_n, extra)), dim3(kEpiThreads), 0, s, m, sc,
                   (const int64_t*)nullptr, ep);
}

}  // namespace fdbcs
