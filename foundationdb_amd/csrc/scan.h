// scan.h — single-pass device-wide exclusive scan with decoupled look-back (gfx950).
//
// One workgroup per 1024-element tile; tiles take ids from an atomic counter in launch order so a
// tile only ever waits on tiles that are already running (no deadlock whatever the dispatch order).
// Each tile publishes, per scanned component, an 8-byte granule {status << 32 | value} with an
// agent-scope atomic store: status 1 = tile aggregate, 2 = inclusive prefix.  Look-back reads the
// granules with agent-scope atomic loads (they bypass the per-CU L1), so the data is the flag and
// no fence is needed (MI355X_MICROARCH.md, inter-workgroup visibility, granule form R2).
//
// The element function object F supplies
//   __device__ void load(int64_t i, uint32_t (&v)[K]);             // visit i, produce K counts
//   __device__ void store(int64_t i, const uint32_t (&excl)[K]);   // exclusive prefixes of i
//   __device__ void finish(const uint32_t (&total)[K]);            // once, by the last tile
// Both visits of an element run on the same thread.  Sums are modulo 2^32, so +/-1 deltas work.
// An F that declares `static constexpr bool kOwn = true` gets store(i, excl, own) instead, own =
// element i's own counts (its inclusive minus exclusive prefixes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "launch.h"

namespace fdbcs {

constexpr int kScanThreads = 256;
constexpr int kScanPer = 4;
constexpr int kScanTile = kScanThreads * kScanPer;  // 1024: many workgroups even for small scans
constexpr int kScanPad = kScanTile + kScanTile / 4;
// elements per thread P: 4 by default; 1 for scans whose visits are chains of dependent gathers
// (a thread's P visits run one after another, so P = 1 spreads the chains over 4x the waves)
constexpr int scan_pad(int P) { return kScanThreads * P + kScanThreads * P / 4; }

__device__ __forceinline__ int scan_slot(int e) { return e + (e >> 2); }  // one pad word per thread run

__device__ __forceinline__ void granule_store(uint64_t* g, uint32_t status, uint32_t value) {
    __hip_atomic_store(g, ((uint64_t)status << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t granule_load(const uint64_t* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class F, class = void>
struct scan_wants_own : std::false_type {};
template <class F>
struct scan_wants_own<F, std::void_t<decltype(F::kOwn)>> : std::true_type {};

// Scan state for one launch: K granules per tile + the tile counter + an error word, zeroed
// before the launch (one hipMemsetAsync covers every scan of a batch).
struct ScanState {
    uint64_t* granules;  // [tiles * K]
    int* counter;
    int* error;          // set if a look-back spin exceeded its bound
};

// Decoupled look-back of one tile over K components, run by one whole wave: publishes the tile's
// aggregate btot, sums the predecessors' (64 tiles per probe, stopping at the first inclusive
// prefix; tile -1 reads as an inclusive 0), publishes the inclusive prefix and leaves the
// exclusive prefix in sbase (lane 0 writes it; the caller's barrier makes it visible).
template <int K>
__device__ __forceinline__ void tile_lookback(ScanState st, int64_t tile, const uint32_t (&btot)[K],
                                              uint32_t (&sbase)[K]) {
    const int lane = threadIdx.x & 63;
    uint64_t* g = st.granules;
    // every component's aggregate first, so successors never wait on this tile's own look-back
    if (lane < K) {
#pragma unroll
        for (int c = 0; c < K; c++)
            if (lane == c) granule_store(&g[(int64_t)tile * K + c], tile == 0 ? 2 : 1, btot[c]);
    }
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint32_t prefix = 0;
        int64_t jhi = (int64_t)tile - 1;
        uint32_t spins = 0;
        while (jhi >= 0) {
            const int64_t j = jhi - lane;
            const uint64_t x = j >= 0 ? granule_load(&g[j * K + c]) : (2ull << 32);
            const uint32_t status = (uint32_t)(x >> 32);
            const uint64_t incl = __ballot(status == 2);
            const uint64_t zero = __ballot(status == 0);
            const int first = incl ? __ffsll((long long)incl) - 1 : 63;
            const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
            if (zero & upto) {  // a tile in the window has not published yet
                if (++spins > (1u << 24)) {  // bounded: never hang the GPU
                    if (lane == 0) atomicOr(st.error, 2);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t v = (lane <= first) ? (uint32_t)x : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            prefix += v;
            if (incl) break;
            jhi -= 64;
        }
        if (lane == 0) {
            if (tile > 0) granule_store(&g[(int64_t)tile * K + c], 2, prefix + btot[c]);
            sbase[c] = prefix;
        }
    }
}

// One tile of a scan (tile ids come from the caller, in launch order).  Ends with a barrier, so
// the LDS arrays can be reused by a following stage.
template <int K, class F, int P = kScanPer>
__device__ __forceinline__ void scan_tile(const F& f, int64_t n, int tile, int64_t ntiles, ScanState st,
                                          uint32_t (&sv)[K][scan_pad(P)], uint32_t (&swave)[K][kScanThreads / 64],
                                          uint32_t (&sbase)[K]) {
    const int64_t base = (int64_t)tile * (kScanThreads * P);

    // phase 1: coalesced visits
#pragma unroll
    for (int k = 0; k < P; k++) {
        const int e = k * kScanThreads + threadIdx.x;
        const int64_t i = base + e;
        uint32_t v[K];
#pragma unroll
        for (int c = 0; c < K; c++) v[c] = 0;
        if (i < n) f.load(i, v);
#pragma unroll
        for (int c = 0; c < K; c++) sv[c][scan_slot(e)] = v[c];
    }
    __syncthreads();
    // phase 2: each thread scans its 16 consecutive elements
    uint32_t tsum[K];
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < P; j++) {
            const int slot = scan_slot(threadIdx.x * P + j);
            const uint32_t x = sv[c][slot];
            sv[c][slot] = s;
            s += x;
        }
        tsum[c] = s;
    }
    // block scan of thread sums
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t texcl[K];
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint32_t x = tsum[c];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        texcl[c] = x - tsum[c];
        if (lane == 63) swave[c][wid] = x;
    }
    __syncthreads();
    uint32_t btot[K];
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int q = 0; q < kScanThreads / 64; q++) {
            if (q < wid) before += swave[c][q];
            all += swave[c][q];
        }
        texcl[c] += before;
        btot[c] = all;
    }
    // phase 3: look-back by wave 0
    if (wid == 0) tile_lookback<K>(st, tile, btot, sbase);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < K; c++) {
        const uint32_t add = sbase[c] + texcl[c];
#pragma unroll
        for (int j = 0; j < P; j++) sv[c][scan_slot(threadIdx.x * P + j)] += add;
    }
    __syncthreads();
    // phase 4: coalesced stores
#pragma unroll
    for (int k = 0; k < P; k++) {
        const int e = k * kScanThreads + threadIdx.x;
        const int64_t i = base + e;
        if (i < n) {
            uint32_t ex[K];
#pragma unroll
            for (int c = 0; c < K; c++) ex[c] = sv[c][scan_slot(e)];
            if constexpr (scan_wants_own<F>::value) {
                uint32_t own[K];  // the next element's exclusive prefix (the tile's end for the last)
#pragma unroll
                for (int c = 0; c < K; c++)
                    own[c] = (e + 1 < kScanThreads * P ? sv[c][scan_slot(e + 1)] : sbase[c] + btot[c]) - ex[c];
                f.store(i, ex, own);
            } else {
                f.store(i, ex);
            }
        }
    }
    if (tile == ntiles - 1 && threadIdx.x == 0) {
        uint32_t tot[K];
#pragma unroll
        for (int c = 0; c < K; c++) tot[c] = sbase[c] + btot[c];
        f.finish(tot);
    }
    __syncthreads();
}

template <int K, class F, int P = kScanPer>
__global__ __launch_bounds__(kScanThreads) void k_scan(F f, const int64_t* n_ptr, int64_t n_host, ScanState st) {
    __shared__ uint32_t sv[K][scan_pad(P)];
    __shared__ uint32_t swave[K][kScanThreads / 64];
    __shared__ uint32_t sbase[K];
    __shared__ int s_tile;
    const int64_t n = n_ptr ? *n_ptr : n_host;
    if (threadIdx.x == 0) s_tile = atomicAdd(st.counter, 1);
    __syncthreads();
    const int tile = s_tile;
    const int64_t ntiles = n > 0 ? (n + kScanThreads * P - 1) / (kScanThreads * P) : 1;
    if (tile >= ntiles) return;  // spare tile of a device-sized launch: nobody waits on it
    scan_tile<K, F, P>(f, n, tile, ntiles, st, sv, swave, sbase);
}

// Two chained scans over the same n elements in one launch: stage 2's load(i) may read what
// stage 1's store(i) wrote (both visits of element i run on the same thread).  A tile runs stage
// 2 after its own stage 1; its stage-2 look-back waits only on tiles that started earlier, which
// finish their stage 1 without waiting on it, so the chain cannot deadlock.  Saves a launch
// and its queue gap on the batch-order stream.
template <int K1, class F1, int K2, class F2>
__global__ __launch_bounds__(kScanThreads) void k_scan2(F1 f1, F2 f2, int64_t n, ScanState st1, ScanState st2) {
    constexpr int K = K1 > K2 ? K1 : K2;
    __shared__ uint32_t sv[K][kScanPad];
    __shared__ uint32_t swave[K][kScanThreads / 64];
    __shared__ uint32_t sbase[K];
    __shared__ int s_tile;
    if (threadIdx.x == 0) s_tile = atomicAdd(st1.counter, 1);
    __syncthreads();
    const int tile = s_tile;
    const int64_t ntiles = n > 0 ? (n + kScanTile - 1) / kScanTile : 1;
    if (tile >= ntiles) return;
    scan_tile<K1>(f1, n, tile, ntiles, st1, reinterpret_cast<uint32_t(&)[K1][kScanPad]>(sv),
                  reinterpret_cast<uint32_t(&)[K1][kScanThreads / 64]>(swave), reinterpret_cast<uint32_t(&)[K1]>(sbase));
    scan_tile<K2>(f2, n, tile, ntiles, st2, reinterpret_cast<uint32_t(&)[K2][kScanPad]>(sv),
                  reinterpret_cast<uint32_t(&)[K2][kScanThreads / 64]>(swave), reinterpret_cast<uint32_t(&)[K2]>(sbase));
}

// Granules needed for a scan of up to n elements with K components (P elements per thread).
inline int64_t scan_granules(int64_t n, int K, int P = kScanPer) {
    return ((n > 0 ? n : 1) + kScanThreads * P - 1) / (kScanThreads * P) * K;
}

template <int K1, class F1, int K2, class F2>
void launch_scan2(hipStream_t s, const F1& f1, const F2& f2, int64_t n, ScanState st1, ScanState st2) {
    int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles < 1) tiles = 1;
    fdb_launch((k_scan2<K1, F1, K2, F2>), dim3((unsigned)tiles), dim3(kScanThreads), 0, s, f1, f2, n, st1, st2);
}

template <int K, int P = kScanPer, class F>
void launch_scan(hipStream_t s, const F& f, const int64_t* n_dev, int64_t n_max, ScanState st) {
    int64_t tiles = (n_max + kScanThreads * P - 1) / (kScanThreads * P);
    if (tiles < 1) tiles = 1;
    fdb_launch((k_scan<K, F, P>), dim3((unsigned)tiles), dim3(kScanThreads), 0, s, f, n_dev, n_max, st);
}

}  // namespace fdbcs
