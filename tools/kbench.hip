// kbench.hip — isolated kernel timings for tuning (not part of the product or the tests).
// Builds the engine's kernels into this binary and times each sort-stage launch with HIP events
// over synthetic C2-shaped endpoints, plus a few probe kernels that bound launch and memory costs.
//   hipcc -O3 --offload-arch=gfx950 -I foundationdb_amd/csrc tools/kbench.hip -o tools/kbench
#include "../foundationdb_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace fdbcs;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ unsigned long long g_wgtime[4096][2];
__device__ unsigned long long g_wgclk[4096][2];
__global__ void k_empty() {}
// LDS loop calibration: cycles per iteration of a compare-count loop over LDS, per wave
template <int MODE>
__global__ void k_ldsloop(unsigned long long* out, int iters) {
    __shared__ uint64_t sh[256];
    __shared__ uint32_t sw[256];
    const int t = threadIdx.x;
    sh[t] = (uint64_t)t * 0x9E3779B97F4A7C15ull;
    sw[t] = t;
    __syncthreads();
    const uint64_t mh = sh[(t * 7) & 255];
    const uint32_t mw = sw[(t * 7) & 255];
    int r = 0;
    const unsigned long long c0 = clock64();
    if (MODE == 0) {  // broadcast reads, one dependent chain
        for (int j = 0; j < iters; j++) r += sh[j & 255] < mh;
    } else if (MODE == 1) {  // broadcast reads, 3 fields like the rank compare
        for (int j = 0; j < iters; j++) {
            const uint64_t h = sh[j & 255], l = sh[(j + 1) & 255];
            const uint32_t w = sw[j & 255];
            r += (h < mh) | ((h == mh) & ((l < mh) | ((l == mh) & (w < mw))));
        }
    } else {  // 8 loads in flight
        for (int j = 0; j < iters; j += 8) {
            uint64_t h[8];
#pragma unroll
            for (int u = 0; u < 8; u++) h[u] = sh[(j + u) & 255];
#pragma unroll
            for (int u = 0; u < 8; u++) r += h[u] < mh;
        }
    }
    const unsigned long long c1 = clock64();
    if (t == 0) out[blockIdx.x] = c1 - c0;
    if (r == 12345) out[1000] = r;
}
// shader clock vs the 100 MHz wall clock over a busy loop
__global__ void k_clock(unsigned long long* out, int iters) {
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    float x = threadIdx.x;
    for (int i = 0; i < iters; i++) x = x * 1.0001f + 0.5f;
    const unsigned long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = w1 - w0;
        out[2] = (unsigned long long)x;
    }
}
__global__ void k_copy_items(const SortItem* a, SortItem* b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// probe: one workgroup per bucket, load -> LDS -> (optional rank count) -> store
template <int NT, int MODE>
__global__ __launch_bounds__(NT) void k_probe_bucket(SortItem* a, const int32_t* boff, const uint8_t* arena,
                                                     SortItem* out = nullptr) {
    __shared__ SortItem sh[NT];
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][0] = wall_clock64();
    if (!out) out = a;
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (m <= 1 || m > NT) return;
    SortItem x{};
    if (t < m) sh[t] = x = a[off + t];
    __syncthreads();
    if (t < m) {
        int r = t;
        if (MODE == 1) {
            SortItem mine[1] = {x};
            int rk[1] = {0};
            bool tail = false;
            rank_count<1>(sh, m, mine, rk, tail);
            r = rk[0];
        } else if (MODE == 2) {  // 64-bit hi-word only
            int c = 0;
            for (int j = 0; j < m; j++) c += sh[j].hi < x.hi;
            r = c;
        }
        out[off + r] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][1] = wall_clock64();
}

// bitonic network alone, NT threads per bucket workgroup (buckets larger than NT skipped)
template <int NT, int MODE>
__global__ __launch_bounds__(NT) void k_bitonic_probe(SortItem* a, const int32_t* boff, const uint8_t* arena) {
    __shared__ SortItem sh[NT];
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][0] = wall_clock64();
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (m > 1 && m <= NT) {
        int L = 2;
        while (L < m) L <<= 1;
        SortItem x{};
        x.hi = x.lo = ~0ull;
        x.meta = kPadMeta;
        if (t < m) x = a[off + t];
        if (MODE == 0) reg_bitonic<false>(x, sh, L, arena);
        if (t < m) a[off + t] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][1] = wall_clock64();
}

// rank sort over SoA LDS copies of (hi, lo, tie word); exact when no two items of the bucket share
// (hi, lo) with both longer than 16 bytes (the probe ignores that case)
__device__ __forceinline__ uint32_t tie_word(const SortItem& x) {
    const uint32_t l = x.len > 16u ? 17u : x.len;
    const uint32_t p = 2u * item_range(x.meta) + item_is_end(x.meta);
    return (l << 27) | (item_class(x.meta) << 25) | p;
}
template <int NT, int MODE>
__global__ __launch_bounds__(NT) void k_rank_probe(const SortItem* a, SortItem* out, const int32_t* boff) {
    __shared__ uint64_t shi[NT], slo[NT];
    __shared__ uint32_t stw[NT];
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][0] = wall_clock64();
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (m > 1 && m <= NT) {
        SortItem x{};
        uint32_t tw = 0;
        if (t < m) {
            x = a[off + t];
            tw = tie_word(x);
            shi[t] = x.hi;
            slo[t] = x.lo;
            stw[t] = tw;
        }
        __syncthreads();
        if (t < m) {
            int r = 0;
            if (MODE == 0) {
                for (int j = 0; j < m; j++) {
                    const uint64_t h = shi[j], l = slo[j];
                    const uint32_t w = stw[j];
                    r += (h < x.hi) | ((h == x.hi) & ((l < x.lo) | ((l == x.lo) & (w < tw))));
                }
            } else {  // hi word decides; ties in hi fall back per pair
                for (int j = 0; j < m; j++) {
                    const uint64_t h = shi[j];
                    int lt = h < x.hi;
                    if (h == x.hi) {
                        const uint64_t l = slo[j];
                        lt = (l < x.lo) | ((l == x.lo) & (stw[j] < tw));
                    }
                    r += lt;
                }
            }
            out[off + r] = x;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][1] = wall_clock64();
}

// rank sort, register-blocked: each wave pulls a 64-item chunk of the bucket into its lanes and
// every lane compares its own item with the chunk's items one lane at a time (readlane -> SGPR)
__device__ __forceinline__ uint64_t rl64(uint64_t v, int q) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, q);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), q);
    return ((uint64_t)hi << 32) | lo;
}
template <int NT>
__global__ __launch_bounds__(NT) void k_rank_reg(const SortItem* a, SortItem* out, const int32_t* boff) {
    __shared__ uint64_t shi[NT], slo[NT];
    __shared__ uint32_t stw[NT];
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][0] = wall_clock64();
    if (threadIdx.x == 0) g_wgclk[blockIdx.x][0] = clock64();
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x, lane = t & 63;
    if (m > 1 && m <= NT) {
        SortItem x{};
        uint32_t tw = 0;
        if (t < m) {
            x = a[off + t];
            tw = tie_word(x);
            shi[t] = x.hi;
            slo[t] = x.lo;
            stw[t] = tw;
        }
        __syncthreads();
        if ((t & ~63) < m) {  // wave has items
            int r = 0;
            for (int c = 0; c < m; c += 64) {
                const int j = c + lane;
                const uint64_t hv = j < m ? shi[j] : ~0ull, lv = j < m ? slo[j] : ~0ull;
                const uint32_t wv = j < m ? stw[j] : ~0u;
                const int cnt = m - c < 64 ? m - c : 64;
                for (int q = 0; q < cnt; q++) {
                    const uint64_t H = rl64(hv, q), L = rl64(lv, q);
                    const uint32_t Wd = __builtin_amdgcn_readlane(wv, q);
                    r += (H < x.hi) | ((H == x.hi) & ((L < x.lo) | ((L == x.lo) & (Wd < tw))));
                }
            }
            if (t < m) out[off + r] = x;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) g_wgclk[blockIdx.x][1] = clock64();
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][1] = wall_clock64();
}

// rank sort with the comparisons of each item split over G = NT / m threads (LDS partial ranks)
template <int NT, int U>
__global__ __launch_bounds__(NT) void k_rank_split(const SortItem* a, SortItem* out, const int32_t* boff) {
    __shared__ uint64_t shi[NT], slo[NT];
    __shared__ uint32_t stw[NT];
    __shared__ int srk[NT];
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][0] = wall_clock64();
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (m > 1 && m <= NT) {
        SortItem x{};
        if (t < m) {
            x = a[off + t];
            shi[t] = x.hi;
            slo[t] = x.lo;
            stw[t] = tie_word(x);
            srk[t] = 0;
        }
        __syncthreads();
        const int G = NT / m;
        const int i = t % m, g = t / m;
        if (g < G) {
            const uint64_t mh = shi[i], ml = slo[i];
            const uint32_t mw = stw[i];
            int r[U] = {};
            int j = g;
            for (; j + (U - 1) * G < m; j += U * G) {
                uint64_t h[U], l[U];
                uint32_t w[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    h[u] = shi[j + u * G];
                    l[u] = slo[j + u * G];
                    w[u] = stw[j + u * G];
                }
#pragma unroll
                for (int u = 0; u < U; u++)
                    r[u] += (h[u] < mh) | ((h[u] == mh) & ((l[u] < ml) | ((l[u] == ml) & (w[u] < mw))));
            }
            for (; j < m; j += G) {
                const uint64_t h = shi[j], l = slo[j];
                const uint32_t w = stw[j];
                r[0] += (h < mh) | ((h == mh) & ((l < ml) | ((l == ml) & (w < mw))));
            }
            int tot = 0;
#pragma unroll
            for (int u = 0; u < U; u++) tot += r[u];
            if (tot) atomicAdd(&srk[i], tot);
        }
        __syncthreads();
        if (t < m) out[off + srk[t]] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) g_wgtime[blockIdx.x][1] = wall_clock64();
}

void wg_report(const char* what, int nb) {
    static unsigned long long t[4096][2];
    CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wgtime), sizeof(t)));
    unsigned long long t0 = ~0ull, t1 = 0, sum = 0, mx = 0;
    for (int i = 0; i < nb; i++) {
        t0 = std::min(t0, t[i][0]);
        t1 = std::max(t1, t[i][1]);
        sum += t[i][1] - t[i][0];
        mx = std::max(mx, t[i][1] - t[i][0]);
    }
    printf("  %s WG times (10 ns ticks): span %llu, avg WG %.1f, max WG %llu\n", what, t1 - t0, (double)sum / nb, mx);
}

// morphs of the bucket probe toward the chunk copy
template <int V>
__global__ __launch_bounds__(512) void k_morph(SortItem* a, const int32_t* boff, const uint8_t* arena, SortItem* out) {
    __shared__ SortItem sh[512];
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (V == 1 && (m <= 1 || m > 512)) return;
    SortItem x;
    if (V == 2) x = SortItem{};
    if (V == 3) {
        SortItem y{};
        if (t < m) y = a[off + t];
        if (t < m) sh[t] = y;
        __syncthreads();
        if (t < m) y = sh[t];
        if (t < m) out[off + t] = y;
        return;
    }
    if (t < m) sh[t] = x = a[off + t];
    __syncthreads();
    if (t < m) out[off + t] = x;
}

// probe: 547 x 512 workgroups, the first m threads copy a chunk
template <int V>
__global__ __launch_bounds__(512) void k_probe_chunk(const SortItem* a, SortItem* b, const int32_t* boff, int per) {
    __shared__ SortItem sh[V >= 4 ? 1024 : 512];
    int off = blockIdx.x * per, m = per;
    if (V >= 4) sh[512 + threadIdx.x].hi = 0;
    if (V >= 2) {
        off = boff[blockIdx.x];
        m = boff[blockIdx.x + 1] - off;
    }
    const int t = threadIdx.x;
    SortItem x{};
    if (t < m) x = a[off + t];
    if (V >= 3) {
        if (t < m) sh[t] = x;
        __syncthreads();
        if (t < m) x = sh[t];
    }
    if (t < m) b[off + t] = x;
}

template <typename F>
float time_us(int reps, F&& f, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();  // warm
    CK(hipStreamSynchronize(s));
    float tot = 0;
    for (int r = 0; r < reps; r++) {
        CK(hipEventRecord(a, s));
        f();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return tot / reps * 1000.f;
}

void* dmalloc(size_t n) {
    void* p;
    CK(hipMalloc(&p, n + 256));
    CK(hipMemset(p, 0, n + 256));
    return p;
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 25000, Wn = argc > 2 ? atoi(argv[2]) : 10000;
    const int E = 2 * (R + Wn);
    const int reps = 50;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::mt19937_64 rng(1);
    std::vector<DKey> keys(E);
    for (auto& k : keys) {
        k.hi = rng();
        k.lo = rng();
        k.len = 16;
        k.tail = 0;
    }
    BatchDev b{};
    b.T = 5000;
    b.R = R;
    b.W = Wn;
    b.keys = (DKey*)dmalloc(sizeof(DKey) * E);
    CK(hipMemcpy(b.keys, keys.data(), sizeof(DKey) * E, hipMemcpyHostToDevice));
    b.tail = (uint8_t*)dmalloc(64);
    Work w{};
    w.items[0] = (SortItem*)dmalloc(sizeof(SortItem) * E);
    w.items[1] = (SortItem*)dmalloc(sizeof(SortItem) * E);
    w.splitters = (SortItem*)dmalloc(sizeof(SortItem) * 2048);
    w.bucket = (uint16_t*)dmalloc(2 * E);
    w.bcount = (int32_t*)dmalloc(4 * 2048);
    w.bcursor = (int32_t*)dmalloc(4 * 2048);
    w.boff = (int32_t*)dmalloc(4 * 2052);
    w.srank = (int32_t*)dmalloc(4 * (8192 + 64));
    const int nb = sort_buckets(E, 0);
    auto zero = [&]() {
        CK(hipMemsetAsync(w.bcount, 0, 4 * 2048, s));
        CK(hipMemsetAsync(w.bcursor, 0, 4 * 2048, s));
        CK(hipMemsetAsync(w.srank, 0, 4 * (8192 + 64), s));
    };
    printf("E=%d nb=%d\n", E, nb);
    {
        unsigned long long* d = (unsigned long long*)dmalloc(64);
        for (int g : {1, 256, 1024}) {
            hipLaunchKernelGGL(k_clock, g, 256, 0, s, d, 200000);
            CK(hipStreamSynchronize(s));
            unsigned long long h[3];
            CK(hipMemcpy(h, d, 24, hipMemcpyDeviceToHost));
            printf("clock (%d WGs): %llu shader cycles in %llu wall ticks -> %.0f MHz\n", g, h[0], h[1], 100.0 * h[0] / h[1]);
        }
    }
    {
        unsigned long long* d = (unsigned long long*)dmalloc(8 * 1024);
        for (int mode = 0; mode < 3; mode++)
            for (int wgs : {1, 256, 1024}) {
                if (mode == 0) hipLaunchKernelGGL(k_ldsloop<0>, wgs, 256, 0, s, d, 1024);
                if (mode == 1) hipLaunchKernelGGL(k_ldsloop<1>, wgs, 256, 0, s, d, 1024);
                if (mode == 2) hipLaunchKernelGGL(k_ldsloop<2>, wgs, 256, 0, s, d, 1024);
                CK(hipStreamSynchronize(s));
                unsigned long long h;
                CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
                printf("ldsloop mode %d, %4d WGs x 256: %.1f cycles per iteration\n", mode, wgs, h / 1024.0);
            }
    }
    printf("empty 1 WG:            %7.2f us\n", time_us(reps, [&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, s); }, s));
    printf("empty 547x512:         %7.2f us\n", time_us(reps, [&] { hipLaunchKernelGGL(k_empty, 547, 512, 0, s); }, s));
    printf("empty 4096x256:        %7.2f us\n", time_us(reps, [&] { hipLaunchKernelGGL(k_empty, 4096, 256, 0, s); }, s));
    printf("copy E items:          %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL(k_copy_items, (E + 255) / 256, 256, 0, s, w.items[0], w.items[1], E); }, s));
    // the stage-A sort chain, kernel by kernel
    float t_sample = 0, t_count = 0, t_scatter = 0, t_sort0 = 0, t_sort1 = 0;
    hipEvent_t ev[6];
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (int r = 0; r < reps + 1; r++) {
        zero();
        CK(hipEventRecord(ev[0], s));
        launch_sample(s, b, w, 0, 0);
        CK(hipEventRecord(ev[1], s));
        const int grid = (E + kBlock - 1) / kBlock;
        const int S = sample_count(E, nb, 0);
        hipLaunchKernelGGL(k_bucket_count, dim3(grid), dim3(kBlock), 0, s, b, w.srank, nb, S, w.bucket, w.bcount,
                           b.tail);
        CK(hipEventRecord(ev[2], s));
        hipLaunchKernelGGL(k_bucket_scatter, dim3(grid), dim3(kBlock), 0, s, b, w.bucket, w.bcount, w.bcursor, w.boff,
                           nb, w.items[0]);
        CK(hipEventRecord(ev[3], s));
        CK(hipMemcpyAsync(w.items[1], w.items[0], sizeof(SortItem) * E, hipMemcpyDeviceToDevice, s));
        CK(hipEventRecord(ev[4], s));
        hipLaunchKernelGGL(k_bucket_sort<0>, dim3(nb), dim3(kSortThreads), 0, s, w.items[0], w.splitters, w.boff, b.tail);
        CK(hipEventRecord(ev[5], s));
        CK(hipEventSynchronize(ev[5]));
        float m[5];
        for (int k = 0; k < 5; k++) CK(hipEventElapsedTime(&m[k], ev[k], ev[k + 1]));
        // bitonic on the same bucketed input
        hipEvent_t x0 = ev[0], x1 = ev[1];
        CK(hipEventRecord(x0, s));
        hipLaunchKernelGGL(k_bucket_sort<1>, dim3(nb), dim3(kSortThreads), 0, s, w.items[1], w.splitters, w.boff, b.tail);
        CK(hipEventRecord(x1, s));
        CK(hipEventSynchronize(x1));
        float mb;
        CK(hipEventElapsedTime(&mb, x0, x1));
        if (r == 0) continue;
        t_sample += m[0];
        t_count += m[1];
        t_scatter += m[2];
        t_sort0 += m[4];
        t_sort1 += mb;
    }
    printf("k_sample:              %7.2f us\n", t_sample / reps * 1000);
    printf("k_bucket_count:        %7.2f us\n", t_count / reps * 1000);
    printf("k_bucket_scatter:      %7.2f us\n", t_scatter / reps * 1000);
    printf("k_bucket_sort<rank>:   %7.2f us\n", t_sort0 / reps * 1000);
    printf("k_bucket_sort<bitonic>:%7.2f us\n", t_sort1 / reps * 1000);
    printf("chunk V4 (32KB LDS):   %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_chunk<4>), nb, 512, 0, s, w.items[1], w.items[0], w.boff, 128); }, s));
    for (int v = 0; v < 4; v++)
        printf("morph V%d:              %7.2f us\n", v, time_us(reps, [&] {
            if (v == 0) hipLaunchKernelGGL((k_morph<0>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]);
            if (v == 1) hipLaunchKernelGGL((k_morph<1>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]);
            if (v == 2) hipLaunchKernelGGL((k_morph<2>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]);
            if (v == 3) hipLaunchKernelGGL((k_morph<3>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]); }, s));
    for (int pass = 0; pass < 2; pass++) {
    printf("chunk V1 (fixed 128):  %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_chunk<1>), nb, 512, 0, s, w.items[1], w.items[0], w.boff, 128); }, s));
    printf("chunk V2 (boff):       %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_chunk<2>), nb, 512, 0, s, w.items[1], w.items[0], w.boff, 128); }, s));
    printf("chunk V3 (boff+LDS):   %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_chunk<3>), nb, 512, 0, s, w.items[1], w.items[0], w.boff, 128); }, s));
    printf("copy E items:          %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL(k_copy_items, (E + 255) / 256, 256, 0, s, w.items[0], w.items[1], E); }, s));
    }
    printf("probe 512 ld/st out-of-place: %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<512, 0>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]); }, s));
    printf("probe 512 ld/st 2 bufs alt:   %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<512, 0>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]);
        hipLaunchKernelGGL((k_probe_bucket<512, 0>), nb, 512, 0, s, w.items[0], w.boff, b.tail, w.items[1]); }, s));
    {
        hipLaunchKernelGGL((k_probe_bucket<512, 0>), nb, 512, 0, s, w.items[1], w.boff, b.tail, w.items[0]);
        CK(hipStreamSynchronize(s));
        static unsigned long long t[4096][2];
        CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wgtime), sizeof(t)));
        unsigned long long t0 = ~0ull, t1 = 0, sum = 0, mx = 0;
        for (int i = 0; i < nb; i++) {
            t0 = std::min(t0, t[i][0]);
            t1 = std::max(t1, t[i][1]);
            sum += t[i][1] - t[i][0];
            mx = std::max(mx, t[i][1] - t[i][0]);
        }
        printf("probe WG times (100MHz ticks): span %llu, avg WG %.1f, max WG %llu\n", t1 - t0, (double)sum / nb, mx);
        for (int i = 0; i < nb; i += 61) printf("  wg %d start %llu dur %llu\n", i, t[i][0] - t0, t[i][1] - t[i][0]);
    }
    printf("bitonic probe 512:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_bitonic_probe<512, 0>), nb, 512, 0, s, w.items[1], w.boff, b.tail); }, s));
    wg_report("bitonic 512", nb);
    printf("bitonic probe 256:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_bitonic_probe<256, 0>), nb, 256, 0, s, w.items[1], w.boff, b.tail); }, s));
    wg_report("bitonic 256", nb);
    printf("no-sort probe 256:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_bitonic_probe<256, 1>), nb, 256, 0, s, w.items[1], w.boff, b.tail); }, s));
    wg_report("no-sort 256", nb);
    printf("rank SoA 256 full:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_probe<256, 0>), nb, 256, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank full", nb);
    printf("rank SoA 256 hi-first: %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_probe<256, 1>), nb, 256, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank hi-first", nb);
    printf("rank reg 256:          %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_reg<256>), nb, 256, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank reg 256", nb);
    {
        static unsigned long long c[4096][2], t[4096][2];
        CK(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_wgclk), sizeof(c)));
        CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wgtime), sizeof(t)));
        double cs = 0, ts = 0;
        for (int i = 0; i < nb; i++) { cs += c[i][1] - c[i][0]; ts += t[i][1] - t[i][0]; }
        printf("  rank reg: WG shader cycles / wall ticks -> %.0f MHz\n", 100.0 * cs / ts);
    }
    printf("rank reg 512:          %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_reg<512>), nb, 512, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank reg 512", nb);
    printf("rank split 256 U4:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_split<256, 4>), nb, 256, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank split 256 U4", nb);
    printf("rank split 512 U4:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_split<512, 4>), nb, 512, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank split 512 U4", nb);
    printf("rank split 1024 U2:    %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_split<1024, 2>), nb, 1024, 0, s, w.items[1], w.items[0], w.boff); }, s));
    wg_report("rank split 1024 U2", nb);
    printf("rank SoA 512 full:     %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_rank_probe<512, 0>), nb, 512, 0, s, w.items[1], w.items[0], w.boff); }, s));
    printf("probe 512 load/store:  %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<512, 0>), nb, 512, 0, s, w.items[1], w.boff, b.tail); }, s));
    printf("probe 512 rank_count:  %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<512, 1>), nb, 512, 0, s, w.items[1], w.boff, b.tail); }, s));
    printf("probe 512 hi-only rank:%7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<512, 2>), nb, 512, 0, s, w.items[1], w.boff, b.tail); }, s));
    printf("probe 1024 rank_count: %7.2f us\n", time_us(reps, [&] {
        hipLaunchKernelGGL((k_probe_bucket<1024, 1>), nb, 1024, 0, s, w.items[1], w.boff, b.tail); }, s));
    std::vector<int32_t> bo(nb + 1);
    CK(hipMemcpy(bo.data(), w.boff, 4 * (nb + 1), hipMemcpyDeviceToHost));
    int mx = 0;
    for (int k = 0; k < nb; k++) mx = std::max(mx, bo[k + 1] - bo[k]);
    printf("largest bucket %d (of %d)\n", mx, nb);
    return 0;
}
