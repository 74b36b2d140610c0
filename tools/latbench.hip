// latbench.hip — per-launch device time of the engine's kernel shapes on this box (a tuning tool,
// not part of the product or the tests): where does a ~10 us "trivial" launch go?
//   copy      one coalesced load + store per element (70k elements, 274 x 256 threads)
//   scan      the engine's decoupled look-back scan (scan.h) over 70k elements
//   chaseD    D dependent random loads per thread (25k threads) in a table of M bytes
//   ldsort    547 workgroups x 512 threads: bucket offsets, 32-byte items, LDS rank count, store
// Each shape is queued N times behind a blocker kernel, so the device runs the launches back to
// back free of the host's submission rate; reported: device us per launch.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I foundationdb_amd/csrc tools/latbench.hip -o tools/latbench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "scan.h"

namespace fdbcs {
thread_local LaunchList* t_record = nullptr;
thread_local hipError_t t_launch_error = hipSuccess;
}  // namespace fdbcs

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_block(const volatile int* flag) {
    for (long spins = 0; spins < (1l << 24) && *flag == 0; spins++) __builtin_amdgcn_s_sleep(8);
}

__global__ __launch_bounds__(256) void k_copy(const uint32_t* a, uint32_t* b, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i] + 1;
}

struct CopyScan {
    const uint32_t* a;
    uint32_t* b;
    __device__ void load(int64_t i, uint32_t (&v)[1]) const { v[0] = a[i] & 1u; }
    __device__ void store(int64_t i, const uint32_t (&ex)[1]) const { b[i] = ex[0]; }
    __device__ void finish(const uint32_t (&)[1]) const {}
};

template <int D>
__global__ __launch_bounds__(256) void k_chase(const uint64_t* tab, uint64_t mask, uint64_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int d = 0; d < D; d++) x = tab[(x ^ (x >> 29)) & mask] + (uint64_t)d;
    out[i] = x;
}

struct Item {
    uint64_t hi, lo;
    uint32_t len, tail, meta, nx;
};

__global__ __launch_bounds__(512) void k_ldsort(const Item* a, Item* o, const int* boff) {
    __shared__ uint64_t shi[512];
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    Item x{};
    if (t < m) {
        x = a[off + t];
        shi[t] = x.hi;
    }
    __syncthreads();
    int lt = 0;
    if (t < m)
        for (int j = 0; j < m; j++) lt += shi[j] < x.hi;
    if (t < m) o[off + lt] = x;
}


// no rank loop: the dispatch + load/store floor of the ldsort shape
__global__ __launch_bounds__(512) void k_ldcopy(const Item* a, Item* o, const int* boff) {
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    if (t < m) o[off + m - 1 - t] = a[off + t];
}
// rank loop unrolled: 16 keys per step through ds_read_b128, all loads of a step issued first
__global__ __launch_bounds__(512) void k_ldsort16(const Item* a, Item* o, const int* boff) {
    __shared__ __attribute__((aligned(16))) uint64_t shi[512 + 16];
    const int off = boff[blockIdx.x], m = boff[blockIdx.x + 1] - off;
    const int t = threadIdx.x;
    Item x{};
    if (t < m) x = a[off + t];
    shi[t] = t < m ? x.hi : ~0ull;
    if (t < 16) shi[512 + t] = ~0ull;
    __syncthreads();
    int lt = 0;
    if (t < m) {
        for (int j = 0; j < m; j += 16) {
            ulonglong2 p[8];
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = *reinterpret_cast<const ulonglong2*>(&shi[j + 2 * u]);
#pragma unroll
            for (int u = 0; u < 8; u++) lt += (p[u].x < x.hi) + (p[u].y < x.hi);
        }
    }
    if (t < m) o[off + lt] = x;
}
// 256-thread workgroups, 2 per bucket of the same shape (1094 workgroups)
__global__ __launch_bounds__(256) void k_ldsort256(const Item* a, Item* o, const int* boff) {
    __shared__ __attribute__((aligned(16))) uint64_t shi[512 + 16];
    const int bk = blockIdx.x >> 1, half = blockIdx.x & 1;
    const int off = boff[bk], m = boff[bk + 1] - off;
    for (int i = threadIdx.x; i < 512 + 16; i += 256) shi[i] = i < m ? a[off + i].hi : ~0ull;
    __syncthreads();
    const int t = half * 256 + threadIdx.x;
    if (t >= m) return;
    const Item x = a[off + t];
    int lt = 0;
    for (int j = 0; j < m; j += 16) {
        ulonglong2 p[8];
#pragma unroll
        for (int u = 0; u < 8; u++) p[u] = *reinterpret_cast<const ulonglong2*>(&shi[j + 2 * u]);
#pragma unroll
        for (int u = 0; u < 8; u++) lt += (p[u].x < x.hi) + (p[u].y < x.hi);
    }
    o[off + lt] = x;
}
// bitonic sort of 1024 (key, index) pairs in LDS by 256 threads, every workgroup redundantly
// (the splitter step of a one-launch partition); writes the 64 splitters of workgroup 0
__global__ __launch_bounds__(256) void k_samplesort(const Item* a, int E, uint64_t* spl) {
    __shared__ uint64_t k[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) k[i] = a[(int)((int64_t)i * E / 1024)].hi;
    __syncthreads();
    for (int sz = 2; sz <= 1024; sz <<= 1) {
        for (int j = sz >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int p = threadIdx.x + q * 256;  // pair index in [0, 512)
                const int lo = 2 * p - (p & (j - 1));
                const int hi = lo + j;
                const bool up = (lo & sz) == 0;
                const uint64_t x = k[lo], y = k[hi];
                if ((x > y) == up) { k[lo] = y; k[hi] = x; }
            }
            __syncthreads();
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) spl[threadIdx.x] = k[threadIdx.x * 16];
}


// in-kernel clock: shader cycles (s_memtime) per 100 MHz tick (s_memrealtime) over a VALU loop
__global__ __launch_bounds__(256) void k_clock(unsigned long long* out, int iters) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = 0; i < iters; i++) x = x * 1664525u + 1013904223u;
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
        out[2] = x;
    }
}
// one bucket (<= 64 items) per wave: rank by broadcasting every lane's key (readlane), no LDS
__global__ __launch_bounds__(256) void k_waverank(const Item* a, Item* o, const int* boff, int nb) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nb) return;
    const int lane = threadIdx.x & 63;
    const int off = boff[b], m = boff[b + 1] - off;
    Item x{};
    x.hi = ~0ull;
    if (lane < m) x = a[off + lane];
    int lt = 0;
    for (int j = 0; j < m; j++) {
        const uint64_t y = __shfl(x.hi, j, 64);
        lt += y < x.hi;
    }
    if (lane < m) o[off + lt] = x;
}
// one bucket (<= 64 items) per wave: bitonic network through cross-lane shuffles
__global__ __launch_bounds__(256) void k_wavebitonic(const Item* a, Item* o, const int* boff, int nb) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nb) return;
    const int lane = threadIdx.x & 63;
    const int off = boff[b], m = boff[b + 1] - off;
    uint64_t k = ~0ull;
    uint32_t id = 0xffffffffu;
    if (lane < m) {
        k = a[off + lane].hi;
        id = lane;
    }
    for (int sz = 2; sz <= 64; sz <<= 1)
        for (int j = sz >> 1; j > 0; j >>= 1) {
            const uint64_t y = __shfl_xor(k, j, 64);
            const uint32_t yi = __shfl_xor(id, j, 64);
            const bool up = ((lane & sz) == 0) == ((lane & j) == 0);
            const bool y_less = y < k || (y == k && yi < id);
            if (up == y_less) { k = y; id = yi; }
        }
    if (lane < m) o[off + lane] = a[off + id];
}


// bucket reservation pattern of k_sort_partition: one returning 64-bit atomic per element on the
// counter of a pseudo-random bucket (stride: u64 words between counters)
__global__ __launch_bounds__(256) void k_resv(unsigned long long* cnt, int stride, int nb, int n, int* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = (int)(((uint32_t)i * 2654435761u) % (uint32_t)nb);
    const unsigned long long old = atomicAdd(&cnt[(size_t)b * stride], 1ull);
    out[i] = (int)old;
}
// the same with the atomics of a workgroup's elements aggregated per bucket in LDS first
__global__ __launch_bounds__(256) void k_resv_lds(unsigned long long* cnt, int stride, int nb, int n, int* out) {
    extern __shared__ int hist[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = threadIdx.x; k < nb; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const int b = (int)(((uint32_t)i * 2654435761u) % (uint32_t)nb);
    int local = i < n ? atomicAdd(&hist[b], 1) : 0;
    __syncthreads();
    for (int k = threadIdx.x; k < nb; k += blockDim.x) {
        const int c = hist[k];
        hist[k] = c ? (int)atomicAdd(&cnt[(size_t)k * stride], (unsigned long long)c) : 0;
    }
    __syncthreads();
    if (i < n) out[i] = hist[b] + local;
}

static int* g_flag = nullptr;
static int* g_dflag = nullptr;

template <class L>
static double timed(hipStream_t s, int N, L launch) {
    launch();  // warm
    CK(hipStreamSynchronize(s));
    *g_flag = 0;
    hipLaunchKernelGGL(k_block, dim3(1), dim3(64), 0, s, g_dflag);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < N; i++) launch();
    CK(hipEventRecord(e1, s));
    __atomic_store_n(g_flag, 1, __ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 1000.0 * ms / N;
}

// one launch at a time from an idle stream (host sync in between): what a serial caller sees
template <class L>
static double single(hipStream_t s, int N, L launch) {
    double tot = 0;
    for (int i = 0; i < N; i++) {
        CK(hipStreamSynchronize(s));
        const auto t0 = std::chrono::steady_clock::now();
        launch();
        CK(hipStreamSynchronize(s));
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    return tot / N;
}

int main() {
    CK(hipHostMalloc((void**)&g_flag, 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&g_dflag, g_flag, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int n = 70000, N = 100;
    uint32_t *a, *b;
    CK(hipMalloc(&a, 4 * n));
    CK(hipMalloc(&b, 4 * n));
    CK(hipMemset(a, 1, 4 * n));
    auto copy = [&] { hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n); };
    printf("copy 70k:   %.2f us/launch back to back, %.2f us single (host wall)\n", timed(s, N, copy), single(s, 20, copy));

    // look-back scan: per-launch zeroed state (the memset is a launch too: time it alone as well)
    const int64_t words = 8 + fdbcs::scan_granules(n, 1);
    uint64_t* arena;
    CK(hipMalloc(&arena, 8 * words));
    auto zero = [&] { CK(hipMemsetAsync(arena, 0, 8 * words, s)); };
    auto scan = [&] {
        zero();
        fdbcs::ScanState st{arena + 8, (int*)arena, (int*)(arena + 1)};
        fdbcs::launch_scan<1>(s, CopyScan{a, b}, nullptr, n, st);
    };
    printf("memset:     %.2f us/launch back to back\n", timed(s, N, zero));
    printf("memset+scan 70k: %.2f us back to back, %.2f single\n", timed(s, N, scan), single(s, 20, scan));

    for (size_t mb : {64, 2048}) {
        const uint64_t cnt = (uint64_t)mb << 17;  // 8-byte entries
        uint64_t* tab;
        uint64_t* out;
        CK(hipMalloc(&tab, 8 * cnt));
        CK(hipMalloc(&out, 8 * 25000));
        std::vector<uint64_t> h(1 << 20);
        for (size_t i = 0; i < h.size(); i++) h[i] = i * 0x2545F4914F6CDD1Dull;
        for (uint64_t o = 0; o < cnt; o += h.size()) CK(hipMemcpy(tab + o, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
        const int th = 25000, g = (th + 255) / 256;
        auto c1 = [&] { hipLaunchKernelGGL(k_chase<1>, dim3(g), dim3(256), 0, s, tab, cnt - 1, out, th); };
        auto c2 = [&] { hipLaunchKernelGGL(k_chase<2>, dim3(g), dim3(256), 0, s, tab, cnt - 1, out, th); };
        auto c4 = [&] { hipLaunchKernelGGL(k_chase<4>, dim3(g), dim3(256), 0, s, tab, cnt - 1, out, th); };
        auto c8 = [&] { hipLaunchKernelGGL(k_chase<8>, dim3(g), dim3(256), 0, s, tab, cnt - 1, out, th); };
        printf("chase %4zu MB: D=1 %.2f  D=2 %.2f  D=4 %.2f  D=8 %.2f us/launch\n", mb, timed(s, N, c1), timed(s, N, c2),
               timed(s, N, c4), timed(s, N, c8));
        CK(hipFree(tab));
        CK(hipFree(out));
    }

    {
        unsigned long long* cnt;
        int* out;
        CK(hipMalloc(&cnt, 8 * 16 * 4096));
        CK(hipMalloc(&out, 4 * n));
        for (int stride : {1, 2, 16}) {
            auto r = [&] {
                CK(hipMemsetAsync(cnt, 0, 8 * 16 * 4096, s));
                hipLaunchKernelGGL(k_resv, dim3((n + 255) / 256), dim3(256), 0, s, cnt, stride, 1094, n, out);
            };
            auto rl = [&] {
                CK(hipMemsetAsync(cnt, 0, 8 * 16 * 4096, s));
                hipLaunchKernelGGL(k_resv_lds, dim3((n + 255) / 256), dim3(256), 4 * 1094, s, cnt, stride, 1094, n, out);
            };
            printf("reserve 70k in 1094 buckets, stride %2d: memset+atomics %.2f us, memset+lds-aggregated %.2f us\n",
                   stride, timed(s, N, r), timed(s, N, rl));
        }
    }
    {
        unsigned long long* ck;
        CK(hipMalloc(&ck, 64));
        unsigned long long h[3];
        for (int it : {1000, 100000}) {
            hipLaunchKernelGGL(k_clock, dim3(256), dim3(256), 0, s, ck, it);
            CK(hipMemcpy(h, ck, 24, hipMemcpyDeviceToHost));
            printf("clock: %d iters: %llu cycles / %llu ticks = %.0f MHz\n", it, h[0], h[1], 100.0 * h[0] / (h[1] ? h[1] : 1));
        }
        for (int nb : {1094}) {
            std::vector<int> bo(nb + 1);
            for (int k = 0; k <= nb; k++) bo[k] = (int)((int64_t)k * n / nb);
            int* boff;
            Item *ia, *io;
            CK(hipMalloc(&boff, 4 * (nb + 1)));
            CK(hipMemcpy(boff, bo.data(), 4 * (nb + 1), hipMemcpyHostToDevice));
            CK(hipMalloc(&ia, sizeof(Item) * n));
            CK(hipMalloc(&io, sizeof(Item) * n));
            std::vector<Item> hi(n);
            for (int i = 0; i < n; i++) hi[i] = Item{(uint64_t)i * 0x9E3779B97F4A7C15ull, 0, 16, 0, (uint32_t)i, 0};
            CK(hipMemcpy(ia, hi.data(), sizeof(Item) * n, hipMemcpyHostToDevice));
            auto wr = [&] { hipLaunchKernelGGL(k_waverank, dim3((nb + 3) / 4), dim3(256), 0, s, ia, io, boff, nb); };
            auto wb = [&] { hipLaunchKernelGGL(k_wavebitonic, dim3((nb + 3) / 4), dim3(256), 0, s, ia, io, boff, nb); };
            printf("waverank %d buckets of ~64: %.2f us/launch\n", nb, timed(s, N, wr));
            printf("wavebitonic %d buckets of ~64: %.2f us/launch\n", nb, timed(s, N, wb));
            hipLaunchKernelGGL(k_clock, dim3(256), dim3(256), 0, s, ck, 100000);
            for (int i = 0; i < 50; i++) wr();
            CK(hipMemcpy(h, ck, 24, hipMemcpyDeviceToHost));
            printf("clock after load: %.0f MHz\n", 100.0 * h[0] / (h[1] ? h[1] : 1));
        }
    }
    {
        const int nb = 547;
        std::vector<int> bo(nb + 1);
        for (int k = 0; k <= nb; k++) bo[k] = (int)((int64_t)k * n / nb);
        int* boff;
        Item *ia, *io;
        CK(hipMalloc(&boff, 4 * (nb + 1)));
        CK(hipMemcpy(boff, bo.data(), 4 * (nb + 1), hipMemcpyHostToDevice));
        CK(hipMalloc(&ia, sizeof(Item) * n));
        CK(hipMalloc(&io, sizeof(Item) * n));
        std::vector<Item> hi(n);
        for (int i = 0; i < n; i++) hi[i] = Item{(uint64_t)i * 0x9E3779B97F4A7C15ull, 0, 16, 0, (uint32_t)i, 0};
        CK(hipMemcpy(ia, hi.data(), sizeof(Item) * n, hipMemcpyHostToDevice));
        auto srt = [&] { hipLaunchKernelGGL(k_ldsort, dim3(nb), dim3(512), 0, s, ia, io, boff); };
        auto cpy = [&] { hipLaunchKernelGGL(k_ldcopy, dim3(nb), dim3(512), 0, s, ia, io, boff); };
        auto s16 = [&] { hipLaunchKernelGGL(k_ldsort16, dim3(nb), dim3(512), 0, s, ia, io, boff); };
        auto s256 = [&] { hipLaunchKernelGGL(k_ldsort256, dim3(2 * nb), dim3(256), 0, s, ia, io, boff); };
        uint64_t* spl;
        CK(hipMalloc(&spl, 8 * 64));
        auto smp = [&] { hipLaunchKernelGGL(k_samplesort, dim3(69), dim3(256), 0, s, ia, n, spl); };
        auto smp274 = [&] { hipLaunchKernelGGL(k_samplesort, dim3(274), dim3(256), 0, s, ia, n, spl); };
        printf("ldcopy (no rank loop): %.2f us/launch\n", timed(s, N, cpy));
        printf("ldsort16 (unrolled b128): %.2f us/launch\n", timed(s, N, s16));
        printf("ldsort256 (2 x 256-thread WGs per bucket): %.2f us/launch\n", timed(s, N, s256));
        printf("samplesort 1024 in LDS, 69 WGs: %.2f, 274 WGs: %.2f us/launch\n", timed(s, N, smp), timed(s, N, smp274));
        printf("ldsort 547x512: %.2f us/launch back to back, %.2f single\n", timed(s, N, srt), single(s, 20, srt));
    }
    return 0;
}
