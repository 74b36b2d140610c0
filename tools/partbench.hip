// partbench.hip — where the time of the sort's partition step goes (a tuning tool, not part of the
// product or the tests).  E random 16-byte keys are partitioned into nb buckets by nb - 1 sorted
// splitters, as k_sort_partition does: the splitters staged in LDS, a binary search, a returning
// atomic per endpoint reserving its slot in the bucket's slab (one 128-byte counter line per
// bucket), a second add counting its class for half of them, and the 32-byte item stored.
// Variants isolate each part:
//   A  splitters read from a 72-byte-stride table (the SplitKey quantile table), two searches
//   B  splitters from a compact 16-byte table, one search (+ one equality probe)
//   C  B without any atomic (slot from the endpoint id): the atomics' cost
//   D  B with each bucket's counter split in 4 (one per wave slot), a 4x shorter queue per word
//   E  B with the slot atomic only (no class-count atomic)
//   hipcc -O3 --offload-arch=gfx950 tools/partbench.hip -o tools/bin/partbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

struct Item {
    unsigned long long hi, lo;
    unsigned len, tail, meta, nx;
};
constexpr int kStride = 16;  // u64 words per counter line
constexpr int kSlab = 256;

template <int V>
__global__ __launch_bounds__(256) void k_part(const ulonglong2* keys, int E, const unsigned long long* spl, int sstride,
                                              int ns, unsigned long long* cnt, Item* slab, int* ovf) {
    extern __shared__ unsigned long long s_spl[];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    ulonglong2 k = make_ulonglong2(0, 0);
    if (p < E) k = keys[p];
    for (int i = threadIdx.x; i < ns; i += blockDim.x) {
        s_spl[2 * i] = spl[(size_t)i * sstride];
        s_spl[2 * i + 1] = spl[(size_t)i * sstride + 1];
    }
    __syncthreads();
    if (p >= E) return;
    int lo = 0, hi = ns;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const unsigned long long h = s_spl[2 * mid], l = s_spl[2 * mid + 1];
        if (h < k.x || (h == k.x && l < k.y)) lo = mid + 1; else hi = mid;
    }
    int up = lo;
    if (V == 0) {
        hi = ns;
        while (up < hi) {
            const int mid = (up + hi) >> 1;
            const unsigned long long h = s_spl[2 * mid], l = s_spl[2 * mid + 1];
            if (h < k.x || (h == k.x && l <= k.y)) up = mid + 1; else hi = mid;
        }
    } else if (lo < ns && s_spl[2 * lo] == k.x && s_spl[2 * lo + 1] == k.y) {
        up = lo + 1;
    }
    const int bk = up > lo ? up : lo;
    const unsigned cls = p & 3;
    unsigned slot;
    if (V == 2) {
        slot = (unsigned)(p % kSlab);
    } else if (V == 3) {
        const int sub = (threadIdx.x >> 6) & 3;
        slot = (unsigned)atomicAdd(&cnt[(size_t)kStride * bk + 4 + sub], 1ull);
        slot = slot * 4 + sub;
    } else {
        slot = (unsigned)atomicAdd(&cnt[(size_t)kStride * bk], 1ull | (cls == 2 ? 1ull << 32 : 0ull));
    }
    if ((V == 0 || V == 1 || V == 3) && (cls == 3 || cls == 1))
        atomicAdd(&cnt[(size_t)kStride * bk + 1], cls == 3 ? 1ull : 1ull << 32);
    Item it{k.x, k.y, 16u, 0u, (unsigned)p << 3 | cls, 0u};
    if (slot < (unsigned)kSlab)
        slab[(size_t)bk * kSlab + slot] = it;
    else
        atomicAdd(ovf, 1);
}

int main(int argc, char** argv) {
    const int E = argc > 1 ? atoi(argv[1]) : 70000;
    const int nb = argc > 2 ? atoi(argv[2]) : (E + 63) / 64;
    const int reps = 50;
    std::mt19937_64 rng(1);
    std::vector<ulonglong2> keys(E);
    for (auto& k : keys) k = make_ulonglong2(rng(), rng());
    std::vector<ulonglong2> sorted = keys;
    std::sort(sorted.begin(), sorted.end(), [](const ulonglong2& a, const ulonglong2& b) {
        return a.x < b.x || (a.x == b.x && a.y < b.y);
    });
    const int ns = nb - 1;
    std::vector<unsigned long long> spl72((size_t)ns * 9), spl16((size_t)ns * 2);
    for (int i = 0; i < ns; i++) {
        const ulonglong2 s = sorted[(size_t)(i + 1) * E / nb];
        spl72[(size_t)i * 9] = s.x;
        spl72[(size_t)i * 9 + 1] = s.y;
        spl16[(size_t)i * 2] = s.x;
        spl16[(size_t)i * 2 + 1] = s.y;
    }
    ulonglong2* dk;
    unsigned long long *d72, *d16, *cnt;
    Item* slab;
    int* ovf;
    CK(hipMalloc(&dk, sizeof(ulonglong2) * E));
    CK(hipMalloc(&d72, 8 * spl72.size()));
    CK(hipMalloc(&d16, 8 * spl16.size()));
    CK(hipMalloc(&cnt, 8 * (size_t)kStride * nb));
    CK(hipMalloc(&slab, sizeof(Item) * (size_t)kSlab * nb));
    CK(hipMalloc(&ovf, 4));
    CK(hipMemcpy(dk, keys.data(), sizeof(ulonglong2) * E, hipMemcpyHostToDevice));
    CK(hipMemcpy(d72, spl72.data(), 8 * spl72.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d16, spl16.data(), 8 * spl16.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = (E + 255) / 256;
    const unsigned shm = 16 * ns;
    auto time = [&](auto kern, const unsigned long long* spl, int sstride, const char* name) {
        double tot = 0;
        for (int r = 0; r < reps + 3; r++) {
            CK(hipMemset(cnt, 0, 8 * (size_t)kStride * nb));
            CK(hipMemset(ovf, 0, 4));
            CK(hipEventRecord(e0, 0));
            kern<<<grid, 256, shm, 0>>>(dk, E, spl, sstride, ns, cnt, slab, ovf);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) tot += ms;
        }
        int o;
        CK(hipMemcpy(&o, ovf, 4, hipMemcpyDeviceToHost));
        printf("%-60s %8.2f us  (overflow %d)\n", name, tot * 1000.0 / reps, o);
    };
    printf("E %d buckets %d\n", E, nb);
    time(k_part<0>, d72, 9, "A strided splitters, two searches, slot+class atomics");
    time(k_part<1>, d16, 2, "B compact splitters, one search, slot+class atomics");
    time(k_part<2>, d16, 2, "C B without atomics");
    time(k_part<3>, d16, 2, "D B with 4 counters per bucket");
    time(k_part<4>, d16, 2, "E B with the slot atomic only");
    return 0;
}
