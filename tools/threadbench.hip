// threadbench.hip — does kernel submission scale across host threads on this box?  (a tuning
// tool, not part of the product or the tests).  N launches of a small kernel with a ~640-byte
// argument struct, on one stream from one thread, then split over two threads each on its own
// stream; prints host microseconds per launch.
//   hipcc -O3 --offload-arch=gfx950 tools/threadbench.hip -o /tmp/threadbench -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

struct Big {
    void* p[80];
};

__global__ void k_big(Big b) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.p[79]) ((int*)b.p[79])[0] += 1;
}

static double launch_many(hipStream_t s, int n, int* d) {
    Big b{};
    b.p[79] = d;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b);
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    const int n = 4000;
    int *d1, *d2;
    CK(hipMalloc(&d1, 64));
    CK(hipMalloc(&d2, 64));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    launch_many(s1, 200, d1);
    launch_many(s2, 200, d2);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; rep++) {
        const double one = launch_many(s1, n, d1);
        CK(hipDeviceSynchronize());
        double a = 0, b = 0;
        const auto t0 = std::chrono::steady_clock::now();
        std::thread th([&] { b = launch_many(s2, n / 2, d2); });
        a = launch_many(s1, n / 2, d1);
        th.join();
        const double two = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        CK(hipDeviceSynchronize());
        printf("one thread: %.2f us/launch; two threads: %.2f us/launch wall (thread times %.0f / %.0f us)\n",
               one / n, two / n, a, b);
    }
    return 0;
}
