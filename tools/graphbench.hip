// graphbench.hip — does a hipGraph run independent branches concurrently on this box, and what do
// per-node parameter updates cost?  (a tuning tool, not part of the product or the tests)
//   hipcc -O3 --offload-arch=gfx950 tools/graphbench.hip -o tools/graphbench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

// spins ~us microseconds (100 MHz wall clock), one workgroup
__global__ void k_spin(int us, int* out) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0 && out) atomicAdd(out, 1);
}

struct BigArg {
    void* p[80];
};
__global__ void k_bigarg(BigArg b) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.p[79]) atomicAdd((int*)b.p[79], 1);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* d;
    CK(hipMalloc(&d, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // graph: fork into two independent chains of 4 x 25 us kernels each, then join
    hipGraph_t g;
    CK(hipGraphCreate(&g, 0));
    hipGraphNode_t prevA = nullptr, prevB = nullptr, nodes[8];
    for (int i = 0; i < 8; i++) {
        hipKernelNodeParams p{};
        int us = 25;
        int* out = d;
        void* args[] = {&us, &out};
        p.func = (void*)k_spin;
        p.gridDim = dim3(1);
        p.blockDim = dim3(64);
        p.kernelParams = args;
        hipGraphNode_t* prev = (i & 1) ? &prevB : &prevA;
        CK(hipGraphAddKernelNode(&nodes[i], g, *prev ? prev : nullptr, *prev ? 1 : 0, &p));
        *prev = nodes[i];
    }
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a, s));
        for (int i = 0; i < 20; i++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("two branches of 4 x 25 us: %.1f us per graph (100 = concurrent, 200 = serial)\n", ms * 1000 / 20);
    }
    // per-node parameter update cost
    {
        hipKernelNodeParams p{};
        int us = 1;
        int* out = d;
        void* args[] = {&us, &out};
        p.func = (void*)k_spin;
        p.gridDim = dim3(2);
        p.blockDim = dim3(64);
        p.kernelParams = args;
        const int n = 2000;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; i++) CK(hipGraphExecKernelNodeSetParams(ge, nodes[i & 7], &p));
        auto t1 = std::chrono::steady_clock::now();
        printf("hipGraphExecKernelNodeSetParams: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
    // a 30-node chain of kernels with 640-byte arguments: launch cost and per-node update cost
    {
        BigArg big{};
        big.p[79] = d;
        hipGraph_t g2;
        CK(hipGraphCreate(&g2, 0));
        hipGraphNode_t prev = nullptr, n2[30];
        for (int i = 0; i < 30; i++) {
            hipKernelNodeParams p{};
            void* args[] = {&big};
            p.func = (void*)k_bigarg;
            p.gridDim = dim3(64);
            p.blockDim = dim3(256);
            p.kernelParams = args;
            CK(hipGraphAddKernelNode(&n2[i], g2, prev ? &prev : nullptr, prev ? 1 : 0, &p));
            prev = n2[i];
        }
        hipGraphExec_t ge2;
        CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
        const int n = 300;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; i++) CK(hipGraphLaunch(ge2, s));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(s));
        printf("hipGraphLaunch, 30 nodes x 640-byte args: %.2f us\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
        hipKernelNodeParams p{};
        void* args[] = {&big};
        p.func = (void*)k_bigarg;
        p.gridDim = dim3(64);
        p.blockDim = dim3(256);
        p.kernelParams = args;
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 3000; i++) CK(hipGraphExecKernelNodeSetParams(ge2, n2[i % 30], &p));
        t1 = std::chrono::steady_clock::now();
        printf("SetParams, 640-byte args:                  %.2f us\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / 3000);
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; i++) {
            for (int k = 0; k < 30; k++) CK(hipGraphExecKernelNodeSetParams(ge2, n2[k], &p));
            CK(hipGraphLaunch(ge2, s));
        }
        t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(s));
        printf("30 SetParams + launch:                     %.2f us\n",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
