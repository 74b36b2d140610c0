// launchbench.hip — host-side cost of kernel submission on this box (a tuning tool, not part of the
// product or the tests): hipLaunchKernelGGL with small and large by-value arguments, events,
// cross-stream waits, and a captured hipGraph of the same launches.
//   hipcc -O3 --offload-arch=gfx950 tools/launchbench.hip -o /tmp/launchbench
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

struct Big {
    void* p[80];
};

__global__ void k_small(int* x) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && x) x[0] += 1;
}
__global__ void k_big(Big b) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.p[79]) ((int*)b.p[79])[0] += 1;
}

template <class F>
double us_per(int n, F f, hipStream_t s) {
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int* d;
    CK(hipMalloc(&d, 4096));
    Big big{};
    big.p[79] = d;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int n = 3000;
    for (int rep = 0; rep < 2; rep++) {
        printf("launch, 8-byte args (256 WGs):    %6.2f us\n",
               us_per(n, [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, d); }, s));
        printf("launch, 640-byte args (256 WGs):  %6.2f us\n",
               us_per(n, [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big); }, s));
        printf("hipEventRecord:                   %6.2f us\n", us_per(n, [&] { (void)hipEventRecord(ev, s); }, s));
        printf("record + cross-stream wait:       %6.2f us\n", us_per(n, [&] {
                   (void)hipEventRecord(ev, s2);
                   (void)hipStreamWaitEvent(s, ev, 0);
               }, s));
    }
    // cross-stream ordering alternatives: a wait on an event already complete, stream memory
    // operations (write a value on one stream, wait for it on another)
    {
        CK(hipEventRecord(ev, s2));
        CK(hipStreamSynchronize(s2));
        printf("wait on a completed event:        %6.2f us\n", us_per(n, [&] { (void)hipStreamWaitEvent(s, ev, 0); }, s));
        uint32_t* flag;
        CK(hipMalloc(&flag, 64));
        CK(hipMemset(flag, 0, 64));
        uint32_t v = 0;
        printf("write value + cross-stream wait:  %6.2f us\n", us_per(n, [&] {
                   v++;
                   (void)hipStreamWriteValue32(s2, flag, v, 0);
                   (void)hipStreamWaitValue32(s, flag, v, hipStreamWaitValueGte, 0xffffffffu);
               }, s));
        CK(hipStreamSynchronize(s2));
        printf("write value alone:                %6.2f us\n", us_per(n, [&] {
                   v++;
                   (void)hipStreamWriteValue32(s2, flag, v, 0);
               }, s2));
    }
    // a 15-kernel graph vs 15 launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 15; i++) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 2; rep++) {
        printf("15 launches (640-byte args):      %6.2f us\n", us_per(n / 15, [&] {
                   for (int i = 0; i < 15; i++) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big);
               }, s));
        printf("hipGraphLaunch of 15 kernels:     %6.2f us\n", us_per(n / 15, [&] { (void)hipGraphLaunch(ge, s); }, s));
    }
    // device time per kernel back to back (empty kernels): launch gap on the GPU
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < 300; i++) (void)hipGraphLaunch(ge, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("device time per graph kernel:     %6.2f us\n", ms * 1000 / (300 * 15));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < 4500; i++) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("device time per stream kernel:    %6.2f us\n", ms * 1000 / 4500);
    return 0;
}
