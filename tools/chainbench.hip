// chainbench.hip — device-side cost of a chain of small dependent kernels on this box (a tuning
// tool, not part of the product or the tests).  Each "batch" is a chain of K tiny kernels on one
// stream (every kernel depends on the previous one, as in a pipeline stage); Q streams run such
// chains side by side, each chain waiting on an event of the previous batch's chain on the next
// stream (the cross-stage edge of the engine's pipeline).  Prints device microseconds per batch
// and per kernel, so the fixed dispatch cost of a launch can be compared with kernel work.
//   hipcc -O3 --offload-arch=gfx950 tools/chainbench.hip -o /tmp/chainbench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

// One dependent global round trip per kernel (read the previous kernel's word, write the next).
__global__ void k_step(int* x, int i) {
    if (threadIdx.x == 0) x[(i + 1) & 1023] = x[i & 1023] + 1;
}

// Holds stream 0 until the host has queued everything (bounded spin on a host-mapped word), so the
// device then runs the queued chains back to back, free of the host's submission rate.
__global__ void k_block(const volatile int* flag) {
    for (long spins = 0; spins < (1l << 24) && *flag == 0; spins++) __builtin_amdgcn_s_sleep(8);
}

static double run(int Q, int K, int batches, int blocks) {
    std::vector<hipStream_t> s(Q);
    std::vector<hipEvent_t> ev(Q);
    std::vector<int*> buf(Q);
    for (int q = 0; q < Q; q++) {
        CK(hipStreamCreateWithFlags(&s[q], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev[q], hipEventDisableTiming));
        CK(hipMalloc(&buf[q], 4096));
        CK(hipMemset(buf[q], 0, 4096));
    }
    int* flag = nullptr;
    int* dflag = nullptr;
    CK(hipHostMalloc(&flag, 64, hipHostMallocMapped));
    *flag = 0;
    CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
    hipEvent_t go;
    CK(hipEventCreateWithFlags(&go, hipEventDisableTiming));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_block, dim3(1), dim3(64), 0, s[0], dflag);
    CK(hipEventRecord(go, s[0]));
    for (int q = 1; q < Q; q++) CK(hipStreamWaitEvent(s[q], go, 0));
    for (int b = 0; b < batches; b++) {
        for (int q = 0; q < Q; q++) {
            if (b > 0 && Q > 1) CK(hipStreamWaitEvent(s[q], ev[(q + 1) % Q], 0));
            for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_step, dim3(blocks), dim3(256), 0, s[q], buf[q], b * K + k);
            CK(hipEventRecord(ev[q], s[q]));
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(flag, 1, __ATOMIC_SEQ_CST);
    CK(hipDeviceSynchronize());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    CK(hipEventDestroy(go));
    CK(hipHostFree(flag));
    for (int q = 0; q < Q; q++) {
        CK(hipStreamDestroy(s[q]));
        CK(hipEventDestroy(ev[q]));
        CK(hipFree(buf[q]));
    }
    return us / batches;
}

int main() {
    const int K = 8, batches = 40;  // <= ~400 packets per queue stay queued behind the blocker
    run(1, K, 20, 1);
    for (int blocks : {1, 256}) {
        for (int Q : {1, 2, 4}) {
            const double us = run(Q, K, batches, blocks);
            printf("blocks %3d  streams %d  chain %d: %.1f us per batch step, %.2f us per kernel (all streams)\n", blocks,
                   Q, K, us, us / (Q * K));
        }
    }
    return 0;
}
