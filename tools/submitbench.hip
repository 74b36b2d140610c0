// submitbench.hip — host cost of submitting one batch's kernels: direct launches with large
// by-value arguments (today's engine), direct launches with a 16-byte argument (a pointer into a
// device-side parameter block), and one static hipGraph per batch (no node updates).  The kernels
// are trivial so the device keeps up; the figure is host microseconds per batch.
// (a tuning tool, not part of the product or the tests)
//   hipcc -O3 --offload-arch=gfx950 tools/submitbench.hip -o tools/submitbench
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

struct BigArg {
    void* p[80];  // 640 bytes, like BatchDev + Work
};
__global__ void k_big(BigArg b) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.p[79]) atomicAdd((int*)b.p[79], 1);
}
struct Params {
    int* ctr;
    int pad[60];
};
__global__ void k_small(const Params* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(p->ctr, 1);
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 10;      // kernels per batch
    const int NB = argc > 2 ? atoi(argv[2]) : 2000;   // batches
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    int* d;
    CK(hipMalloc(&d, 64));
    Params* dp;
    CK(hipMalloc(&dp, sizeof(Params)));
    Params hp{};
    hp.ctr = d;
    CK(hipMemcpy(dp, &hp, sizeof(hp), hipMemcpyHostToDevice));
    BigArg big{};
    big.p[79] = d;
    hipEvent_t ea, eb;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    const int KA = K / 2, KB = K - KA;

    auto batch_direct = [&](bool small) {
        CK(hipStreamWaitEvent(sa, eb, 0));
        for (int i = 0; i < KA; i++) {
            if (small) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, sa, dp);
            else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, sa, big);
        }
        CK(hipEventRecord(ea, sa));
        CK(hipStreamWaitEvent(sb, ea, 0));
        for (int i = 0; i < KB; i++) {
            if (small) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, sb, dp);
            else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, sb, big);
        }
        CK(hipEventRecord(eb, sb));
    };
    for (int mode = 0; mode < 2; mode++) {
        for (int i = 0; i < 50; i++) batch_direct(mode == 1);
        CK(hipDeviceSynchronize());
        auto t = clk::now();
        for (int i = 0; i < NB; i++) batch_direct(mode == 1);
        const double host = us_since(t);
        CK(hipDeviceSynchronize());
        const double all = us_since(t);
        printf("direct %s args: %d kernels/batch, host %.2f us/batch (%.2f us/launch), device done %.2f us/batch\n",
               mode ? "16-byte" : "640-byte", K, host / NB, host / NB / K, all / NB);
    }
    // one static graph per batch: the same two-stream shape captured once, launched NB times
    for (int small = 0; small < 2; small++) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStream_t cap;
        CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
        hipEvent_t fork, join;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
        CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(fork, cap));
        CK(hipStreamWaitEvent(sb, fork, 0));
        for (int i = 0; i < KA; i++) {
            if (small) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, cap, dp);
            else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, cap, big);
        }
        CK(hipEventRecord(join, cap));
        CK(hipStreamWaitEvent(sb, join, 0));
        for (int i = 0; i < KB; i++) {
            if (small) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, sb, dp);
            else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, sb, big);
        }
        CK(hipEventRecord(join, sb));
        CK(hipStreamWaitEvent(cap, join, 0));
        CK(hipStreamEndCapture(cap, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 50; i++) CK(hipGraphLaunch(ge, sa));
        CK(hipDeviceSynchronize());
        auto t = clk::now();
        for (int i = 0; i < NB; i++) CK(hipGraphLaunch(ge, sa));
        const double host = us_since(t);
        CK(hipDeviceSynchronize());
        const double all = us_since(t);
        printf("graph  %s args: %d kernels/batch, host %.2f us/batch, device done %.2f us/batch\n",
               small ? "16-byte" : "640-byte", K, host / NB, all / NB);
        // single-stream graph (a chain, no fork)
        hipGraph_t g2;
        hipGraphExec_t ge2;
        CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < K; i++) {
            if (small) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, cap, dp);
            else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, cap, big);
        }
        CK(hipStreamEndCapture(cap, &g2));
        CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
        for (int i = 0; i < 50; i++) CK(hipGraphLaunch(ge2, sa));
        CK(hipDeviceSynchronize());
        t = clk::now();
        for (int i = 0; i < NB; i++) CK(hipGraphLaunch(ge2, sa));
        const double host2 = us_since(t);
        CK(hipDeviceSynchronize());
        const double all2 = us_since(t);
        printf("chain  %s args: %d kernels/graph, host %.2f us/batch, device done %.2f us/batch\n",
               small ? "16-byte" : "640-byte", K, host2 / NB, all2 / NB);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        CK(hipGraphExecDestroy(ge2));
        CK(hipGraphDestroy(g2));
    }
    // per-batch node parameter updates: a chain graph of K kernels (640-byte arguments), every
    // node's parameters set before each launch, as a graph of a stage with per-batch arguments
    for (int nk : {1, 4, 5, K}) {
        hipStream_t cap;
        CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < nk; i++) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, cap, big);
        CK(hipStreamEndCapture(cap, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        CK(hipGraphGetNodes(g, nodes.data(), &nn));
        std::vector<hipKernelNodeParams> kp(nn);
        for (size_t i = 0; i < nn; i++) CK(hipGraphKernelNodeGetParams(nodes[i], &kp[i]));
        BigArg arg = big;
        void* argv[] = {&arg, nullptr};
        for (size_t i = 0; i < nn; i++) kp[i].kernelParams = argv;
        auto one = [&](int it) {
            arg.p[0] = (void*)(uintptr_t)it;
            for (size_t i = 0; i < nn; i++) CK(hipGraphExecKernelNodeSetParams(ge, nodes[i], &kp[i]));
            CK(hipGraphLaunch(ge, sa));
        };
        for (int i = 0; i < 50; i++) one(i);
        CK(hipDeviceSynchronize());
        auto t = clk::now();
        for (int i = 0; i < NB; i++) one(i);
        const double host = us_since(t);
        CK(hipDeviceSynchronize());
        const double all = us_since(t);
        // launch only (no updates), same graph
        auto t2 = clk::now();
        for (int i = 0; i < NB; i++) CK(hipGraphLaunch(ge, sa));
        const double host2 = us_since(t2);
        CK(hipDeviceSynchronize());
        printf("updated graph: %d kernels, host %.2f us/batch with updates (%.2f us launch only), device done %.2f us/batch\n",
               (int)nn, host / NB, host2 / NB, all / NB);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    // the rest of a batch's host calls: a 2 MB pinned H2D copy, an event record, a cross-stream wait
    {
        void* hpin;
        void* dbuf;
        CK(hipHostMalloc(&hpin, 2 << 20, 0));
        CK(hipMalloc(&dbuf, 2 << 20));
        auto t = clk::now();
        for (int i = 0; i < NB; i++) CK(hipMemcpyAsync(dbuf, hpin, 2 << 20, hipMemcpyHostToDevice, sb));
        const double h1 = us_since(t);
        CK(hipDeviceSynchronize());
        t = clk::now();
        for (int i = 0; i < NB; i++) {
            CK(hipEventRecord(ea, sa));
            CK(hipStreamWaitEvent(sb, ea, 0));
        }
        const double h2 = us_since(t);
        CK(hipDeviceSynchronize());
        t = clk::now();
        for (int i = 0; i < NB; i++) (void)hipEventQuery(ea);
        const double h3 = us_since(t);
        printf("host: 2 MB H2D memcpyAsync %.2f us, event record + stream wait %.2f us, event query %.2f us\n", h1 / NB,
               h2 / NB, h3 / NB);
    }
    int h = 0;
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    printf("counter %d\n", h);
    return 0;
}
