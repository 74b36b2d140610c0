// Checks kernels.hip's lane_xor32<J> (DPP / permlane swaps) against __shfl_xor for J = 1..32 on
// random data, on the device.
// Build: hipcc -O3 --offload-arch=gfx950 tools/xorbench.hip -o tools/bin/xorbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "../foundationdb_amd/csrc/lane_xor.h"

template <int J>
__global__ void k_check(const uint32_t* in, uint32_t* out_dpp, uint32_t* out_ref) {
    const uint32_t v = in[blockIdx.x * 64 + threadIdx.x];
    out_dpp[blockIdx.x * 64 + threadIdx.x] = fdbcs::lane_xor32<J>(v);
    out_ref[blockIdx.x * 64 + threadIdx.x] = (uint32_t)__shfl_xor((int)v, J, 64);
}

template <int J>
int check() {
    const int n = 64 * 64;
    std::vector<uint32_t> h(n), a(n), b(n);
    for (int i = 0; i < n; i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x9e3779b9u;
    uint32_t *d, *da, *db;
    hipMalloc(&d, 4 * n); hipMalloc(&da, 4 * n); hipMalloc(&db, 4 * n);
    hipMemcpy(d, h.data(), 4 * n, hipMemcpyHostToDevice);
    k_check<J><<<64, 64>>>(d, da, db);
    hipMemcpy(a.data(), da, 4 * n, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), db, 4 * n, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; i++) bad += a[i] != b[i];
    printf("J=%2d mismatches %d\n", J, bad);
    hipFree(d); hipFree(da); hipFree(db);
    return bad;
}

int main() {
    int bad = check<1>() + check<2>() + check<4>() + check<8>() + check<16>() + check<32>();
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
