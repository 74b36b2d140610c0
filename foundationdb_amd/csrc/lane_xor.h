// lane_xor.h — cross-lane exchange of a wave64 value with lane (lane ^ J) on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdbcs {

// The value of lane (lane ^ J), without the LDS crossbar (ds_bpermute) for J < 16: DPP quad
// permutes for 1 and 2, a half-row mirror then a quad reversal for 4, a row rotation by 8 for 8;
// gfx950's permlane16 / permlane32 swaps (an exchange between neighbouring rows / halves) for 16
// and 32.  tools/xorbench.hip checks every J against __shfl_xor on the device.
template <int J>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const int m = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, m, 0x1B, 0xF, 0xF, false);     // quad_perm [3,2,1,0]
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {
        static_assert(J == 32, "lane_xor32: J in 1..32");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
#else
    return v;
#endif
}
template <int J>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
    return (uint64_t)lane_xor32<J>((uint32_t)(v >> 32)) << 32 | lane_xor32<J>((uint32_t)v);
}
__device__ __forceinline__ uint64_t lane_xor64_rt(uint64_t v, int j) {  // j folds once unrolled
    switch (j) {
        case 1: return lane_xor64<1>(v);
        case 2: return lane_xor64<2>(v);
        case 4: return lane_xor64<4>(v);
        case 8: return lane_xor64<8>(v);
        case 16: return lane_xor64<16>(v);
        default: return lane_xor64<32>(v);
    }
}

}  // namespace fdbcs
