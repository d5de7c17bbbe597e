// lane_xchg.hpp — the value of lane (lane ^ J) of a wave64, without an LDS round trip where the
// hardware has a lane path: J = 1, 2 quad permutes, J = 4, 8 row shifts (DPP), J = 16, 32 the
// gfx950 permlane swaps. Checked against __shfl_xor by tools/probes/xchg_probe.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wq {

template <int J>
__device__ __forceinline__ uint32_t xchg_u32(uint32_t v, int lane) {
    static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "xor distance");
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4 || J == 8) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x100 + J, 0xF, 0xF, false);  // row_shl: v[l + J]
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x110 + J, 0xF, 0xF, false);  // row_shr: v[l - J]
        return (lane & J) ? dn : up;
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}

template <int J>
__device__ __forceinline__ uint64_t xchg_u64(uint64_t v, int lane) {
    const uint32_t lo = xchg_u32<J>((uint32_t)v, lane), hi = xchg_u32<J>((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

}  // namespace wq
