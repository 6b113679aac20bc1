// armour-mi355x — wave64 data movement on gfx950 without the LDS crossbar.
//
// ds_bpermute (what __shfl / __shfl_xor compile to) goes through the LDS pipeline, about a hundred
// cycles per dependent step. The PZ engine's wave-level sorts, scans and reductions are long
// dependent chains of such steps, so they use DPP and the CDNA4 permlane swaps instead:
//   xor 1, 2        DPP quad_perm
//   xor 4, 8        DPP row_shl / row_shr by 4 or 8, selected by the lane bit
//   xor 16          v_permlane16_swap (rows 0<->1, 2<->3)
//   xor 32          v_permlane32_swap (halves)
//   lane +-1        DPP row_shl:1 / row_shr:1, row-boundary lanes patched from v_readlane
//                   (the DPP wave_shl / wave_shr controls assemble for gfx950 but do not shift)
// 64-bit values move as two 32-bit halves. tests/test_gpu_wave.py checks every primitive against
// __shfl on the device.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace armour {

#define WAVE_FN __device__ inline __attribute__((always_inline))

WAVE_FN int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// partner value at lane ^ m, m in {1, 2, 4, 8, 16, 32} (m uniform; a constant after unrolling)
WAVE_FN uint32_t xor_u32(uint32_t v, int m) {
    const int l = lane_id();
    switch (m) {
        case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        case 4: {
            const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
            const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
            return (l & 4) ? dn : up;
        }
        case 8: {
            const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xF, 0xF, false);  // row_shl:8
            const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
            return (l & 8) ? dn : up;
        }
        case 16: {
            const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (l & 16) ? p[0] : p[1];
        }
        default: {
            const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (l & 32) ? p[0] : p[1];
        }
    }
}
WAVE_FN uint64_t xor_u64(uint64_t v, int m) {
    const uint32_t lo = xor_u32((uint32_t)v, m), hi = xor_u32((uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
WAVE_FN double xor_f64(double v, int m) { return __builtin_bit_cast(double, xor_u64(__builtin_bit_cast(uint64_t, v), m)); }
WAVE_FN int xor_i32(int v, int m) { return (int)xor_u32((uint32_t)v, m); }

// value of lane + 1 (lane 63: 0) and of lane - 1 (lane 0: 0)
WAVE_FN uint32_t next_u32(uint32_t v) {
    const int l = lane_id();
    uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, true);  // row_shl:1
    const uint32_t b16 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t b32 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t b48 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    r = l == 15 ? b16 : r;
    r = l == 31 ? b32 : r;
    r = l == 47 ? b48 : r;
    return r;
}
WAVE_FN uint32_t prev_u32(uint32_t v) {
    const int l = lane_id();
    uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    const uint32_t b15 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t b31 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t b47 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    r = l == 16 ? b15 : r;
    r = l == 32 ? b31 : r;
    r = l == 48 ? b47 : r;
    return r;
}
WAVE_FN double next_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = ((uint64_t)next_u32((uint32_t)(b >> 32)) << 32) | next_u32((uint32_t)b);
    return __builtin_bit_cast(double, r);
}
WAVE_FN uint64_t prev_u64(uint64_t v) { return ((uint64_t)prev_u32((uint32_t)(v >> 32)) << 32) | prev_u32((uint32_t)v); }

// butterfly sum: every lane gets the same total (fixed association, deterministic)
WAVE_FN double wave_sum(double v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = v + xor_f64(v, m);
    return v;
}
WAVE_FN int wave_max(int v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = max(v, xor_i32(v, m));
    return v;
}

// inclusive prefix sum over the wave (DPP row shifts, then row broadcasts)
WAVE_FN int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false); // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false); // row_bcast:31 into rows 2, 3
    return v;
}

}  // namespace armour
