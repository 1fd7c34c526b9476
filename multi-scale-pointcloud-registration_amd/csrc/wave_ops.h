// wave_ops.h — wave-wide reductions on gfx950 (DPP row ops + readlane, no LDS).
#pragma once
#include <hip/hip_runtime.h>

namespace orpcd {

// all-reduce within each row of 16 lanes: quad_perm[1,0,3,2], quad_perm[2,3,0,1],
// row_half_mirror, row_mirror
template <typename Op>
__device__ __forceinline__ unsigned row_reduce(unsigned v, Op op) {
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false));
    return v;
}
// max of non-negative float bit patterns (or any uint) over the wave -> SGPR
__device__ __forceinline__ unsigned wave_umax(unsigned v) {
    v = row_reduce(v, [](unsigned a, unsigned b) { return a > b ? a : b; });
    const unsigned r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const unsigned r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    const unsigned a = r0 > r1 ? r0 : r1, b = r2 > r3 ? r2 : r3;
    return a > b ? a : b;
}
__device__ __forceinline__ float wave_fmax(float x) {
    unsigned v = row_reduce(__float_as_uint(x), [](unsigned a, unsigned b) {
        return __float_as_uint(fmaxf(__uint_as_float(a), __uint_as_float(b)));
    });
    return fmaxf(fmaxf(__uint_as_float(__builtin_amdgcn_readlane(v, 0)), __uint_as_float(__builtin_amdgcn_readlane(v, 16))),
                 fmaxf(__uint_as_float(__builtin_amdgcn_readlane(v, 32)), __uint_as_float(__builtin_amdgcn_readlane(v, 48))));
}
__device__ __forceinline__ float wave_fmin(float x) { return -wave_fmax(-x); }

}  // namespace orpcd
