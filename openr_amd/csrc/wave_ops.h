// Wave-wide scans and reductions with DPP moves (shared by the BFS kernels).
//
// row_shr 1/2/4/8 inside each 16-lane row (lanes shifted in from outside the
// row read 0 -- the identity of +, | and max over unsigned values), then
// row_bcast15 / row_bcast31 carry the row results upwards; lane 63 ends with
// the whole wave's.  __shfl compiles to ds_bpermute, one LDS round trip per
// step (msbfs_kernel<10>'s per-slice record made 18 of them in a dependent
// chain).  Every lane of the wave must be active.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace spfi {

#define SPF_DPP_STEPS(OP)                                                        \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true)); \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true)); \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true)); \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true)); \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false)); \
  x = OP(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));
__device__ __forceinline__ uint32_t dpp_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t dpp_or(uint32_t a, uint32_t b) { return a | b; }
__device__ __forceinline__ uint32_t dpp_max(uint32_t a, uint32_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t* total) {
  const uint32_t own = x;
  SPF_DPP_STEPS(dpp_add)
  *total = __builtin_amdgcn_readlane(x, 63);
  return x - own;
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
  SPF_DPP_STEPS(dpp_or)
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t x) {
  SPF_DPP_STEPS(dpp_max)
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
  return ((uint64_t)wave_or32((uint32_t)(x >> 32)) << 32) | wave_or32((uint32_t)x);
}

}  // namespace spfi
