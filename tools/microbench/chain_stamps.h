// Dev build only (tools/runs/gpu_r03_chain.sh): potrf_diag_kernel records its start and end
// wall clock (100 MHz) per block column, read back by gp2d_debug_chain_stamps.
#pragma once
#include <hip/hip_runtime.h>
__device__ unsigned long long gp2d_chain_stamp[2048];
#define GP2D_STAMP(slot)                                                                         \
  do {                                                                                           \
    if (((slot) == 0 || (slot) == 12) && threadIdx.x == 0)                                       \
      gp2d_chain_stamp[2 * (k0 / 128) + ((slot) == 12)] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
extern "C" int gp2d_debug_chain_stamps(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(gp2d_chain_stamp), sizeof(unsigned long long) * n);
}
