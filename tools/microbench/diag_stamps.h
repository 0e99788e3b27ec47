// diag_stamps.h — dev builds only (hipcc ... -include tools/microbench/diag_stamps.h, tools/runs/r05_diaginv.sh):
// GP2D_STAMP(slot) in potrf_diag_kernel records the cycle counter of workgroup 0's first thread
// per phase; tools/probe_diag.py reads them through gp2d_debug_diag_stamps.
#pragma once
#include <hip/hip_runtime.h>
__device__ unsigned long long gp2d_diag_stamps[16];
#define GP2D_STAMP(slot) \
  do { if (threadIdx.x == 0 && blockIdx.x == 0) gp2d_diag_stamps[slot] = __builtin_readcyclecounter(); } while (0)
extern "C" int gp2d_debug_diag_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(gp2d_diag_stamps), sizeof(gp2d_diag_stamps));
}
