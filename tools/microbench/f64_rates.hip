// Microbenchmark: FP64 MFMA vs FP64 VALU throughput on gfx950, and whether the
// two pipes overlap when MFMA waves and VALU waves share a CU. Also verifies the
// v_mfma_f64_16x16x4_f64 operand/accumulator lane maps with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

template<int NACC>
__device__ __forceinline__ void mfma_loop(int iters, double a, double b, double* out){
  d4 acc[NACC];
  #pragma unroll
  for(int i=0;i<NACC;i++) acc[i] = d4{0,0,0,0};
  for(int it=0; it<iters; ++it){
    #pragma unroll
    for(int i=0;i<NACC;i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0,0,0);
  }
  double s=0;
  #pragma unroll
  for(int i=0;i<NACC;i++) s += acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3];
  out[blockIdx.x*blockDim.x+threadIdx.x] = s;
}
__device__ __forceinline__ void valu_loop(int iters, double a, double b, double* out){
  double x[8];
  #pragma unroll
  for(int i=0;i<8;i++) x[i]=a*(i+1);
  for(int it=0; it<iters; ++it){
    #pragma unroll
    for(int r=0;r<4;r++){
    #pragma unroll
    for(int i=0;i<8;i++) x[i] = __builtin_fma(x[i], b, a);
    }
  }
  double s=0;
  #pragma unroll
  for(int i=0;i<8;i++) s+=x[i];
  out[blockIdx.x*blockDim.x+threadIdx.x] = s;
}
__global__ void k_mfma(int iters, double a, double b, double* out){ mfma_loop<4>(iters,a,b,out); }
__global__ void k_valu(int iters, double a, double b, double* out){ valu_loop(iters,a,b,out); }
// 512 threads: waves 0-3 MFMA, waves 4-7 VALU
__global__ void k_mixed(int iters_m, int iters_v, double a, double b, double* out){
  int w = threadIdx.x/64;
  if(w<4) mfma_loop<4>(iters_m,a,b,out); else valu_loop(iters_v,a,b,out);
}
__global__ void k_layout(const double* A, const double* B, double* D){
  int l = threadIdx.x;
  // A is 16x4 row-major, B is 4x16 row-major; guide: lane l holds A[l&15][l>>4], B[l>>4][l&15]
  double a = A[(l&15)*4 + (l>>4)];
  double b = B[(l>>4)*16 + (l&15)];
  d4 acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0,0,0);
  for(int r=0;r<4;r++) D[l*4+r] = acc[r];
}

int main(){
  double* out; CK(hipMalloc(&out, 1<<26));
  hipEvent_t e0,e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int nblk = 256*4; int iters = 4000;
  // layout check
  {
    std::vector<double> A(64), B(64), D(256);
    for(int i=0;i<16;i++) for(int k=0;k<4;k++) A[i*4+k] = i*4+k+1;
    for(int k=0;k<4;k++) for(int j=0;j<16;j++) B[k*16+j] = (k+1)*100 + j*j;
    double *dA,*dB,*dD; CK(hipMalloc(&dA,512)); CK(hipMalloc(&dB,512)); CK(hipMalloc(&dD,2048));
    CK(hipMemcpy(dA,A.data(),512,hipMemcpyHostToDevice)); CK(hipMemcpy(dB,B.data(),512,hipMemcpyHostToDevice));
    k_layout<<<1,64>>>(dA,dB,dD); CK(hipMemcpy(D.data(),dD,2048,hipMemcpyDeviceToHost));
    int bad_guide=0, bad_f32=0;
    for(int l=0;l<64;l++) for(int r=0;r<4;r++){
      int col=l&15;
      int row_g=(l>>4)+4*r, row_f=(l>>4)*4+r;
      double ref_g=0, ref_f=0;
      for(int k=0;k<4;k++){ ref_g += A[row_g*4+k]*B[k*16+col]; ref_f += A[row_f*4+k]*B[k*16+col]; }
      if(ref_g!=D[l*4+r]) bad_guide++;
      if(ref_f!=D[l*4+r]) bad_f32++;
    }
    printf("{\"layout_mismatch_row=(l>>4)+4r\": %d, \"layout_mismatch_row=(l>>4)*4+r\": %d}\n", bad_guide, bad_f32);
  }
  for(int rep=0; rep<2; rep++){
    // MFMA: 256 threads/block (4 waves, one per SIMD), 4 blocks per CU
    k_mfma<<<nblk,256>>>(10,1.0,1.0,out); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); k_mfma<<<nblk,256>>>(iters,1e-3,0.999,out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms,e0,e1));
    double fl = (double)nblk*4*iters*4*2048.0;
    printf("{\"kernel\":\"mfma_f64_16x16x4\", \"ms\": %.3f, \"TFLOPs\": %.2f}\n", ms, fl/ms/1e9);
    double t_m = ms;
    k_valu<<<nblk,256>>>(10,1.0,1.0,out); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); k_valu<<<nblk,256>>>(iters,1e-3,0.999,out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms,e0,e1));
    double flv = (double)nblk*256*iters*32*2.0;
    printf("{\"kernel\":\"valu_fma_f64\", \"ms\": %.3f, \"TFLOPs\": %.2f}\n", ms, flv/ms/1e9);
    // mixed: choose iters so each half alone would take about the same time
    int itv = (int)(iters * (double)ms/t_m * 0 + iters); // same iteration count; report combined
    CK(hipEventRecord(e0)); k_mixed<<<nblk/2,512>>>(iters,itv,1e-3,0.999,out); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms,e0,e1));
    double flm = (double)(nblk/2)*4*iters*4*2048.0 + (double)(nblk/2)*256*itv*32*2.0;
    printf("{\"kernel\":\"mixed_mfma+valu\", \"ms\": %.3f, \"TFLOPs\": %.2f}\n", ms, flm/ms/1e9);
  }
  return 0;
}
