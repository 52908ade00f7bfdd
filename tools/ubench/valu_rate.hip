// Microbenchmark (diagnostic only): issue cost of the depthwise VALU forms on gfx950,
// alone and interleaved with v_mfma_f32_16x16x32_f16, at 1 and 2 waves per SIMD.
// Prints cycles per loop iteration (s_memtime, wave 0) for each variant.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MODE, int NV, int NM>
__global__ void kern(float* out, long long* cyc, int iters) {
  half2_t a[8], b[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = half2_t{(_Float16)(threadIdx.x * 0.001f + i), (_Float16)0.5f};
    b[i] = half2_t{(_Float16)0.999f, (_Float16)1.001f};
  }
  float fa[8], fb[8];
  for (int i = 0; i < 8; ++i) { fa[i] = threadIdx.x * 0.001f + i; fb[i] = 0.999f; }
  half8 ma = half8{1, 1, 1, 1, 1, 1, 1, 1}, mb = ma;
  floatx4 acc[4] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ma, mb, acc[m & 3], 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int k = v & 7;
      if constexpr (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(fa[k]) : "v"(fb[k]), "v"(fb[(k + 1) & 7]));
      if constexpr (MODE == 1) asm volatile("v_pk_fma_f16 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]));
      if constexpr (MODE == 2) asm volatile("v_pk_fmac_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]));
      if constexpr (MODE == 3) asm volatile("v_pk_mul_f16 %0, %1, %2" : "=v"(a[k]) : "v"(b[k]), "v"(a[(k + 1) & 7]));
      if constexpr (MODE == 4) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(fa[k]) : "v"(fb[k]), "v"(fb[(k + 1) & 7]));
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += (float)a[i].x + fa[i];
  for (int m = 0; m < 4; ++m) s += acc[m][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  // block wall: first start .. last end over the block's waves (lane 0 of each wave)
  __shared__ long long st[16], en[16];
  if ((threadIdx.x & 63) == 0) { st[threadIdx.x >> 6] = t0; en[threadIdx.x >> 6] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long a = st[0], b = en[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { a = st[w] < a ? st[w] : a; b = en[w] > b ? en[w] : b; }
    cyc[blockIdx.x] = b - a;
  }
}

template <int MODE, int NV, int NM>
void run(const char* name, int waves_per_simd) {
  const int iters = 2000;
  const int blocks = 256;
  const int threads = 256 * waves_per_simd;   // 4 SIMDs x waves
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&cyc, blocks * 8);
  hipFuncSetAttribute((const void*)kern<MODE, NV, NM>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  kern<MODE, NV, NM><<<blocks, threads, 96 * 1024>>>(out, cyc, 10);   // 96 KB LDS: 1 block per CU
  hipDeviceSynchronize();
  kern<MODE, NV, NM><<<blocks, threads, 96 * 1024>>>(out, cyc, iters);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  // per SIMD: waves_per_simd waves each doing NV VALU + NM MFMA per iteration
  printf("%-28s waves/SIMD %d  VALU/iter %2d MFMA/iter %d : %7.1f SIMD cyc/iter  (%5.2f per wave-VALU, %5.2f per wave-MFMA)\n",
         name, waves_per_simd, NV, NM, m / iters, NV ? m / iters / (NV * waves_per_simd) : 0.0,
         NM ? m / iters / (NM * waves_per_simd) : 0.0);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run<0, 16, 0>("v_fma_f32", w);
    run<1, 16, 0>("v_pk_fma_f16", w);
    run<2, 16, 0>("v_pk_fmac_f16_dpp", w);
    run<3, 16, 0>("v_pk_mul_f16", w);
    run<4, 16, 0>("v_fmac_f32_dpp", w);
    run<0, 0, 8>("mfma16x16x32 only", w);
    run<1, 16, 8>("mfma x8 + pk_fma x16", w);
    run<2, 16, 8>("mfma x8 + pk_fmac_dpp x16", w);
    run<2, 32, 8>("mfma x8 + pk_fmac_dpp x32", w);
    run<0, 16, 8>("mfma x8 + fma_f32 x16", w);
    run<2, 36, 8>("mfma x8 + pk_fmac_dpp x36", w);
    run<2, 36, 4>("mfma x4 + pk_fmac_dpp x36", w);
  }
  return 0;
}
