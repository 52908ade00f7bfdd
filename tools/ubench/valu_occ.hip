// Microbenchmark (diagnostic only, round 3): VALU issue rate vs waves per SIMD, the MFMA
// shapes that could carry the depthwise 3x3 (4x4x4 16-block f16) and the VALU slots left
// beside 16x16x32 vs 32x32x16 f16 MFMAs.  Prints cycles per loop iteration (s_memtime,
// block wall) per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// MODE: 0 v_fma_f32, 1 v_pk_fma_f16, 2 v_pk_fmac_f16_dpp
// MM:   0 mfma 16x16x32 f16, 1 mfma 32x32x16 f16, 2 mfma 4x4x4 16-block f16
template <int MODE, int NV, int MM, int NM>
__global__ void kern(float* out, long long* cyc, int iters) {
  half2_t a[16], b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    a[i] = half2_t{(_Float16)(threadIdx.x * 0.001f + i), (_Float16)0.5f};
    b[i] = half2_t{(_Float16)0.999f, (_Float16)1.001f};
  }
  float fa[16], fb[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { fa[i] = threadIdx.x * 0.001f + i; fb[i] = 0.999f; }
  half8 ma = half8{1, 1, 1, 1, 1, 1, 1, 1}, mb = ma;
  half4_t qa = half4_t{1, 1, 1, 1}, qb = qa;
  floatx4 acc[4] = {};
  floatx16 acc32[2] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int v = 0; v < (NV > NM ? NV : NM); ++v) {
      if (v < NM) {
        if constexpr (MM == 0) acc[v & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ma, mb, acc[v & 3], 0, 0, 0);
        if constexpr (MM == 1) acc32[v & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ma, mb, acc32[v & 1], 0, 0, 0);
        if constexpr (MM == 2) acc[v & 3] = __builtin_amdgcn_mfma_f32_4x4x4f16(qa, qb, acc[v & 3], 0, 0, 0);
      }
      // spread the VALU ops evenly between the MFMAs
#pragma unroll
      for (int s = 0; s < (NM ? (NV + NM - 1) / NM : NV); ++s) {
        const int vi = NM ? v * ((NV + NM - 1) / NM) + s : s;
        if (NM == 0 && v > 0) break;
        if (vi >= NV) break;
        const int k = vi & 15;
        if constexpr (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(fa[k]) : "v"(fb[k]), "v"(fb[(k + 1) & 15]));
        if constexpr (MODE == 1) asm volatile("v_pk_fma_f16 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 15]));
        if constexpr (MODE == 2) asm volatile("v_pk_fmac_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 15]));
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += (float)a[i].x + fa[i];
  for (int m = 0; m < 4; ++m) s += acc[m][0];
  s += acc32[0][0] + acc32[1][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  __shared__ long long st[32], en[32];
  if ((threadIdx.x & 63) == 0) { st[threadIdx.x >> 6] = t0; en[threadIdx.x >> 6] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long x = st[0], y = en[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { x = st[w] < x ? st[w] : x; y = en[w] > y ? en[w] : y; }
    cyc[blockIdx.x] = y - x;
  }
}

template <int MODE, int NV, int MM, int NM>
void run(const char* name, int waves_per_simd) {
  const int iters = 1000;
  const int blocks = 256;
  const int threads = 256 * waves_per_simd;
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, blocks * threads * 4);
  (void)hipMalloc(&cyc, blocks * 8);
  (void)hipFuncSetAttribute((const void*)kern<MODE, NV, MM, NM>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  kern<MODE, NV, MM, NM><<<blocks, threads, 96 * 1024>>>(out, cyc, 10);
  (void)hipDeviceSynchronize();
  kern<MODE, NV, MM, NM><<<blocks, threads, 96 * 1024>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  long long h[256];
  (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  const double per = m / iters;
  printf("%-34s w/SIMD %d VALU %2d MFMA %2d : %8.1f cyc/iter  %5.2f per VALU-slot  %6.2f per MFMA (all waves)\n", name,
         waves_per_simd, NV, NM, per, NV ? per / (NV * waves_per_simd) : 0.0, NM ? per / (NM * waves_per_simd) : 0.0);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  const int ws[3] = {1, 2, 4};
  for (int wi = 0; wi < 3; ++wi) {
    const int w = ws[wi];
    run<0, 64, 0, 0>("v_fma_f32 x64", w);
    run<1, 64, 0, 0>("v_pk_fma_f16 x64", w);
    run<2, 64, 0, 0>("v_pk_fmac_f16_dpp x64", w);
    run<0, 0, 0, 16>("mfma16x16x32 x16", w);
    run<0, 0, 1, 8>("mfma32x32x16 x8", w);
    run<0, 0, 2, 16>("mfma4x4x4_16b x16", w);
    run<2, 72, 0, 16>("16x16x32 x16 + dpp x72", w);
    run<2, 72, 1, 8>("32x32x16 x8 + dpp x72", w);
    run<2, 32, 0, 16>("16x16x32 x16 + dpp x32", w);
    run<2, 48, 1, 8>("32x32x16 x8 + dpp x48", w);
  }
  return 0;
}
