// Microbenchmark (diagnostic only): VALU + MFMA co-issue on one gfx950 SIMD.
// Each wave runs, per loop iteration, NM MFMAs interleaved with NV v_pk_fmac_f16_dpp
// (NV / NM VALU after each MFMA), all hand-ordered in inline asm.  Variants:
//   OP 0: v_mfma_f32_16x16x32_f16, A/B/C in VGPRs
//   OP 1: v_mfma_f32_16x16x32_f16, A/B in VGPRs, C/D in AGPRs
//   OP 2: v_mfma_f32_16x16x32_f16, A/B/C in AGPRs
//   OP 3: v_mfma_f32_32x32x16_f16, A/B in VGPRs, C/D in AGPRs (16 accumulators)
// Prints SIMD cycles per iteration (s_memtime, block wall) at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int OP>
__device__ __forceinline__ void mfma(floatx4 (&acc)[4], floatx16 (&acc32)[2], int m, half8 a, half8 b) {
  if constexpr (OP == 0) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc[m & 3]) : "v"(a), "v"(b));
  if constexpr (OP == 1) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[m & 3]) : "v"(a), "v"(b));
  if constexpr (OP == 2) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[m & 3]) : "a"(a), "a"(b));
  if constexpr (OP == 3) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc32[m & 1]) : "v"(a), "v"(b));
}

template <int OP, int NV, int NM, bool BLOCK = false>
__global__ void kern(float* out, long long* cyc, int iters) {
  half2_t x[8], w[8];
  for (int i = 0; i < 8; ++i) {
    x[i] = half2_t{(_Float16)(threadIdx.x * 0.001f + i), (_Float16)0.5f};
    w[i] = half2_t{(_Float16)0.999f, (_Float16)1.001f};
  }
  half8 ma = half8{1, 1, 1, 1, 1, 1, 1, 1}, mb = ma;
  floatx4 acc[4] = {};
  floatx16 acc32[2] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (BLOCK) {
      // block form (as the conv kernel's compiled stream): all VALU, then all MFMAs
#pragma unroll
      for (int v = 0; v < NV; ++v)
        asm volatile("v_pk_fmac_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                     : "+v"(x[v & 7]) : "v"(w[v & 7]), "v"(w[(v + 1) & 7]));
#pragma unroll
      for (int m = 0; m < NM; ++m) mfma<OP>(acc, acc32, m, ma, mb);
      continue;
    }
#pragma unroll
    for (int m = 0; m < (NM > 0 ? NM : 1); ++m) {
      if constexpr (NM > 0) mfma<OP>(acc, acc32, m, ma, mb);
      constexpr int PER = NM > 0 ? NV / NM : NV;
#pragma unroll
      for (int v = 0; v < PER; ++v) {
        const int k = (m * PER + v) & 7;
        asm volatile("v_pk_fmac_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                     : "+v"(x[k]) : "v"(w[k]), "v"(w[(k + 1) & 7]));
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += (float)x[i].x;
  for (int m = 0; m < 4; ++m) s += acc[m][0];
  s += acc32[0][0] + acc32[1][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  __shared__ long long st[16], en[16];
  if ((threadIdx.x & 63) == 0) { st[threadIdx.x >> 6] = t0; en[threadIdx.x >> 6] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long a = st[0], b = en[0];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) { a = st[q] < a ? st[q] : a; b = en[q] > b ? en[q] : b; }
    cyc[blockIdx.x] = b - a;
  }
}

template <int OP, int NV, int NM, bool BLOCK = false>
void run(const char* name, int wps) {
  const int iters = 2000, blocks = 256, threads = 256 * wps;
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&cyc, blocks * 8);
  hipFuncSetAttribute((const void*)kern<OP, NV, NM, BLOCK>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  kern<OP, NV, NM, BLOCK><<<blocks, threads, 96 * 1024>>>(out, cyc, 10);
  hipDeviceSynchronize();
  kern<OP, NV, NM, BLOCK><<<blocks, threads, 96 * 1024>>>(out, cyc, iters);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-34s waves/SIMD %d VALU/iter %2d MFMA/iter %d : %7.1f SIMD cyc/iter per wave %6.1f\n", name, wps, NV, NM,
         m / iters, m / iters / wps);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 2; w <= 2; ++w) {
    // the conv chunk of one wave (R = 4 rows, 128 outputs): 144 VALU + 32 MFMA 16x16x32
    run<0, 144, 32, true>("chunk block m16 vgpr", w);
    run<0, 144, 32>("chunk interleaved m16 vgpr", w);
    run<1, 144, 32>("chunk interleaved m16 acc-agpr", w);
    run<3, 144, 16, true>("chunk block m32", w);
    run<3, 144, 16>("chunk interleaved m32", w);
    // 64-output layer (conv3): 144 VALU + 16 MFMA
    run<0, 144, 16, true>("conv3 chunk block m16", w);
    run<0, 144, 16>("conv3 chunk interleaved m16", w);
    run<3, 144, 8>("conv3 chunk interleaved m32", w);
  }
  for (int w = 1; w <= 2; ++w) {
    run<0, 36, 0>("valu only x36", w);
    run<0, 0, 8>("m16 vgpr only x8", w);
    run<1, 0, 8>("m16 acc-agpr only x8", w);
    run<3, 0, 4>("m32 acc-agpr only x4", w);
    run<0, 32, 8>("m16 vgpr x8 + valu x32", w);
    run<1, 32, 8>("m16 acc-agpr x8 + valu x32", w);
    run<2, 32, 8>("m16 all-agpr x8 + valu x32", w);
    run<3, 32, 4>("m32 acc-agpr x4 + valu x32", w);
    run<0, 32, 4>("m16 vgpr x4 + valu x32", w);
    run<1, 32, 4>("m16 acc-agpr x4 + valu x32", w);
    run<3, 32, 2>("m32 acc-agpr x2 + valu x32", w);
    run<1, 64, 8>("m16 acc-agpr x8 + valu x64", w);
  }
  return 0;
}
