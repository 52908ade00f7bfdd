// Microbenchmark (diagnostic only): VALU throughput vs waves per SIMD and chain count.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
template <int MODE, int CH>
__global__ void kern(float* out, long long* cyc, int iters) {
  float f[CH];
  half2_t h[CH];
  for (int i = 0; i < CH; ++i) { f[i] = threadIdx.x * 1e-3f + i; h[i] = half2_t{(_Float16)(0.1f * i), (_Float16)0.2f}; }
  const float m = 0.999f; const half2_t hm = half2_t{(_Float16)0.999f, (_Float16)0.999f};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if constexpr (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[k]) : "v"(m));
      else asm volatile("v_pk_fma_f16 %0, %0, %1, %1" : "+v"(h[k]) : "v"(hm));
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  __shared__ long long st[16], en[16];
  if ((threadIdx.x & 63) == 0) { st[threadIdx.x >> 6] = t0; en[threadIdx.x >> 6] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long a = st[0], b = en[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { a = st[w] < a ? st[w] : a; b = en[w] > b ? en[w] : b; }
    cyc[blockIdx.x] = b - a;
  }
  float s = 0;
  for (int i = 0; i < CH; ++i) s += f[i] + (float)h[i].x;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int MODE, int CH>
void run(int wps) {
  const int iters = 1000, blocks = 256, threads = 256 * wps;
  float* out; long long* cyc;
  (void)hipMalloc(&out, blocks * threads * 4); (void)hipMalloc(&cyc, blocks * 8);
  (void)hipFuncSetAttribute((const void*)kern<MODE, CH>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  kern<MODE, CH><<<blocks, threads, 96 * 1024>>>(out, cyc, 10);
  kern<MODE, CH><<<blocks, threads, 96 * 1024>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  long long h[256]; (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (int i = 0; i < blocks; ++i) m += h[i]; m /= blocks;
  printf("%s chains %2d waves/SIMD %d: %.2f SIMD cycles per VALU\n", MODE ? "v_pk_fma_f16" : "v_fma_f32   ", CH, wps,
         m / iters / (CH * wps));
  (void)hipFree(out); (void)hipFree(cyc);
}
int main() {
  run<0, 8>(1); run<0, 16>(1); run<0, 32>(1); run<0, 8>(2); run<0, 16>(2); run<0, 16>(4);
  run<1, 8>(1); run<1, 16>(1); run<1, 32>(1); run<1, 16>(2); run<1, 16>(4);
  return 0;
}
