// Microbenchmark (diagnostic only): LDS store / load throughput on gfx950 with the strip
// image's swizzled addressing, 8 waves (one 512-thread workgroup per CU, all CUs busy).
// Modes: 0 ds_write_b64 in the in-place epilogue pattern (lane (t,g): chunk 2n + (g>>1),
// half (g&1)); 1 ds_write_b128 (lane (t,g): chunk 4j + ck); 2 ds_read_b128 (conv row read:
// lane (t,g) chunk 4kc + g); 3 = mode 0 with 2 rows of VALU-free stores interleaved with
// MFMAs of the other wave (not used).  Prints bytes per cycle per CU (s_memtime, wave span).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int intx2 __attribute__((ext_vector_type(2)));
typedef int intx4 __attribute__((ext_vector_type(4)));

// global -> LDS DMA (global_load_lds_dwordx4) from an L2-resident 64 KB buffer: each wave
// fills 8 x 1 KB per iteration (the LDS write side of weight staging by DMA)
__global__ __launch_bounds__(512) void kern_dma(long long* cyc, const intx4* src, int iters) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  typedef __attribute__((address_space(3))) void lds_void;
  typedef const __attribute__((address_space(1))) void glb_void;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int n = 0; n < 8; ++n)
      __builtin_amdgcn_global_load_lds((glb_void*)(src + (wave * 8 + n) * 64 + lane), (lds_void*)(lds + (wave * 8 + n) * 1024), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  __shared__ long long st[8], en[8];
  if (lane == 0) { st[wave] = t0; en[wave] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long lo = st[0], hi = en[0];
    for (int w = 1; w < 8; ++w) { lo = st[w] < lo ? st[w] : lo; hi = en[w] > hi ? en[w] : hi; }
    cyc[blockIdx.x] = hi - lo;
  }
}

template <int MODE>
__global__ __launch_bounds__(512) void kern(long long* cyc, int* sink, int iters) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds + wave * 4 * 4096;
  unsigned a[8];
  for (int n = 0; n < 8; ++n) {
    if (MODE == 0) a[n] = base + (t * 16 + ((2 * n + (g >> 1)) ^ t)) * 16 + (g & 1) * 8;
    if (MODE == 1) a[n] = base + (t * 16 + ((4 * (n & 3) + 2 * (g & 1) + (g >> 1)) ^ t)) * 16 + (n >> 2) * 4096;
    if (MODE == 2) a[n] = base + (t * 16 + ((4 * (n & 3) + g) ^ t)) * 16 + (n >> 2) * 4096;
    if (MODE == 3 || MODE == 6 || MODE == 7) a[n] = base + lane * 16 + n * 1024;
    if (MODE == 4) a[n] = base + lane * 8 + n * 512;
    if (MODE == 5) a[n] = base + lane * 4 + n * 256;
  }
  intx4 v4 = intx4{lane, wave, 1, 2};
  intx2 v2 = intx2{lane, wave};
  intx4 acc = intx4{0, 0, 0, 0};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  const bool on = MODE != 6 || wave < 4;
  for (int it = 0; it < iters && on; ++it) {
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      if constexpr (MODE == 3 || MODE == 6) asm volatile("ds_write_b128 %0, %1" ::"v"(a[n]), "v"(v4) : "memory");
      if constexpr (MODE == 4) asm volatile("ds_write_b64 %0, %1" ::"v"(a[n]), "v"(v2) : "memory");
      if constexpr (MODE == 5) asm volatile("ds_write_b32 %0, %1" ::"v"(a[n]), "v"(lane) : "memory");
      if constexpr (MODE == 7) {
        intx4 r;
        asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a[n]) : "memory");
        acc += r;
      }
      if constexpr (MODE == 0) asm volatile("ds_write_b64 %0, %1" ::"v"(a[n]), "v"(v2) : "memory");
      if constexpr (MODE == 1) asm volatile("ds_write_b128 %0, %1" ::"v"(a[n]), "v"(v4) : "memory");
      if constexpr (MODE == 2) {
        intx4 r;
        asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a[n]) : "memory");
        acc += r;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  __shared__ long long st[8], en[8];
  if (lane == 0) { st[wave] = t0; en[wave] = t1; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long lo = st[0], hi = en[0];
    for (int w = 1; w < 8; ++w) { lo = st[w] < lo ? st[w] : lo; hi = en[w] > hi ? en[w] : hi; }
    cyc[blockIdx.x] = hi - lo;
  }
}

template <int MODE>
static void run(const char* name, int bytes_per_instr) {
  const int blocks = 256, iters = 2000;
  long long* cyc;
  int* sink;
  (void)hipMalloc(&cyc, blocks * sizeof(long long));
  (void)hipMalloc(&sink, blocks * 512 * sizeof(int));
  const int L = 8 * 4 * 4096;
  (void)hipFuncSetAttribute((const void*)kern<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, L);
  for (int rep = 0; rep < 2; ++rep) kern<MODE><<<blocks, 512, L>>>(cyc, sink, iters);
  (void)hipDeviceSynchronize();
  long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += (double)h[i];
  m /= blocks;
  const double bytes = 8.0 * iters * 8 * bytes_per_instr;   // 8 waves x iters x 8 instructions
  printf("%-34s %8.1f B/cycle/CU  (%.1f cycles per instruction per CU)\n", name, bytes / m,
         m / (8.0 * iters * 8));
  (void)hipFree(cyc);
  (void)hipFree(sink);
}

static void run_dma() {
  const int blocks = 256, iters = 500;
  long long* cyc;
  intx4* src;
  (void)hipMalloc(&cyc, blocks * sizeof(long long));
  (void)hipMalloc(&src, 64 * 1024);
  (void)hipMemset(src, 0, 64 * 1024);
  const int L = 64 * 1024;
  (void)hipFuncSetAttribute((const void*)kern_dma, hipFuncAttributeMaxDynamicSharedMemorySize, L);
  for (int rep = 0; rep < 2; ++rep) kern_dma<<<blocks, 512, L>>>(cyc, src, iters);
  (void)hipDeviceSynchronize();
  long long h[256];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += (double)h[i];
  m /= blocks;
  printf("%-34s %8.1f B/cycle/CU\n", "global_load_lds_dwordx4 (L2 hits)", 8.0 * iters * 8 * 1024 / m);
  (void)hipFree(cyc);
  (void)hipFree(src);
}

int main() {
  run_dma();
  run<0>("ds_write_b64 (in-place pattern)", 512);
  run<1>("ds_write_b128 (chunk pattern)", 1024);
  run<2>("ds_read_b128 (conv row pattern)", 1024);
  run<3>("ds_write_b128 (linear)", 1024);
  run<4>("ds_write_b64 (linear)", 512);
  run<5>("ds_write_b32 (linear)", 256);
  run<6>("ds_write_b128 (linear, 4 waves = 1/SIMD)", 512);   // half the waves: bytes/2
  run<7>("ds_read_b128 (linear)", 1024);
  return 0;
}
