// Largest by-value kernel argument the runtime accepts (diagnostic): a kernel whose argument
// is a struct of N ints sums them; the host compares with the expected sum for N = 1 K .. 8 K
// ints (4 .. 32 KB).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
struct Arg {
  int v[N];
};

template <int N>
__global__ void k_sum(Arg<N> a, long long* out) {
  long long s = 0;
  for (int i = threadIdx.x; i < N; i += 64) s += a.v[i];
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (threadIdx.x == 0) out[0] = s;
}

template <int N>
static void one(long long* d) {
  Arg<N> a;
  long long want = 0;
  for (int i = 0; i < N; ++i) {
    a.v[i] = i * 7 + 1;
    want += a.v[i];
  }
  hipMemset(d, 0, 8);
  k_sum<N><<<1, 64>>>(a, d);
  hipError_t e = hipDeviceSynchronize();
  long long got = 0;
  hipMemcpy(&got, d, 8, hipMemcpyDeviceToHost);
  printf("arg %6d bytes: %s (%s)\n", (int)sizeof(a), got == want ? "ok" : "WRONG", hipGetErrorString(e));
}

int main() {
  long long* d = nullptr;
  hipMalloc(&d, 8);
  one<512>(d);
  one<1024>(d);
  one<1536>(d);
  one<2048>(d);
  one<4096>(d);
  hipFree(d);
  return 0;
}
