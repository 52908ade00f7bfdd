// nrx_k_fwd2.hip -- k_forward MODE 2 instantiations (nrx_device.inc, "fused forward"), one
// code object of their own.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t launch_kforward_m2(int a2p, const FusedParams<P16>& fp, int grid, hipStream_t st) {
  constexpr int L = fused_lds<P16>();
  if (a2p == 32) { k_forward<P16, 32, 32, 2><<<grid, 512, L, st>>>(fp); return hipGetLastError(); }
  if (a2p == 8) k_forward<P16, 8, 16, 2><<<grid, 512, L, st>>>(fp);
  else if (a2p == 16) k_forward<P16, 16, 16, 2><<<grid, 512, L, st>>>(fp);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t setup_kforward_m2() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, fused_lds<P16>());
    if (r != hipSuccess) e = r;
  };
  set((const void*)k_forward<P16, 8, 16, 2>);
  set((const void*)k_forward<P16, 16, 16, 2>);
  set((const void*)k_forward<P16, 32, 32, 2>);
  return e;
}

}  // namespace nrx
