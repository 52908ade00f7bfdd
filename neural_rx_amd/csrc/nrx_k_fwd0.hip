// nrx_k_fwd0.hip -- k_forward MODE 0 instantiations (nrx_device.inc, "fused forward"), one
// code object of their own.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t launch_kforward_m0(int a2p, const FusedParams<P16>& fp, int grid, hipStream_t st) {
  constexpr int L = fused_lds<P16>();

  if (a2p == 8) k_forward<P16, 8, 16, 0><<<grid, 512, L, st>>>(fp);
  else if (a2p == 16) k_forward<P16, 16, 16, 0><<<grid, 512, L, st>>>(fp);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t setup_kforward_m0() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, fused_lds<P16>());
    if (r != hipSuccess) e = r;
  };
  set((const void*)k_forward<P16, 8, 16, 0>);
  set((const void*)k_forward<P16, 16, 16, 0>);

  return e;
}

}  // namespace nrx

#ifdef NRX_STAMPS
extern "C" int nrx_debug_fused_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nrx::g_nrx_rr_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
