// nrx_k_p16.hip -- the three-launch forward of the P16 strip tier (k_init / k_update /
// k_combine instantiations of nrx_device.inc), one code object of its own.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t run_tier_p16(const FwdArgs<_Float16, float, _Float16>& a, const ModelW<_Float16, float>& W, int num_it,
                       hipStream_t st, Prof* prof, int update_rr) {
  return Launch<P16>::run(a, W, num_it, st, prof, update_rr);
}

hipError_t setup_tier_p16() { return Launch<P16>::setup(); }

}  // namespace nrx

#ifdef NRX_STAMPS
extern "C" int nrx_debug_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nrx::g_nrx_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
