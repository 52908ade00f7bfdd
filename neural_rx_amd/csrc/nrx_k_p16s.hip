// nrx_k_p16s.hip -- the three-launch forward of the P16S strip tier (k_init / k_update /
// k_combine instantiations of nrx_device.inc), one code object of its own.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t run_tier_p16s(const FwdArgs<_Float16, float, _Float16>& a, const ModelW<_Float16, float>& W, int num_it,
                       hipStream_t st, Prof* prof) {
  return Launch<P16S>::run(a, W, num_it, st, prof);
}

hipError_t setup_tier_p16s() { return Launch<P16S>::setup(); }

}  // namespace nrx
