// nrx_k_p64.hip -- the parity-mode (f32 storage, f64 MFMA) three-launch forward, one code
// object of its own.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t run_tier_p64(const FwdArgs<double, double, float>& a, const ModelW<double, double>& W, int num_it,
                        hipStream_t st, Prof* prof) {
  return Launch<P64>::run(a, W, num_it, st, prof);
}

hipError_t setup_tier_p64() { return Launch<P64>::setup(); }

}  // namespace nrx
