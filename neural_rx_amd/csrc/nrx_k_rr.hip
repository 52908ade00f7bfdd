// nrx_k_rr.hip -- the register-resident UpdateState launch (k_update_rr, nrx_rr.inc), one code
// object of its own; called by the f16 24-row tier's launch loop (Launch<P16>::run) for the
// update stages it applies to.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

#include "nrx_rr.inc"

bool update_rr_applicable(const FwdArgs<_Float16, float, _Float16>& a, bool gz, bool inline_combine, bool last) {
  // conv1 reads [a | s | pe] from memory: a = the other user's act*sp plane (U = 2, inline
  // combine), none (U = 1) or the a_u plane the combine pass wrote (U > 2); see gz_make
  (void)inline_combine;
  const int chp = 2 * a.A <= 16 ? 16 : 32;
  if (!gz || 2 * a.A > 32) return false;
  return !last || (a.H == 1 && rr_heads_fit(a.bits_max, chp, 2 * a.A));
}

hipError_t launch_update_rr(const BlockParams<P16>& bp0, bool last, hipStream_t st) {
  BlockParams<P16> bp = bp0;
  bp.strips = (bp.a.F + kRrFO - 1) / kRrFO;
  bp.pair = 0;
  const int items = bp.a.B * bp.a.U * bp.strips;
  const int grid = items < cu_count() ? items : cu_count();
  const bool ch32 = 2 * bp.a.A > 16;
#ifdef NRX_STAMPS
  {
    // NRX_STAMP_RR = i: stamp the i-th RR launch of the process (0-based)
    static int launch_no = 0;
    static const int sel = getenv("NRX_STAMP_RR") ? atoi(getenv("NRX_STAMP_RR")) : -1;
    const int on = launch_no++ == sel;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_nrx_stamp_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, st);
  }
#endif
  if (last) {
    if (ch32) k_update_rr<32, TAIL_READOUT_WB><<<grid, 512, kRrLds, st>>>(bp, items);
    else k_update_rr<16, TAIL_READOUT_WB><<<grid, 512, kRrLds, st>>>(bp, items);
  } else {
    if (ch32) k_update_rr<32, TAIL_AGG><<<grid, 512, kRrLds, st>>>(bp, items);
    else k_update_rr<16, TAIL_AGG><<<grid, 512, kRrLds, st>>>(bp, items);
  }
  return hipGetLastError();
}

hipError_t setup_update_rr() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kRrLds);
    if (r != hipSuccess) e = r;
  };
  set((const void*)k_update_rr<16, TAIL_AGG>);
  set((const void*)k_update_rr<32, TAIL_AGG>);
  set((const void*)k_update_rr<16, TAIL_READOUT_WB>);
  set((const void*)k_update_rr<32, TAIL_READOUT_WB>);
  return e;
}

}  // namespace nrx

#ifdef NRX_STAMPS
extern "C" int nrx_debug_rr_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nrx::g_nrx_rr_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
