// nrx_k_col.hip -- the whole-column register-resident launches (k_init_col, k_update_col;
// nrx_col.inc), one code object of their own; called by the f16 24-row tier's launch loop
// (Launch<P16>::run) for the stages the schedule mask gives them (nrx_update_schedule).
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

#include "nrx_rr.inc"
#include "nrx_col.inc"

bool col_init_applicable(const FwdArgs<_Float16, float, _Float16>& a) {
  // one StateInit (no Var-IO mix) over 4 rx antennas (2A = A2P = 8: z chunk 0 = [y | h | pe | 0])
  return a.num_init == 1 && 2 * a.A == 8 && a.init_cinp == 32;
}

bool update_col_applicable(const FwdArgs<_Float16, float, _Float16>& a, bool gz, bool last) {
  // conv1 reads [a | s | pe] from memory (GZ): a = the other user's act*sp plane (U = 2), none
  // (U = 1) or the a_u plane the combine pass wrote (U > 2)
  const int chp = 2 * a.A <= 16 ? 16 : 32;
  if (!gz || 2 * a.A > 32) return false;
  return !last || (a.H == 1 && rr_heads_fit(a.bits_max, chp, 2 * a.A));
}

static int col_grid(const BlockParams<P16>& bp, int* items) {
  *items = bp.a.B * bp.a.U * bp.strips;
  return *items < cu_count() ? *items : cu_count();
}

#ifdef NRX_STAMPS
static void col_stamp_select(hipStream_t st) {
  // NRX_STAMP_COL = i: stamp the i-th column launch of the process (0-based)
  static int launch_no = 0;
  static const int sel = getenv("NRX_STAMP_COL") ? atoi(getenv("NRX_STAMP_COL")) : -1;
  const int on = launch_no++ == sel;
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_nrx_stamp_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, st);
}
#else
static void col_stamp_select(hipStream_t) {}
#endif

hipError_t launch_init_col(const BlockParams<P16>& bp0, hipStream_t st) {
  BlockParams<P16> bp = bp0;
  bp.strips = col_strips(bp.a.F);
  bp.pair = 0;
  int items = 0;
  const int grid = col_grid(bp, &items);
  col_stamp_select(st);
  k_init_col<TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
  return hipGetLastError();
}

hipError_t launch_update_col(const BlockParams<P16>& bp0, bool last, hipStream_t st) {
  BlockParams<P16> bp = bp0;
  bp.strips = col_strips(bp.a.F);
  bp.pair = 0;
  int items = 0;
  const int grid = col_grid(bp, &items);
  const bool ch32 = 2 * bp.a.A > 16;
  col_stamp_select(st);
  if (last) {
    if (ch32) k_update_col<32, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
    else k_update_col<16, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
  } else {
    if (ch32) k_update_col<32, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
    else k_update_col<16, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
  }
  return hipGetLastError();
}

hipError_t setup_col() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kColLds);
    if (r != hipSuccess) e = r;
  };
  set((const void*)k_init_col<TAIL_AGG>);
  set((const void*)k_update_col<16, TAIL_AGG>);
  set((const void*)k_update_col<32, TAIL_AGG>);
  set((const void*)k_update_col<16, TAIL_READOUT_WB>);
  set((const void*)k_update_col<32, TAIL_READOUT_WB>);
  return e;
}

}  // namespace nrx

#ifdef NRX_STAMPS
extern "C" int nrx_debug_col_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nrx::g_nrx_rr_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
