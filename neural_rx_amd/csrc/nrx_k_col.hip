// nrx_k_col.hip -- the whole-column register-resident launches (k_init_col, k_update_col;
// nrx_col.inc), one code object of their own; called by the f16 24-row tier's launch loop
// (Launch<P16>::run) for the stages the schedule mask gives them (nrx_update_schedule).
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

#include "nrx_rr.inc"
#include "nrx_col.inc"

bool col_init_applicable(const FwdArgs<_Float16, float, _Float16>& a) {
  // 4 rx antennas (2A = A2P = 8: z chunk 0 = [y | h | pe | 0]); Var-IO: one launch per StateInit m
  return 2 * a.A == 8 && a.init_cinp == 32;
}

bool update_col_applicable(const FwdArgs<_Float16, float, _Float16>& a, bool gz, bool last, int sched) {
  // conv1 reads [a | s | pe] from memory (GZ): a = the other user's act*sp plane (U = 2), none
  // (U = 1) or the a_u plane the combine pass wrote (U > 2); a grid wider than one column only
  // with kSchedColWide (44-output strips measured slower than the RR launch at cfg3 / cfg5)
  const int chp = 2 * a.A <= 16 ? 16 : 32;
  if (!gz || 2 * a.A > 32) return false;
  if (col_strips(a.F) > 1 && !(sched & kSchedColWide)) return false;
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
  // the last StateInit launch runs iteration 0's aggregation MLP (TAIL_AGG), earlier ones (Var-IO) none
  const bool agg = bp.tail == TAIL_AGG;
  if (items <= grid) {
    if (agg) k_init_col<TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
    else k_init_col<TAIL_NONE><<<grid, 512, kColLds, st>>>(bp, items);
  } else {
    if (agg) k_init_col_multi<TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
    else k_init_col_multi<TAIL_NONE><<<grid, 512, kColLds, st>>>(bp, items);
  }
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
  // one item per workgroup (the single-column BASELINE shapes) or the looping kernel
  const bool one = items <= grid;
  if (last) {
    if (ch32) {
      if (one) k_update_col<32, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
      else k_update_col_multi<32, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
    } else {
      if (one) k_update_col<16, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
      else k_update_col_multi<16, TAIL_READOUT_WB><<<grid, 512, kColLds, st>>>(bp, items);
    }
  } else {
    if (ch32) {
      if (one) k_update_col<32, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
      else k_update_col_multi<32, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
    } else {
      if (one) k_update_col<16, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
      else k_update_col_multi<16, TAIL_AGG><<<grid, 512, kColLds, st>>>(bp, items);
    }
  }
  return hipGetLastError();
}

// the one-launch column forward (k_fwd_col): U <= 2 (no combine stage), one StateInit over 2A = 8,
// GZ conv1 (workspace below 1 GB), one LLR head whose readout fits, at most one item per CU and
// stage (every item stages its weights), a device whose XCDs hold equal CU counts
bool fwd_col_applicable(const FwdArgs<_Float16, float, _Float16>& a, int num_it, const FusedCtl& fc) {
  // fc.enabled == 0 (NRX_FUSED=0, nrx_fused_config(h, 0, ..)): no one-launch forward of any kind
  if (!fc.sync || !fc.enabled || !(fc.update_rr & kSchedColFwd)) return false;
  const int cus = cu_count(), nx = xcc_count();
  if (nx < 1 || nx > 8 || cus % nx != 0) return false;
  const long items = (long)a.B * a.U * col_strips(a.F);
  return a.U <= kInlineUsers && a.num_init == 1 && col_init_applicable(a) && a.ws_bytes < kGzOob && a.pe16 &&
         a.H == 1 &&
         rr_heads_fit(a.bits_max, 16, 2 * a.A) && items <= cus && num_it >= 1 && 1 + num_it <= kColMaxStages &&
         a.B <= kFusedMaxB;
}

hipError_t launch_fwd_col(const FwdArgs<_Float16, float, _Float16>& args, const ModelW<_Float16, float>& W, int num_it,
                          hipStream_t st, Prof* prof, const FusedCtl& fc) {
  auto B_ = [&](int kid) { if (prof) prof->begin(kid, st); };
  auto E_ = [&](int kid) { if (prof) prof->end(kid, st); };
  ColFwdParams fp{};
  fp.sync = reinterpret_cast<FusedSync*>(fc.sync);
  fp.nst = 1 + num_it;
  fp.nq = xcc_count();
  fp.spin_limit = fc.spin_limit;
  fp.dbg_err = fc.dbg_err;
  const int nq = args.F * kT * 2 * args.A / 4;
  const bool norm_pre = nq > kNormFusedMaxQ;
  if (norm_pre) {
    B_(K_NORM);
    k_norm<<<args.B, 1024, 0, st>>>(args.y, nq, args.norm);
    E_(K_NORM);
  }
  FwdArgs<_Float16, float, _Float16> a = args;
  for (int s = 0; s < fp.nst; ++s) {
    BlockParams<P16>& bp = fp.st[s];
    bp.inline_combine = 1;
    bp.pair = 0;
    bp.order_rev = 0;
    bp.norm_pre = norm_pre;
    bp.strips = col_strips(args.F);
    bp.m = 0;
    bp.gz = 1;
    bp.llr[0][0] = W.llr[0][0];
    bp.llr[0][1] = W.llr[0][1];
    bp.chest[0] = W.chest[0];
    bp.chest[1] = W.chest[1];
    if (s == 0) {
      for (int l = 0; l < 3; ++l) bp.w[l] = W.init[0][l];
      bp.tail = TAIL_AGG;
      bp.agg[0] = W.agg[0][0];
      bp.agg[1] = W.agg[0][1];
    } else {
      std::swap(a.s_in, a.s_out);
      std::swap(a.a, a.a_out);
      const int i = s - 1;
      for (int l = 0; l < 3; ++l) bp.w[l] = W.upd[i][l];
      const bool last = i == num_it - 1;
      bp.tail = last ? TAIL_READOUT_WB : TAIL_AGG;
      if (!last) {
        bp.agg[0] = W.agg[i + 1][0];
        bp.agg[1] = W.agg[i + 1][1];
      }
    }
    bp.a = a;
  }
  col_stamp_select(st);
  B_(K_FWD_COL);
  k_fwd_col<16><<<cu_count(), 512, kColLds, st>>>(fp);
  E_(K_FWD_COL);
  return hipGetLastError();
}

hipError_t setup_col() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kColLds);
    if (r != hipSuccess) e = r;
  };
  set((const void*)k_init_col<TAIL_AGG>);
  set((const void*)k_init_col<TAIL_NONE>);
  set((const void*)k_init_col_multi<TAIL_AGG>);
  set((const void*)k_init_col_multi<TAIL_NONE>);
  set((const void*)k_update_col<16, TAIL_AGG>);
  set((const void*)k_update_col<32, TAIL_AGG>);
  set((const void*)k_update_col<16, TAIL_READOUT_WB>);
  set((const void*)k_update_col<32, TAIL_READOUT_WB>);
  set((const void*)k_update_col_multi<16, TAIL_AGG>);
  set((const void*)k_update_col_multi<32, TAIL_AGG>);
  set((const void*)k_update_col_multi<16, TAIL_READOUT_WB>);
  set((const void*)k_update_col_multi<32, TAIL_READOUT_WB>);
  set((const void*)k_fwd_col<16>);
  return e;
}

}  // namespace nrx

#ifdef NRX_STAMPS
extern "C" int nrx_debug_col_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nrx::g_nrx_rr_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif
