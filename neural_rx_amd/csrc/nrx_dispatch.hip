// nrx_dispatch.hip -- which schedule runs a forward (strip tier, one-launch k_forward or the
// three-launch path), the one-launch forward's status word, kernel attribute setup.  The
// kernels themselves live in the per-tier translation units nrx_k_*.hip.
#include "nrx_device.inc"
#include "nrx_launch.inc"

namespace nrx {

hipError_t launch_forward_f16(const FwdArgs<_Float16, float, _Float16>& args,
                              const ModelW<_Float16, float>& W, int num_it, hipStream_t st,
                              Prof* prof, const FusedCtl& fc) {
  if (NRX_SMALL_STRIPS != 0) {
    if (small_strips_fit<P16S>(args)) return run_tier_p16s(args, W, num_it, st, prof);
    if (small_strips_fit<P16M>(args)) return run_tier_p16m(args, W, num_it, st, prof);
  }
  if (fwd_col_applicable(args, num_it, fc)) return launch_fwd_col(args, W, num_it, st, prof, fc);
  if (fused_applicable<P16>(args, num_it, fc)) return run_fused<P16>(args, W, num_it, st, prof, fc);
  return run_tier_p16(args, W, num_it, st, prof, fc.update_rr);
}

// whether a forward takes a one-launch path (k_fwd_col or k_forward: the handle's counters, one
// stream at a time)
bool fused_would_run(const FwdArgs<_Float16, float, _Float16>& args, int num_it, const FusedCtl& fc) {
  if (NRX_SMALL_STRIPS != 0 && (small_strips_fit<P16S>(args) || small_strips_fit<P16M>(args))) return false;
  return fwd_col_applicable(args, num_it, fc) || fused_applicable<P16>(args, num_it, fc);
}

size_t fused_sync_bytes() { return kFusedSyncBytes; }

// {error word, items that waited, polls} of the fused forward since the last reset.  Blocking:
// the handle's event recorded behind its last one-launch forward is waited for first (ADVICE r04:
// an event the handle owns, never the caller's stream, which may have been destroyed since), so
// the read and the reset never race with a k_forward in flight; reset clears the three words.
hipError_t fused_sync_status(void* sync, int* st, bool reset, hipEvent_t last) {
  FusedSync* sy = reinterpret_cast<FusedSync*>(sync);
  hipError_t e = last ? hipEventSynchronize(last) : hipSuccess;
  if (e == hipSuccess) e = hipMemcpy(st, &sy->err, 3 * sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) e = hipMemset(&sy->err, 0, 3 * sizeof(int));
  if (e == hipSuccess && reset) e = hipDeviceSynchronize();
  return e;
}

hipError_t launch_forward_f64(const FwdArgs<double, double, float>& args,
                              const ModelW<double, double>& W, int num_it, hipStream_t st,
                              Prof* prof) {
  return run_tier_p64(args, W, num_it, st, prof);
}

hipError_t setup_kernels() {
  (void)cu_count();
  (void)xcc_count();
  const hipError_t es[] = {setup_tier_p16(),     setup_tier_p16m(),    setup_tier_p16s(),   setup_tier_p64(),
                           setup_kforward_m0(), setup_kforward_m1(), setup_kforward_m2(), setup_update_rr(),
                           setup_col()};
  for (hipError_t e : es)
    if (e != hipSuccess) return e;
  return hipSuccess;
}

int strip_width(int precision) { return precision == 0 ? P16::FO : P64::FO; }

// Device probe of the buffer range check the GZ z-row loader relies on (tests only): one
// raw_buffer_load_dword per lane through a descriptor of `records` bytes at `base`, with the
// lane offset voff + 4 lane in voffset and `soff` in soffset.  Out-of-range loads return 0.  The
// caller keeps base + voff + soff + 256 inside its own allocation, so no outcome can fault.
static __global__ void k_probe_buffer_oob(const char* base, unsigned records, unsigned voff, unsigned soff,
                                          unsigned* out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, (int)records,
                                                                     0x00020000);
  out[threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(r, voff + 4u * threadIdx.x, (int)soff, 0);
}

}  // namespace nrx

extern "C" int nrx_probe_buffer_oob(const void* base, uint32_t records, uint32_t voff, uint32_t soff, uint32_t* out,
                                    void* stream) {
  nrx::k_probe_buffer_oob<<<1, 64, 0, (hipStream_t)stream>>>((const char*)base, records, voff, soff, out);
  return (int)hipGetLastError();
}
