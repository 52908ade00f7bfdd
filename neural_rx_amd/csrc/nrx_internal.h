// nrx_internal.h -- shared between the HIP kernels and the host side of libnrx.so.
//
// Device data layout (see DESIGN.md "Data layout in HBM"):
//   state / aggregate buffers  s, a : [B][U][F][14][56]   (compact, no padding in HBM;
//                                     the kernels pad T -> 16 and channels in LDS)
//   storage type: _Float16 (NRX_PREC_F16) or float (NRX_PREC_F32X)
// Packed weights (one blob per precision, built by nrx_create):
//   separable conv: dw [9][CINP] (tap = i*3 + j, i along F, j along T),
//                   pwT [COUTP][CINP] (transposed pointwise kernel), bias [COUTP]
//   dense:          wT [COUTP][CINP], bias [COUTP]
//   WT = _Float16 / double, BT = float / double.  Zero padding everywhere.
#pragma once
#include <stdint.h>

#include "../../include/nrx.h"

namespace nrx {

constexpr int kT = 14;        // OFDM symbols (fixed by 5G NR slot)
constexpr int kTP = 16;       // padded symbol axis = MFMA tile width
constexpr int kDS = 56;       // state width d_s
constexpr int kDSP = 64;      // padded state width
constexpr int kHID = 128;     // conv hidden width / readout hidden width
constexpr int kAGG = 64;      // aggregation hidden width
constexpr int kUPD_CINP = 128;  // [a, s, pe] = 114 -> 128
constexpr int kMaxInit = 8;
constexpr int kMaxIt = 8;
// users whose leave-one-out combine the update z-load forms itself (the other user's act*sp plane
// IS a_u for U = 2); U >= 3 runs the f32 combine pass (k_combine / combine stages) and every
// update reads its a_u plane -- one rounding for every U > 2 and every schedule, and conv1 can
// read a_u from memory (GZ) for any U
constexpr int kInlineUsers = 2;
constexpr int kMaxHeads = 8;
constexpr int kMaxUsers = 16;
constexpr int kHalo = 3;      // 3 stacked 3x3 convs per block
// f16 workspaces stay below this many bytes: conv1's z-row loader (struct GZ) addresses the
// workspace through one buffer descriptor with 32-bit offsets and marks zero chunks with offsets
// at or beyond it; a larger forward runs in slot chunks (nrx_api.cpp chunk_slots)
constexpr unsigned kGzRange = 0x40000000u;

// ---- LDS images of the f16 weights (kernels: SepStage / DenseStage).  A W^T [COUTP][CINP] image is a stack
// of 16-row tiles addressed like an activation image: element (co, chunk q of 8 inputs) at
// lds_off<NQ>(co >> 4, co & 15, q), NQ = CINP / 8 chunks per row, chunk index XOR-swizzled
// with the row so that a ds_read_b128 lane group hits distinct bank slots.
constexpr int kTPImg = 16;
__host__ __device__ constexpr int swz_q(int nq, int t) {
  return nq >= 16 ? (t & 15) : (nq == 8 ? ((t >> 1) & 7) : (nq == 4 ? ((t >> 2) & 3) : 0));
}
__host__ __device__ constexpr int lds_img_off(int nq, int row, int t, int q) {
  return ((row * kTPImg + t) * nq + (q ^ swz_q(nq, t))) * 16;
}
// separable layer: pw^T at 0 (<= 32 KB), dw [9][CINP] at kWPw, bias [COUTP] f32 at kWBias
constexpr int kWPw = kHID * kHID * 2;          // 32 KB
constexpr int kWDw = 9 * kHID * 2;             // 2304 B
constexpr int kWBias = kWPw + kWDw;            // conv bias [COUTP] f32
constexpr int kWTailBias = kWBias + kHID * 4;  // aggregation-MLP biases (2 x 64 f32)
constexpr int kWBytes = kWTailBias + 2 * kAGG * 4;
// readout heads (TAIL_READOUT_WB layout): LLR W1^T at 0, ChEst W1^T at kHW1C, biases, then
// the W2^T images truncated to their real rows
constexpr int kHW1C = 16 * 1024;                 // ChEst W1^T (LLR W1^T at 0)
constexpr int kHB1 = 32 * 1024;                  // b1: LLR [128] f32, ChEst [128] f32
constexpr int kHB2 = kHB1 + 2 * kHID * 4;        // b2: LLR [16] f32, ChEst [<= 32] f32
constexpr int kHW2 = kHB2 + (16 + 32) * 4;       // LLR W2^T rows [bits], then ChEst rows [2A]

template <class WT, class BT>
struct SepW {
  const WT* dw;
  const WT* pw;   // transposed [COUTP][CINP]
  const BT* b;
};

template <class WT, class BT>
struct DenseW {
  const WT* w;    // transposed [COUTP][CINP]
  const BT* b;
};

template <class WT, class BT>
struct ModelW {
  SepW<WT, BT> init[kMaxInit][3];
  DenseW<WT, BT> agg[kMaxIt][2];
  SepW<WT, BT> upd[kMaxIt][3];
  DenseW<WT, BT> llr[kMaxHeads][2];
  DenseW<WT, BT> chest[2];
};

// Shapes + pointers of one forward (kernel argument).
template <class WT, class BT, class S>
struct FwdArgs {
  int B, U, F, A, M, H;            // H = number of LLR heads
  int llr_B;                       // slots of the caller's llr tensor (the head stride; > B when
                                   // the forward runs in slot chunks, nrx_api.cpp)
  int init_cinp;                   // padded StateInit input width
  int num_init;
  int masking;
  int use_h;
  int bits_max;
  int head_bits[kMaxHeads];
  const float* y;                  // [B][F][T][2A]
  const float* pe;                 // [U][F][T][2]
  const float* h_hat;              // [B][U][F][T][2A] or null
  const float* active;             // [B][U]
  const float* mcs_mask;           // [B][U][M] or null
  float* llr;                      // [H][B][U][F][T][bits_max]
  float* h_ref;                    // [B][U][F][T][2A] or null
  double* norm;                    // [B] workspace
  S* s_in;                         // [B][U][F][14][56]
  S* s_out;
  S* a;                            // aggregate read by this update
  S* a_out;                        // aggregate written by the tail
  // one-launch forward (f16): the workspace as one buffer resource for conv1's z rows, and
  // the pe16 plane [U][F][14][56] (pe as f16 in channels 0, 1 of each 8-channel chunk 0;
  // written by the StateInit items, read as z chunk 14 by the update items' conv1)
  const char* ws_base;
  unsigned ws_bytes;
  S* pe16;
};

// The one-launch forward's control block (nrx_api.cpp fills it from the handle): the
// work-queue / counter buffer, whether the path may run (NRX_FUSED, read once at nrx_create),
// the dependency-wait bound and debug error bits (nrx_debug_fused).
struct FusedCtl {
  void* sync;
  int enabled;   // 0 off, 1 where measured faster (the bench-type schedule), 2 every applicable shape
  int spin_limit;
  int dbg_err;
  int update_rr;   // three-launch f16 forward: stage mask (nrx_update_schedule: 1 / 2 RR aggregation / readout,
                   // 4 / 8 column aggregation / readout, 16 column StateInit)
};
// schedule-mask bits of the three-launch f16 forward (nrx_update_schedule)
constexpr int kSchedRrAgg = 1, kSchedRrRo = 2, kSchedColAgg = 4, kSchedColRo = 8, kSchedColInit = 16;
constexpr int kSchedColFwd = 32;   // the one-launch column forward (k_fwd_col) where it applies
// bits 2 / 3 on grids wider than one 48-position column too (44-output strips with a halo; by
// default those grids keep the RR / strip updates, measured faster there: profiles/r06/configs)
constexpr int kSchedColWide = 64;
constexpr int kSchedMax = 127;
// default: the whole-column launches for every stage they apply to, the RR aggregation update
// where they do not (same-box A/B in profiles/r06/)
constexpr int kSchedDefault = kSchedColInit | kSchedColAgg | kSchedColRo | kSchedRrAgg;
constexpr int kFusedSpinLimit = 1 << 21;   // ~0.5 s of s_sleep 4 polls

// Optional per-kernel timing (nrx_profile_enable): events recorded around each launch on
// the launch stream.  Kernel ids:
enum KernelId {
  K_NORM = 0, K_INIT = 1, K_UPDATE = 2, K_FUSED = 3, K_UPDATE_RR = 4, K_COMBINE = 5, K_UPDATE_COL = 6, K_INIT_COL = 7,
  K_FWD_COL = 8, K_COUNT = 9
};

struct Prof {
  virtual void begin(int kid, void* stream) = 0;
  virtual void end(int kid, void* stream) = 0;
  virtual ~Prof() {}
};

// Aerial front/back-end (nrx_aerial.hip)
hipError_t launch_aerial_tables(const int32_t* ofdm_pos, const int32_t* sc_pos, int U, int nsym, int npil, int T,
                                int F, int32_t* nn, float* pe, hipStream_t st);
hipError_t launch_aerial_inputs(const float* y_re, const float* y_im, const float* h_re, const float* h_im,
                                const int32_t* nn, int B, int U, int F, int T, int A, int nsym, int npil, float* y,
                                float* h, hipStream_t st);
hipError_t launch_y_layout(const float* y0, const float* y1, int layout, int B, int F, int T, int A, float* y,
                           hipStream_t st);
hipError_t launch_aerial_llr(const float* llr, int B, int U, int F, int T, int bits_max, int bits, float* out,
                             hipStream_t st);

// Slot generator + error counters (nrx_synth.hip); struct types from include/nrx.h.
// gen_workspace_bytes(d, nullptr, nullptr) = workspace size.
struct GenWs;
size_t gen_workspace_bytes(const nrx_gen_desc& d, GenWs* w, char* base);
hipError_t launch_generate(const nrx_gen_desc& d, const nrx_gen_out& o, void* ws, hipStream_t st);
hipError_t launch_count_errors(const nrx_count_io& c, hipStream_t st);

hipError_t launch_llr_demap(const float* llr, int B, int U, int F, int T, int bits_stride, int bits,
                            const int32_t* data_re, int n_data, float* out, hipStream_t st);

}  // namespace nrx
