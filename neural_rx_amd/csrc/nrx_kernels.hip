// nrx_kernels.hip -- CDNA4 (gfx950) kernels of the CGNN neural-receiver forward pass.
//
// Reference semantics: CGNN.forward, neural_rx.py:544-595, with
// the TF structure of "neural_rx copy_pytorch.py" (StateInit :82-188, AggregateUserStates
// :191-231, UpdateState :234-287, ReadoutLLRs/ChEst :324-362).
//
// Kernel map (per forward: M_init + num_it launches):
//   k_init      StateInit: z=[y,pe,h] -> 3 separable convs       (copy_pytorch.py:160-188)
//               the slot normalisation 1/sqrt(mean(y^2)) (neural_rx.py:551-557) is computed
//               in its prologue (slot_norm)
//               one launch per init head m, accumulating the Var-IO mcs mix
//               (neural_rx.py:562-569); the last one runs the aggregation MLP of
//               iteration 0 in its conv3 epilogue and stores act_u * sp_u
//   k_update    z=[a,s,pe] -> 3 separable convs + skip           (copy_pytorch.py:267-287)
//               z-load forms the leave-one-out user mean from the act * sp rows
//               (neural_rx.py:135-207; U <= 2: LDS-DMA copy, U <= 4: register sum);
//               epilogue: next iteration's aggregation MLP, or after the last
//               iteration the LLR head(s) + ChEst head           (neural_rx.py:309-404)
//   k_combine   U > 4 only: the leave-one-out mean as its own pass
//
// Tiling.  The resource grid of one (slot, user) is an F x 16 image (T = 14 padded to 16
// with zero rows).  One MFMA tile = one subcarrier row: 16 symbols x 16 output channels.
// Lane l of a wave owns symbol t = l & 15 and channel group g = l >> 4 of the B operand
// (the activation), so the depthwise 3x3 of a lane needs its own column of three rows
// (f-1, f, f+1) from LDS plus the t +- 1 neighbours, which come from lanes l -+ 1 through
// DPP row shifts (row_shr/row_shl stay inside the 16-lane row = the symbol axis, and the
// bound control supplies the t = -1 / t = 16 zero padding).  The depthwise result is the
// MFMA B fragment directly (no LDS round trip); the transposed pointwise kernel is the A
// fragment.  Separable-conv stacks run strip-wise: a workgroup owns FO output subcarriers
// plus a 3-row halo on each side (3 stacked 3x3 convs), ping-ponging two LDS buffers.
//
// Precision policies:
//   P16: f16 storage, f16 packed depthwise (v_pk_fma_f16), mfma_f32_16x16x32_f16.
//   P64: f32 storage, f64 depthwise, mfma_f64_16x16x4f64 (parity mode).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "nrx_internal.h"

#ifndef NRX_ABLATE
#define NRX_ABLATE 0   // diagnostic builds only: 1 skip conv math, 2 skip z loads, 4 skip weight
                       // staging, 8 skip tails, 16 skip conv3 global epilogue, 32 skip the
                       // state stores, 64 skip the act*sp stores (MLP still computed), 128
                       // skip the aggregation MLP (stores kept)
#endif

namespace nrx {

#ifdef NRX_STAMPS
// diagnostic builds only: s_memtime per phase, wave 0 lane 0 of each workgroup
__device__ unsigned long long g_nrx_stamps[4096][64];
// set by the host for the k_update launch to record; __constant__ so that the flag is a
// scalar (SMEM) load and a stamp does not wait for the wave's outstanding vector loads
__constant__ int g_nrx_stamp_on;
// one-launch forward (g_nrx_stamp_on == 100): per item i < 8 of a workgroup, slots
// g_nrx_rr_stamps[wg][8 i + m]: 0 item start, 1 conv1 start, 2 conv1 end, 3 conv2 end,
// 4 conv3 epilogue start, 5 item body done, 6 signalled, 7 = stage + 1 (not a time)
__device__ unsigned long long g_nrx_rr_stamps[4096][64];
__device__ int g_fstamp_item[4096];
__device__ __forceinline__ void fstamp(int m) {
  if (threadIdx.x == 0 && g_nrx_stamp_on == 100) {
    const int wg = blockIdx.x, it = g_fstamp_item[wg];
    if (wg < 4096 && it < 8) g_nrx_rr_stamps[wg][8 * it + m] = __builtin_amdgcn_s_memtime();
  }
}
__device__ __forceinline__ void stamp(int k) {
  if (threadIdx.x == 0 && g_nrx_stamp_on) {
    const int wg = blockIdx.x;
    if (g_nrx_stamp_on == 100) {
      const int m = k == 1 ? 1 : k == 2 ? 2 : k == 3 ? 3 : k == 6 ? 4 : -1;
      if (m >= 0) fstamp(m);
    } else if (wg < 4096) {
      g_nrx_stamps[wg][k] = __builtin_amdgcn_s_memtime();
    }
  }
}
// per-wave stamp k + wave (lane 0 of every wave), k in {40, 48, 56}
__device__ __forceinline__ void stamp_w(int k) {
  if ((threadIdx.x & 63) == 0 && g_nrx_stamp_on) {
    const int wg = blockIdx.x;
    if (wg < 4096) g_nrx_stamps[wg][k + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();
  }
}
// register-resident kernels (own array): phase ph (0..31) of the workgroup's item ks == 1,
// for wave 0 (R = 3, no DMA duty) and wave 4 (R = 2, DMA issuer) of the same SIMD
__device__ __forceinline__ void rr_stamp(int ks, int ph) {
  if (ks == 1 && (threadIdx.x & 255) == 0 && g_nrx_stamp_on) {
    const int wg = blockIdx.x;
    if (wg < 4096) g_nrx_rr_stamps[wg][ph * 2 + (threadIdx.x >> 8)] = __builtin_amdgcn_s_memtime();
  }
}
#else
__device__ __forceinline__ void fstamp(int) {}
__device__ __forceinline__ void stamp(int) {}
__device__ __forceinline__ void stamp_w(int) {}
__device__ __forceinline__ void rr_stamp(int, int) {}
#endif

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2 __attribute__((ext_vector_type(2)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef int intx4 __attribute__((ext_vector_type(4)));
typedef int intx8 __attribute__((ext_vector_type(8)));

// Work-item id as an opaque value (one volatile asm per use): the one-launch forward runs
// the item code inside a loop, and LLVM's LICM hoisted every thread-index-derived address of
// every item body out of it -- ~70 values live across the whole loop, spilled to scratch and
// reloaded in the conv loops.  An opaque id per use keeps each derivation where it is used.
#ifndef NRX_OPAQUE_TID
#define NRX_OPAQUE_TID 2
#endif
__device__ __forceinline__ unsigned nrx_tid() {
  unsigned t = threadIdx.x;
  if (NRX_OPAQUE_TID == 1) asm volatile("" : "+v"(t));
  if (NRX_OPAQUE_TID == 2) asm("" : "+v"(t));   // CSE-able, not speculatable: not hoisted
  if (NRX_OPAQUE_TID) __builtin_assume(t < 1024);   // the range the compiler loses
  return t;
}

// DPP: lane l receives lane l-1 (row_shr:1) / lane l+1 (row_shl:1) inside its 16-lane
// row; the lane without a source gets 0 (bound_ctrl).
__device__ __forceinline__ int dpp_shr1(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_shl1(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true);
}

// d += x(t -+ 1) * w on packed halves: v_pk_fmac_f16 with a DPP row shift on x (the
// lane without a source reads 0: bound_ctrl).  The compiler's hazard recognizer covers
// inline asm (it inserts the VALU-write -> DPP-read wait states).
__device__ __forceinline__ void fmac_shr(half2& d, half2 x, half2 w) {
  asm("v_pk_fmac_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(d) : "v"(x), "v"(w));
}
__device__ __forceinline__ void fmac_shl(half2& d, half2 x, half2 w) {
  asm("v_pk_fmac_f16_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(d) : "v"(x), "v"(w));
}
// y * ns rounded to f32 before the storage conversion: without the barrier the compiler fuses
// the product and the f16 conversion into one single-rounding v_fma_mix in some kernels and
// not in others (1-ulp z differences between kernel families)
__device__ __forceinline__ float f32_rounded(float v) {
  asm("" : "+v"(v));
  return v;
}
__device__ __forceinline__ double f32_rounded(double v) { return v; }

__device__ __forceinline__ half2 h2(half8 v, int k) {
  return half2{v[2 * k], v[2 * k + 1]};
}

// FO_: output subcarriers per strip.  P16 (24) is the throughput shape; P16M (16) and P16S
// (8) are taken for grids that would leave CUs idle (batch-1 latency): more workgroups per
// slot, each with fewer rows (launch_forward_f16).
template <int FO_>
struct P16T {
  using S = _Float16;
  using WT = _Float16;
  using BT = float;
  using DV = half8;
  using Acc = floatx4;
  using Real = float;
  static constexpr int KC = 32;   // channels per K chunk (one MFMA K)
  static constexpr int CPL = 8;   // channels per lane per chunk
  static constexpr int EPC = 8;   // storage elements per 16-byte LDS chunk
  static constexpr int FO = FO_;  // output subcarriers per strip
  static constexpr int R = 4;     // consecutive subcarrier rows per wave pass
  static constexpr bool WLDS = true;  // stage each layer's weights in LDS
  __device__ static DV ld_lds(const char* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static DV ld_glb(const S* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static DV ld_w(const WT* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static Acc zero() { return Acc{0.f, 0.f, 0.f, 0.f}; }
  __device__ static Acc mma(const WT* a, DV b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const half8*>(a), b, c, 0, 0, 0);
  }
  __device__ static Acc mma_v(DV a, DV b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ static int co(int g, int j) { return 4 * g + j; }
  // accumulator-layout bias of output tile n (C operand of the first MFMA of a chain)
  __device__ static Acc bias_acc(const float* b, int n, int g) {
    return *reinterpret_cast<const floatx4*>(b + 16 * n + 4 * g);
  }
  // depthwise 3x3 of one output row from its three input rows (x0 = f-1, x1 = f, x2 = f+1);
  // tap = i*3 + j, i along subcarriers, j along symbols (j = 0 reads t-1).
  __device__ static DV dw_row(DV x0, DV x1, DV x2, const DV (&w)[9]) {
    // the centre column's contraction is fixed in the source (not left to the compiler,
    // which contracted it differently in different kernels: 1-ulp differences between
    // kernel families); the six side taps are inline-asm DPP FMACs on top of it
    const DV c = __builtin_elementwise_fma(w[7], x2, __builtin_elementwise_fma(w[4], x1, w[1] * x0));
    half2 d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[k] = h2(c, k);
      fmac_shr(d[k], h2(x0, k), h2(w[0], k));
      fmac_shr(d[k], h2(x1, k), h2(w[3], k));
      fmac_shr(d[k], h2(x2, k), h2(w[6], k));
      fmac_shl(d[k], h2(x0, k), h2(w[2], k));
      fmac_shl(d[k], h2(x1, k), h2(w[5], k));
      fmac_shl(d[k], h2(x2, k), h2(w[8], k));
    }
    return DV{d[0][0], d[0][1], d[1][0], d[1][1], d[2][0], d[2][1], d[3][0], d[3][1]};
  }
  __device__ static DV shr(DV v) {
    intx4 x = __builtin_bit_cast(intx4, v);
    x = intx4{dpp_shr1(x[0]), dpp_shr1(x[1]), dpp_shr1(x[2]), dpp_shr1(x[3])};
    return __builtin_bit_cast(DV, x);
  }
  __device__ static DV shl(DV v) {
    intx4 x = __builtin_bit_cast(intx4, v);
    x = intx4{dpp_shl1(x[0]), dpp_shl1(x[1]), dpp_shl1(x[2]), dpp_shl1(x[3])};
    return __builtin_bit_cast(DV, x);
  }
};

using P16 = P16T<24>;
using P16M = P16T<16>;
using P16S = P16T<8>;

struct P64 {
  using S = float;
  using WT = double;
  using BT = double;
  using DV = doublex4;
  using Acc = doublex4;
  using Real = double;
  static constexpr int KC = 16;
  static constexpr int CPL = 4;
  static constexpr int EPC = 4;
  static constexpr int FO = 8;
  static constexpr int R = 1;
  static constexpr bool WLDS = false;   // weights read from global (L2-resident)
  __device__ static DV ld_lds(const char* p) {
    floatx4 v = *reinterpret_cast<const floatx4*>(p);
    return DV{v[0], v[1], v[2], v[3]};
  }
  __device__ static DV ld_glb(const S* p) { return ld_lds(reinterpret_cast<const char*>(p)); }
  __device__ static DV ld_w(const WT* p) { return *reinterpret_cast<const doublex4*>(p); }
  __device__ static Acc zero() { return Acc{0.0, 0.0, 0.0, 0.0}; }
  __device__ static Acc mma(const WT* a, DV b, Acc c) {
    doublex4 av = *reinterpret_cast<const doublex4*>(a);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], b[3], c, 0, 0, 0);
    return c;
  }
  __device__ static Acc mma_v(DV av, DV b, Acc c) {
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], b[3], c, 0, 0, 0);
    return c;
  }
  __device__ static int co(int g, int j) { return g + 4 * j; }
  __device__ static DV dw_row(DV x0, DV x1, DV x2, const DV (&w)[9]) {
    const DV cm = w[0] * x0 + w[3] * x1 + w[6] * x2;
    const DV c0 = w[1] * x0 + w[4] * x1 + w[7] * x2;
    const DV cp = w[2] * x0 + w[5] * x1 + w[8] * x2;
    return c0 + shr(cm) + shl(cp);
  }
  __device__ static Acc bias_acc(const double* b, int n, int g) {
    return Acc{b[16 * n + g], b[16 * n + g + 4], b[16 * n + g + 8], b[16 * n + g + 12]};
  }
  __device__ static DV shr(DV v) {
    intx8 x = __builtin_bit_cast(intx8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = dpp_shr1(x[i]);
    return __builtin_bit_cast(DV, x);
  }
  __device__ static DV shl(DV v) {
    intx8 x = __builtin_bit_cast(intx8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = dpp_shl1(x[i]);
    return __builtin_bit_cast(DV, x);
  }
};

// ---------------------------------------------------------------- LDS image addressing
// Image [row][t (16)][NQ chunks of 16 B]; the chunk index is XOR-swizzled with the
// symbol so that the 16 lanes of a ds_read_b128 group (distinct t, same chunk) hit
// distinct bank slots.
template <int NQ>
__device__ __forceinline__ int swz(int t) {
  if constexpr (NQ >= 16) return t & 15;
  else if constexpr (NQ == 8) return (t >> 1) & 7;
  else if constexpr (NQ == 4) return (t >> 2) & 3;
  else return 0;
}
template <int NQ>
__device__ __forceinline__ int lds_off(int row, int t, int q) {
  return ((row * kTP + t) * NQ + (q ^ swz<NQ>(t))) * 16;
}
template <class P, int C>
__device__ __forceinline__ int lds_elem_off(int row, int t, int c) {
  constexpr int NQ = C * (int)sizeof(typename P::S) / 16;
  return lds_off<NQ>(row, t, c / P::EPC) + (c % P::EPC) * (int)sizeof(typename P::S);
}

template <class P>
__device__ __forceinline__ void lds_store(char* base, int off, typename P::Real v) {
  *reinterpret_cast<typename P::S*>(base + off) = (typename P::S)v;
}

// ------------------------------------------------ z rows straight from memory
// The z image of a k_forward update item, [a | s | pe] = chunks [0, 7) of the other user's
// act*sp plane, [7, 14) of the own state plane and chunk 14 of the pe16 plane (pe as f16,
// zero-padded to 8 channels), read by conv1 straight from L2 / HBM into its depthwise
// registers with buffer loads instead of being staged in the LDS strip image.  One buffer
// resource spans the workspace; lane (t, g) keeps, per K chunk kc, the byte offset of its
// 16-byte chunk q = 4 kc + g in grid row 0 (kGzOob for zero chunks: pad symbols, q = 15, the
// missing other user of U = 1), and a grid row adds f * kGzRow as the wave-uniform soffset
// (kGzOob for rows outside the grid).  Out-of-range buffer loads return zeros.
constexpr unsigned kGzOob = 0x40000000u;          // > any workspace this path is taken for
constexpr unsigned kGzRow = kT * kDS * 2;          // bytes per grid row of a state plane
struct GZ {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned off[4];   // per K chunk
  int f_start, F;
  half8 x0[6];       // K chunk 0 of the wave's R + 2 input rows, loaded in the item prologue
  __device__ unsigned row_soff(int slot) const {
    const int f = f_start + slot;
    return (f >= 0 && f < F) ? (unsigned)f * kGzRow : kGzOob;
  }
  __device__ half8 load(int kc, unsigned soff) const {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[kc], (int)soff, 0);
    return __builtin_bit_cast(half8, v);
  }
};

// ------------------------------------------------ depthwise 3x3 + pointwise on MFMA
// Strip image in LDS: slot (one subcarrier row) x 16 symbols x up to 128 channels, with a
// fixed slot pitch so that every layer of a block can run in place in one buffer.
template <class P>
constexpr int slot_pitch() { return kTP * kHID * (int)sizeof(typename P::S); }
template <class P, int NQ>
__device__ __forceinline__ int xoff(int slot, int t, int q) {
  return slot * slot_pitch<P>() + (t * NQ + (q ^ swz<NQ>(t))) * 16;
}

// Per-layer weight image in LDS (P16): layout constants kWPw .. kHW2 in nrx_internal.h
// (shared with the host, which packs the same images for the LDS-DMA of nrx_rr.inc).
// The paired readout tail gives WB the rest of the 160 KB LDS (P16: 160 KB - 30 x 4 KB) and
// stages the heads there, so that the strip image X is free for the next item's z DMA
// during the readout epilogue.  W1^T images in full; W2^T images truncated to their real
// rows (bits, 2A): the lanes of the padding rows read whatever follows, which only reaches
// output channels that are never stored.  One LLR head only.
constexpr int kWAlloc = 160 * 1024 - 30 * kTP * kHID * 2;
static_assert(kWBytes <= kWAlloc, "layer weight image exceeds the LDS left by the strip image");
// The truncated W2^T images put the LLR rows [0, bits_max) in the b2 slot of 16 outputs and
// the ChEst rows [0, 2A) in a CHP-row slot: bits_max <= 16 and 2A <= CHP <= 32 are
// required besides the byte budget (the padding rows the lanes read beyond the real ones
// only reach output channels that are never stored).
__host__ __device__ constexpr bool heads_fit_wb(int bits_max, int chp, int a2 = 0) {
  return bits_max <= 16 && a2 <= chp && chp <= 32 && kHW2 + 256 * (bits_max + chp) <= kWAlloc;
}

template <class P, int CINP, int COUTP>
struct WLds {
  const char* base;
  static constexpr int NQ = CINP * 2 / 16;
  __device__ typename P::DV afrag(int n, int kc, int lane, int g) const {
    return *reinterpret_cast<const half8*>(base + lds_off<NQ>(n, lane & 15, kc * 4 + g));
  }
  __device__ typename P::DV dwv(int tap, int kc, int g) const {
    return *reinterpret_cast<const half8*>(base + kWPw + (tap * CINP + kc * 32 + g * 8) * 2);
  }
  // the 9 taps of chunk kc from one opaque base register: the image sits ~155 KB into LDS,
  // beyond the 16-bit ds_read offset, so with a foldable base the compiler emits one v_add
  // per tap; hidden, every tap is an immediate offset (tap * CINP * 2 <= 2 KB)
  __device__ void dw_taps(int kc, int g, typename P::DV (&w)[9]) const {
    typedef const __attribute__((address_space(3))) char lds_char;
    typedef const __attribute__((address_space(3))) half8 lds_half8;
    unsigned p = (unsigned)(size_t)(lds_char*)(base + kWPw) + (unsigned)((kc * 32 + g * 8) * 2);
    asm volatile("" : "+v"(p));
    lds_char* q = (lds_char*)(size_t)p;
#pragma unroll
    for (int k = 0; k < 9; ++k) w[k] = *reinterpret_cast<lds_half8*>(q + k * CINP * 2);
  }
  __device__ typename P::Acc bias_acc(int n, int g) const {
    return P::bias_acc(reinterpret_cast<const float*>(base + kWBias), n, g);
  }
};

template <class P, int CINP, int COUTP>
struct WGlb {
  SepW<typename P::WT, typename P::BT> w;
  __device__ typename P::DV afrag(int n, int kc, int lane, int g) const {
    return P::ld_w(w.pw + (16 * n + (lane & 15)) * CINP + kc * P::KC + g * P::CPL);
  }
  __device__ typename P::DV dwv(int tap, int kc, int g) const {
    return P::ld_w(w.dw + tap * CINP + kc * P::KC + g * P::CPL);
  }
  __device__ void dw_taps(int kc, int g, typename P::DV (&w9)[9]) const {
#pragma unroll
    for (int k = 0; k < 9; ++k) w9[k] = dwv(k, kc, g);
  }
  __device__ typename P::Acc bias_acc(int n, int g) const { return P::bias_acc(w.b, n, g); }
};

// Cooperative copy of one separable layer's packed weights into the LDS image, split in
// a global-load half (issued one layer ahead, so its latency hides behind the current
// layer's math) and an LDS-store half.
template <int CINP, int COUTP>
struct SepStage {
  static constexpr int NQ = CINP * 2 / 16;
  static constexpr int NPW = COUTP * NQ;                 // W^T chunks
  static constexpr int NDW = 9 * NQ;                     // dw chunks
  static constexpr int NB = COUTP / 4;                   // bias chunks (4 floats)
  static constexpr int PER = (NPW + 511) / 512;
  intx4 v[PER];
  intx4 vx;
  __device__ void load(const SepW<_Float16, float>& w) {
    const int tid = nrx_tid();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + i * 512;
      if (idx < NPW) v[i] = *reinterpret_cast<const intx4*>(w.pw + (idx / NQ) * CINP + (idx % NQ) * 8);
    }
    vx = intx4{0, 0, 0, 0};
    if (tid < NDW) vx = reinterpret_cast<const intx4*>(w.dw)[tid];
    else if (tid - NDW < NB) vx = reinterpret_cast<const intx4*>(w.b)[tid - NDW];
  }
  __device__ void store(char* wb) const {
    const int tid = nrx_tid();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + i * 512;
      if (idx < NPW) {
        const int co = idx / NQ, q = idx % NQ;
        *reinterpret_cast<intx4*>(wb + lds_off<NQ>(co >> 4, co & 15, q)) = v[i];
      }
    }
    if (tid < NDW) reinterpret_cast<intx4*>(wb + kWPw)[tid] = vx;
    else if (tid - NDW < NB) reinterpret_cast<intx4*>(wb + kWPw + kWDw)[tid - NDW] = vx;
  }
};

// Same split for a dense layer: W^T image (K permuted on the host) + bias.
template <int CINP, int COUTP>
struct DenseStage {
  static constexpr int NQ = CINP * 2 / 16;
  static constexpr int NW = COUTP * NQ;
  static constexpr int PER = (NW + 511) / 512;
  intx4 v[PER];
  float bias;
  __device__ void load(const DenseW<_Float16, float>& w) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = nrx_tid() + i * 512;
      if (idx < NW) v[i] = *reinterpret_cast<const intx4*>(w.w + (idx / NQ) * CINP + (idx % NQ) * 8);
    }
    bias = nrx_tid() < COUTP ? w.b[nrx_tid()] : 0.f;
  }
  __device__ void store(char* dst, float* bias_dst, int rows = COUTP) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = nrx_tid() + i * 512;
      if (idx < NW && idx / NQ < rows) {
        const int co = idx / NQ, q = idx % NQ;
        *reinterpret_cast<intx4*>(dst + lds_off<NQ>(co >> 4, co & 15, q)) = v[i];
      }
    }
    if (nrx_tid() < COUTP) bias_dst[nrx_tid()] = bias;
  }
};

// R consecutive output rows (input slots s0 .. s0+R-1, neighbours s0-1 and s0+R) of one
// wave, all COUTP channels, bias included (it is the C operand of the first K chunk).
// acc[r][n][j] = out[row r][co = 16 n + P::co(g,j)][t].  The depthwise weights and every
// pointwise A fragment are loaded once per K chunk and reused over the R rows; the three
// input rows of consecutive outputs overlap, so a pass reads R + 2 activation rows
// instead of 3 R.
template <class P, int CINP, int COUTP, bool FIRST, int R, class WS>
__device__ __forceinline__ void conv_chunk(const char* X, const int (&rb)[R + 2], int sw, int kc, int g,
                                           int lane, const WS& ws, typename P::Acc (&acc)[R][COUTP / 16]) {
  using DV = typename P::DV;
  constexpr int NT = COUTP / 16;
  const int off = ((kc * 4 + g) ^ sw) * 16;
  DV xs[R + 2];
#pragma unroll
  for (int i = 0; i < R + 2; ++i) xs[i] = P::ld_lds(X + rb[i] + off);
  DV w[9];
  ws.dw_taps(kc, g, w);
  // A fragments one tile ahead (two registers): with one register the compiler serialises
  // `ds_read -> s_waitcnt -> MFMA x R` per tile and exposes the LDS latency NT times a chunk
  DV a_cur = ws.afrag(0, kc, lane, g);
  DV d[R];
#pragma unroll
  for (int r = 0; r < R; ++r) d[r] = P::dw_row(xs[r], xs[r + 1], xs[r + 2], w);
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    DV a_nxt = a_cur;
    if (n + 1 < NT) a_nxt = ws.afrag(n + 1, kc, lane, g);
    if constexpr (FIRST) {
      const typename P::Acc bn = ws.bias_acc(n, g);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r][n] = P::mma_v(a_cur, d[r], bn);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r][n] = P::mma_v(a_cur, d[r], acc[r][n]);
    }
    a_cur = a_nxt;
  }
}

template <class P, int CINP, int COUTP, int R, class WS, bool GZIN = false>
__device__ __forceinline__ void conv_rows(const char* X, int s0, int nslots, int t, int g, int lane,
                                          const WS& ws,
                                          typename P::Acc (&acc)[R][COUTP / 16], const GZ* gz = nullptr) {
  constexpr int NQ = CINP * (int)sizeof(typename P::S) / 16;
  constexpr int NKC = CINP / P::KC;
  const int sw = swz<NQ>(t);
  int rb[R + 2];
  if constexpr (P::WLDS) {
    // f16 layers have no inactive passes: rows s0-1 .. s0+R are inside the strip for every
    // wave (conv1 [0, R0-1], conv2 [0, R0-3], conv3 [0, R0-4]), so no clamp -- the rows are
    // then immediate offsets of one base register
#pragma unroll
    for (int i = 0; i < R + 2; ++i) rb[i] = (s0 - 1 + i) * slot_pitch<P>() + t * NQ * 16;
  } else {
#pragma unroll
    for (int i = 0; i < R + 2; ++i) {
      int sl = s0 - 1 + i;
      sl = sl < 0 ? 0 : (sl >= nslots ? nslots - 1 : sl);
      rb[i] = sl * slot_pitch<P>() + t * NQ * 16;
    }
  }
  if constexpr (P::WLDS) {
    // software-pipelined over the K chunks: chunk kc+1's activation rows and depthwise taps
    // are read into the registers of chunk kc as soon as its depthwise is done (they are
    // dead then), so their LDS latency hides behind chunk kc's MFMAs instead of stalling the
    // start of chunk kc+1
    using DV = typename P::DV;
    constexpr int NT = COUTP / 16;
    DV xs[R + 2], w[9];
    unsigned soff[R + 2];
    if constexpr (GZIN) {
#pragma unroll
      for (int i = 0; i < R + 2; ++i) soff[i] = gz->row_soff(s0 - 1 + i);
    }
    auto load = [&](int kc) {
      if constexpr (GZIN) {
        static_assert(sizeof(typename P::S) == 2 && CINP == 128 && R + 2 <= 6, "global z rows: f16 update conv1");
        // chunk 0 was issued in the item prologue (its latency behind the conv1-weight staging)
#pragma unroll
        for (int i = 0; i < R + 2; ++i) xs[i] = kc == 0 ? gz->x0[i] : gz->load(kc, soff[i]);
      } else {
        const int off = ((kc * 4 + g) ^ sw) * 16;
#pragma unroll
        for (int i = 0; i < R + 2; ++i) xs[i] = P::ld_lds(X + rb[i] + off);
      }
      ws.dw_taps(kc, g, w);
    };
    load(0);
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      DV a_cur = ws.afrag(0, kc, lane, g);
      DV d[R];
#pragma unroll
      for (int r = 0; r < R; ++r) d[r] = P::dw_row(xs[r], xs[r + 1], xs[r + 2], w);
      if (kc + 1 < NKC) load(kc + 1);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        DV a_nxt = a_cur;
        if (n + 1 < NT) a_nxt = ws.afrag(n + 1, kc, lane, g);
        if (kc == 0) {
          const typename P::Acc bn = ws.bias_acc(n, g);
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r][n] = P::mma_v(a_cur, d[r], bn);
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r][n] = P::mma_v(a_cur, d[r], acc[r][n]);
        }
        a_cur = a_nxt;
      }
    }
  } else {
    conv_chunk<P, CINP, COUTP, true, R>(X, rb, sw, 0, g, lane, ws, acc);
    for (int kc = 1; kc < NKC; ++kc) conv_chunk<P, CINP, COUTP, false, R>(X, rb, sw, kc, g, lane, ws, acc);
  }
}

// One pass of a layer for one wave: R output rows from position p0 (act: any row valid).
// Every pass computes into registers, then hands the accumulators to `epi`, which may
// overwrite input slots of rows this round consumed (in-place layers: the output of
// position p goes to slot p - in_off - 1, which no later round reads).  All waves execute
// the same barriers.
template <class P, int CINP, int COUTP, int R, bool GZIN, class WS, class Epi, class Post>
__device__ __forceinline__ void layer_pass(const char* X, int nslots, int in_off, int p0, bool act, bool first_round,
                                           const WS& ws, Epi& epi, Post& post_math, const GZ* gz, bool skip = false) {
  using E = std::decay_t<Epi>;
  const int lane = nrx_tid() & 63;
  const int t = lane & 15, g = lane >> 4;
  typename P::Acc acc[R][COUTP / 16];
  typename E::template PrefT<R> pf;
  stamp(8 + 5 * in_off);
  if (act) epi.template prefetch<R>(pf, p0, t, g);   // epilogue global loads, in flight during the math
  if (act) {
    if (skip || (NRX_ABLATE & 1)) {
      // skip: a StateInit_m item whose MCS weight is 0 (its conv output only ever enters as
      // 0 * finite): no math, any finite accumulator (the bias) gives the same state
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int n = 0; n < COUTP / 16; ++n) acc[r][n] = ws.bias_acc(n, g);
    } else {
      conv_rows<P, CINP, COUTP, R, WS, GZIN>(X, p0 - in_off, nslots, t, g, lane, ws, acc, gz);
    }
  }
  stamp(9 + 5 * in_off);
  if (in_off == 0) stamp_w(40);
  if constexpr (E::kNoBarrier) {
    // the epilogue neither writes LDS nor reads anything staged after the math: each
    // wave runs it as soon as its own math is done (post_math is empty for these)
    if constexpr (E::kNextHook) {
      // outside the nb test too: the waitcnt pass joins the paths after it
      epi.template settle<R>(pf);
      if (epi.nb >= 0) {
        // paired items: once every wave is past its conv3 reads the strip image is free,
        // and the next item's z image is DMA'd into it while this epilogue runs.  The
        // epilogue's own global loads are settled first (a use of a load result behind
        // an LDS-DMA would wait for the DMA too).  Settled on every wave, not only under
        // `act`: the waitcnt pass merges the pending-load state of both paths, so a
        // conditional settle left the skip-row loads pending and the first use in the
        // epilogue waited for vmcnt(0), i.e. for the whole DMA.
        __syncthreads();
        stamp(30);
        epi.next_hook();
        stamp(31);
      }
    }
    if (act) epi.template run<R>(acc, pf, p0, t, g, 0, R);
    stamp(12 + 5 * in_off);
  } else {
    // rows r >= kEarlyRow of an in-place layer land in slots no other wave reads this
    // round (wave w-1 reads up to slot p0 - in_off): written before the barrier
    constexpr int ER = E::kEarlyRow < R ? E::kEarlyRow : R;
    if (act) epi.template run<R>(acc, pf, p0, t, g, ER, R);
    if constexpr (E::kNextHookRO) epi.template settle<R>(pf);   // before any next-item DMA
    if (in_off == 0) stamp_w(48);
    __syncthreads();
    stamp(10 + 5 * in_off);
    if (first_round) post_math();      // all threads: this layer's weights are dead (P16)
    epi.pre();                       // all threads (e.g. stage tail weights into X)
    if constexpr (E::kNextHookRO) {
      // paired readout items: the heads are in WB and every wave is past its conv3 reads,
      // so the next item's z image is DMA'd into X while this epilogue runs
      if (epi.nb >= 0) {
        stamp(30);
        epi.next_hook();
        stamp(31);
      }
    }
    stamp(11 + 5 * in_off);
    if (act) epi.template run<R>(acc, pf, p0, t, g, 0, ER);
    stamp(12 + 5 * in_off);
    if (in_off == 0) stamp_w(56);
    __syncthreads();
  }
}

// One layer over output positions [pos_lo, pos_hi).  f16 policy: one round; the rows are
// split 4 / 3 per wave so that the 4 SIMDs (waves w and w + 4 share one) carry equal row
// counts (28 rows: 7 per SIMD; 26: 7,7,6,6; 24: 6 each) instead of whole waves idling.
// f64 policy: rounds of 8 waves x P::R rows.
template <class P, int CINP, int COUTP, bool GZIN = false, class WS, class Epi, class Post>
__device__ __forceinline__ void conv_layer(const char* X, int nslots, int in_off, int pos_lo,
                                           int pos_hi, const WS& ws, Epi&& epi, Post&& post_math,
                                           const GZ* gz = nullptr, bool skip = false) {
  const int wave = __builtin_amdgcn_readfirstlane(nrx_tid() >> 6);
  if constexpr (P::WLDS) {
    static_assert(P::R == 4, "f16 row split assumes passes of 4 / 3 rows");
    const int nrows = pos_hi - pos_lo;   // <= 32 (static_assert on FO)
    int n4 = nrows - 24;
    n4 = n4 < 0 ? 0 : n4;
    const int p0 = pos_lo + 4 * (wave < n4 ? wave : n4) + 3 * (wave > n4 ? wave - n4 : 0);
    const bool act = p0 < pos_hi;
    if (wave < n4) layer_pass<P, CINP, COUTP, 4, GZIN>(X, nslots, in_off, p0, act, true, ws, epi, post_math, gz, skip);
    else layer_pass<P, CINP, COUTP, 3, GZIN>(X, nslots, in_off, p0, act, true, ws, epi, post_math, gz, skip);
  } else {
    for (int base = pos_lo; base < pos_hi; base += 8 * P::R) {
      const int p0 = base + wave * P::R;
      layer_pass<P, CINP, COUTP, P::R, false>(X, nslots, in_off, p0, p0 < pos_hi, base == pos_lo, ws, epi, post_math,
                                              nullptr, skip);
    }
  }
}

struct NoPref {};

// In-place epilogue: ReLU, zero outside the grid, store to slot p-in_off-1.  Lanes
// t >= 14 do not store: the pad symbols of every slot are zero from the start of the
// block and stay zero (P16); P64 writes them as zeros.
// ER: the first row written before the layer barrier (rows 0, 1 of a wave land in slots the
// previous wave may still read; 0 when the layer's input is not in the image: GZ conv1).
template <class P, int COUTP, class WS, int ER = 2>
struct EpiInPlace {
  template <int R>
  using PrefT = NoPref;
  static constexpr bool kNoBarrier = false;
  static constexpr bool kNextHook = false;
  static constexpr bool kNextHookRO = false;
  static constexpr int kEarlyRow = ER;
  char* X;
  int in_off, pos_hi, f_start, F;
  WS ws;
  __device__ void pre() const {}
  template <int R>
  __device__ void prefetch(NoPref&, int, int, int) const {}
  template <int R>
  __device__ void run(const typename P::Acc (&acc)[R][COUTP / 16], const NoPref&, int p0, int t,
                      int g, int r_lo, int r_hi) const {
    using Real = typename P::Real;
    using S = typename P::S;
    constexpr int NQ = COUTP * (int)sizeof(S) / 16;
    if constexpr (sizeof(S) == 2) {
      // f16: the image of an in-place layer's output is in the K-permuted channel order of
      // the consumer (nrx_api.cpp build_model, hpos): lane (t, g)'s 4 channels of tiles
      // 2kc and 2kc+1 are chunk 4kc + g, so each tile pair is one 16-byte store of the
      // lane's own values.  The lane's chunk addresses are formed once per pass (opaque
      // to LLVM so that they stay registers); a row adds r * slot_pitch as the DS
      // immediate offset.
      typedef __attribute__((address_space(3))) half8 lds_half8;
      constexpr int NKC = COUTP / 32;
      unsigned lo[NKC];
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        lo[kc] = (unsigned)(size_t)(__attribute__((address_space(3))) char*)X +
                 (unsigned)((p0 - in_off - 1) * slot_pitch<P>() + (t * NQ + ((4 * kc + g) ^ swz<NQ>(t))) * 16);
        asm("" : "+v"(lo[kc]));
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < r_lo || r >= r_hi) continue;
        const int p = p0 + r;
        if (p >= pos_hi) continue;
        const int f = f_start + p;
        const bool z = f < 0 || f >= F;   // wave-uniform: scalar branch
        if (t < kT) {   // pad symbols t >= 14 stay zero from the start of the block
          if (!z) {
#pragma unroll
            for (int kc = 0; kc < NKC; ++kc) {
              const auto& a0 = acc[r][2 * kc];
              const auto& a1 = acc[r][2 * kc + 1];
              half8 h = half8{(S)a0[0], (S)a0[1], (S)a0[2], (S)a0[3], (S)a1[0], (S)a1[1], (S)a1[2], (S)a1[3]};
              h = __builtin_elementwise_max(h, half8{});
              *(lds_half8*)(size_t)(lo[kc] + r * slot_pitch<P>()) = h;
            }
          } else {
#pragma unroll
            for (int kc = 0; kc < NKC; ++kc) *(lds_half8*)(size_t)(lo[kc] + r * slot_pitch<P>()) = half8{};
          }
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < r_lo || r >= r_hi) continue;
        const int p = p0 + r;
        if (p >= pos_hi) continue;
        const int f = f_start + p;
        const bool z = f < 0 || f >= F;
        const int slot = p - in_off - 1;
#pragma unroll
        for (int n = 0; n < COUTP / 16; ++n) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int co = 16 * n + P::co(g, j);
            Real v = (Real)acc[r][n][j];
            v = v > (Real)0 ? v : (Real)0;
            if (z || t >= kT) v = (Real)0;
            *reinterpret_cast<S*>(X + xoff<P, NQ>(slot, t, co / P::EPC) + (co % P::EPC) * (int)sizeof(S)) = (S)v;
          }
        }
      }
    }
  }
};

// Dense layer on one 16-row tile with the B operand from a 16-byte-chunk source.
template <class P, int CINP, int COUTP, class Src>
__device__ __forceinline__ void dense_tile(Src src, int lane, int g,
                                           const DenseW<typename P::WT, typename P::BT>& w,
                                           typename P::Acc (&acc)[COUTP / 16]) {
  constexpr int NKC = CINP / P::KC;
#pragma unroll
  for (int n = 0; n < COUTP / 16; ++n) acc[n] = P::zero();
  const typename P::WT* wrow = w.w + (lane & 15) * CINP + g * P::CPL;
#pragma unroll
  for (int kc = 0; kc < NKC; ++kc) {
    const typename P::DV b = src(kc * 4 + g);
#pragma unroll
    for (int n = 0; n < COUTP / 16; ++n)
      acc[n] = P::mma(wrow + n * 16 * CINP + kc * P::KC, b, acc[n]);
  }
}

// Epilogue: +bias (, ReLU) -> LDS image of COUTP channels; zero rows t >= 14 or `zero`.
template <class P, int COUTP>
__device__ __forceinline__ void epi_lds(char* out, int row, int t, int g,
                                        const typename P::Acc (&acc)[COUTP / 16],
                                        const typename P::BT* bias, bool relu, bool zero) {
  using Real = typename P::Real;
  const bool z = zero || t >= kT;
#pragma unroll
  for (int n = 0; n < COUTP / 16; ++n) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = 16 * n + P::co(g, j);
      Real v = (Real)acc[n][j] + (Real)bias[co];
      if (relu) v = v > (Real)0 ? v : (Real)0;
      if (z) v = (Real)0;
      lds_store<P>(out, lds_elem_off<P, COUTP>(row, t, co), v);
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave complete in order; this only stops the compiler from
  // moving the dependent LDS accesses across the point.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ===================================================== separable-conv block kernels
// One workgroup = one (slot, user, subcarrier strip) running the 3-conv block of the
// state init or of one iteration's state update.  The per-user MLPs that consume the new
// state run in the conv3 epilogue straight from the accumulators: the MFMA C layout of a
// 16-channel tile (lane (t, g) holds channels 16 n + P::co(g, j)) is reused as the B
// operand of the next MFMA, with that layer's K axis permuted on the host to match
// (nrx_api.cpp, kperm_*).  After an update that is not the last, the epilogue applies
// the aggregation MLP of the next iteration and stores act_u * sp_u; the next launch's
// z-load (or k_combine for U > 4) forms the leave-one-out mean.  After the last update the
// epilogue runs the LLR / ChEst readouts instead.
//
// State / aggregate buffers are compact: [B][U][F][14][56] (no padding in HBM).

// TAIL_READOUT_WB: readout tail with the heads staged into WB, two items per workgroup
enum Tail { TAIL_NONE = -1, TAIL_AGG = 0, TAIL_READOUT = 1, TAIL_READOUT_WB = 2 };
constexpr bool readout_tail(int t) { return t == TAIL_READOUT || t == TAIL_READOUT_WB; }

template <class P>
struct BlockParams {
  FwdArgs<typename P::WT, typename P::BT, typename P::S> a;
  SepW<typename P::WT, typename P::BT> w[3];             // the block's separable layers
  DenseW<typename P::WT, typename P::BT> agg[2];         // next iteration's aggregation MLP
  DenseW<typename P::WT, typename P::BT> llr[kMaxHeads][2];
  DenseW<typename P::WT, typename P::BT> chest[2];
  int tail;                                              // TAIL_AGG / TAIL_READOUT / TAIL_NONE
  int m;                                                 // init: which StateInit (Var-IO)
  int strips;                                            // strips per (slot, user)
  int order_rev;                                         // XCD-local work order reversed
  int inline_combine;                                    // U <= kInlineUsers: z-load forms a
  int norm_pre;                                          // a.norm[b] holds the slot norm (k_norm ran)
  int pair;                                              // k_update: two items per workgroup (2nd prefetched)
  int gz;                                                // k_update: conv1 reads its z rows from memory
};

template <class P>
constexpr int strip_slots() { return P::FO + 2 * kHalo; }
template <class P>
constexpr int strip_lds_bytes(bool heads_wb = false) {
  return strip_slots<P>() * slot_pitch<P>() + (P::WLDS ? (heads_wb ? kWAlloc : kWBytes) : 0);
}
static_assert(strip_lds_bytes<P16>(true) == 160 * 1024, "P16 strip image + WB = LDS");
static_assert(P16::FO <= 8 * P16::R && P16M::FO <= 8 * P16M::R && P16S::FO <= 8 * P16S::R,
              "the conv3 of a strip must run in one round");

// in-plane element offset of (f, t) in a [F][14][56] state plane (< 2^31 for F <= 3276)
__device__ __forceinline__ int sre(int f, int t) { return (f * kT + t) * kDS; }
__device__ __forceinline__ size_t srow(int b, int u, int f, int t, int U, int F) {
  return ((((size_t)b * U + u) * F + f) * kT + t) * kDS;
}

// Runs one separable layer of a block over the strip.  P16: the layer's weights are
// already in the LDS image WB (staged by the previous phase); `post` runs after the math.
template <class P, int CINP, int COUTP, bool GZIN = false, class Epi, class Post>
__device__ __forceinline__ void run_layer(char* X, char* WB, const SepW<typename P::WT, typename P::BT>& w,
                                          int in_off, int pos_lo, int pos_hi, Epi&& epi_of, Post&& post,
                                          const GZ* gz = nullptr, bool skip = false) {
  constexpr int R0 = strip_slots<P>();
  if constexpr (P::WLDS) {
    WLds<P, CINP, COUTP> ws{WB};
    conv_layer<P, CINP, COUTP, GZIN>(X, R0, in_off, pos_lo, pos_hi, ws, epi_of(ws), post, gz, skip);
  } else {
    WGlb<P, CINP, COUTP> ws{w};
    conv_layer<P, CINP, COUTP>(X, R0, in_off, pos_lo, pos_hi, ws, epi_of(ws), post, nullptr, skip);
  }
}

static_assert(P16::FO + 4 <= 8 * P16::R && P16M::FO + 4 <= 8 * P16M::R && P16S::FO + 4 <= 8 * P16S::R,
              "P16 layers must run in one round (weights are swapped after it)");

// ------------------------------------------------------ dense layers from registers
// Dense weights: LDS image (P16, staged by the workgroup) or global (P64); K permuted.
template <class P, int CINP>
struct DLds {
  const char* base;
  const float* bias_p;
  static constexpr int NQ = CINP * 2 / 16;
  // Fragment address = one register per K chunk + the tile row as an immediate offset.  A
  // plain `base + lds_off(n, ..)` compiles to or + shift + add per fragment: LLVM turns the
  // disjoint-bit sum into an OR that the DS addressing match cannot split, and WB lies
  // beyond the 16-bit offset range.  The asm (not volatile, so equal (base, kc) calls are
  // CSE'd) hides the per-lane part from that rewrite.
  __device__ typename P::DV afrag(int n, int kc, int lane, int g) const {
    typedef const __attribute__((address_space(3))) char lds_char;
    typedef const __attribute__((address_space(3))) half8 lds_half8;
    unsigned a = (unsigned)(size_t)(lds_char*)base + (unsigned)lds_off<NQ>(0, lane & 15, kc * 4 + g);
    asm("" : "+v"(a));
    return *reinterpret_cast<lds_half8*>((lds_char*)(size_t)a + n * (kTP * NQ * 16));
  }
  __device__ typename P::Acc bias_acc(int n, int g) const { return P::bias_acc(bias_p, n, g); }
};
template <class P, int CINP>
struct DGlb {
  DenseW<typename P::WT, typename P::BT> w;
  __device__ typename P::DV afrag(int n, int kc, int lane, int g) const {
    return P::ld_w(w.w + (16 * n + (lane & 15)) * CINP + kc * P::KC + g * P::CPL);
  }
  __device__ typename P::Acc bias_acc(int n, int g) const { return P::bias_acc(w.b, n, g); }
};

// Stage a dense layer (P16) at `dst` (W^T image, K permuted on the host) and its bias at
// `bias_dst`.
template <int CINP, int COUTP>
__device__ __forceinline__ void stage_dense(char* dst, float* bias_dst, const DenseW<_Float16, float>& w) {
  constexpr int NQ = CINP * 2 / 16;
  constexpr int NW = COUTP * NQ;
  for (int idx = nrx_tid(); idx < NW; idx += 512) {
    const int co = idx / NQ, q = idx % NQ;
    *reinterpret_cast<intx4*>(dst + lds_off<NQ>(co >> 4, co & 15, q)) =
        *reinterpret_cast<const intx4*>(w.w + co * CINP + q * 8);
  }
  for (int idx = nrx_tid(); idx < COUTP; idx += 512) bias_dst[idx] = w.b[idx];
}

// B fragments of a dense layer whose input is NT accumulator tiles in C layout.
template <class P, int NT>
struct CFrag {
  static constexpr int NKC = NT * 16 / P::KC;
  typename P::DV b[NKC];
  __device__ CFrag() {}
  __device__ CFrag(const typename P::Real (&v)[NT][4]) {
    if constexpr (P::KC == 32) {
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc)
        b[kc] = typename P::DV{(_Float16)v[2 * kc][0], (_Float16)v[2 * kc][1], (_Float16)v[2 * kc][2],
                               (_Float16)v[2 * kc][3], (_Float16)v[2 * kc + 1][0], (_Float16)v[2 * kc + 1][1],
                               (_Float16)v[2 * kc + 1][2], (_Float16)v[2 * kc + 1][3]};
    } else {
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc)
        b[kc] = typename P::DV{(double)v[kc][0], (double)v[kc][1], (double)v[kc][2], (double)v[kc][3]};
    }
  }
  // f16 policy: ReLU on the packed f16 fragments (v_pk_max_f16, two values an instruction)
  // instead of on the f32 accumulators; round(relu(x)) == relu(round(x)) since rounding is
  // monotone and keeps zero, so the layer outputs are unchanged
  static constexpr bool kPackedRelu = P::KC == 32;
  __device__ void relu() {
    if constexpr (kPackedRelu) {
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) b[kc] = __builtin_elementwise_max(b[kc], typename P::DV{});
    }
  }
};

// Dense layer over NR rows at once: every A fragment and bias tile is loaded once and
// reused by the NR rows' MFMAs (the rows are independent chains).
template <class P, int NT, int COUTP, int NR, class WS>
__device__ __forceinline__ void dense_rows(const CFrag<P, NT> (&in)[NR], const WS& ws, int lane, int g,
                                           typename P::Real (&out)[NR][COUTP / 16][4], bool relu) {
  using Real = typename P::Real;
  constexpr int NKC = CFrag<P, NT>::NKC;
#pragma unroll
  for (int n = 0; n < COUTP / 16; ++n) {
    typename P::Acc acc[NR];
    const typename P::Acc bn = ws.bias_acc(n, g);
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const typename P::DV a = ws.afrag(n, kc, lane, g);
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r] = P::mma_v(a, in[r].b[kc], kc == 0 ? bn : acc[r]);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const Real v = (Real)acc[r][j];
        out[r][n][j] = relu ? (v > (Real)0 ? v : (Real)0) : v;
      }
  }
}

// Readout weight images staged into the (then free) strip buffer X (P16).
constexpr int kHeadSlot = 24 * 1024;   // W1^T 16 KB | W2^T <= 8 KB ... per head, 256-aligned
__device__ __forceinline__ int head_w1(int h) { return h * (kHeadSlot + 1024); }
__device__ __forceinline__ int head_w2(int h) { return head_w1(h) + 16 * 1024; }
__device__ __forceinline__ int head_b1(int h) { return head_w1(h) + kHeadSlot; }
__device__ __forceinline__ int head_b2(int h) { return head_b1(h) + 512; }

#ifndef NRX_RO_STRAIGHT
#define NRX_RO_STRAIGHT 1
#endif

// conv3 epilogue: new state rows (+ aggregation MLP or readouts) for the R rows of a
// wave.  All R rows are computed unconditionally (rows past the strip or the grid hold
// finite values from zero inputs) so the MLP chains of the rows interleave; only the
// stores are predicated.  The skip / Var-IO partial sum is prefetched before the conv3
// math (prefetch()), so its global latency hides behind it.
template <class P, class WS, int CHP, int TAILM>
struct EpiConv3 {
  using S = typename P::S;
  using Real = typename P::Real;
  static constexpr int NTS = kDSP / 16;        // state tiles (64 channels, >= 56 are 0)
  // previous state rows, kept in storage precision (packed) until the epilogue
  template <int R>
  struct PrefT {
    std::conditional_t<sizeof(S) == 2, half4, Real[4]> prev[R][NTS];
  };
  // no LDS writes; the readout tail reads head weights staged into X after the math
  static constexpr bool kNoBarrier = !readout_tail(TAILM);
  static constexpr bool kNextHook = TAILM == TAIL_AGG && P::WLDS;
  // paired readout items: the next z DMA is issued once the head weights are in WB
  static constexpr bool kNextHookRO = TAILM == TAIL_READOUT_WB && P::WLDS;
  static constexpr int kEarlyRow = 8;      // readout: every row after the barrier
  const BlockParams<P>* prm;
  char* X;
  char* WB;
  WS ws;
  int b, u, f_start, pos_hi, mode;   // mode 0: update (+skip), 1: init (x wm, Var-IO accumulate)
  Real wm;
  bool first;
  Real act_h;             // active[b][u], loaded before the conv3 math
  int nb, nu, nfs;        // paired k_update: next item (nb < 0: none)
  int pos_lo = 0;         // first strip position with an output row (RR blocks: kHalo)
  // fused forward (k_forward): the next item belongs to stage nprm and may start only once
  // its dependency counter has reached its target; strip_block polls the counter at the start
  // of conv2 and leaves the verdict in nflag (LDS) for conv3.  ndone == nullptr: no
  // dependency (paired items of one launch).
  const BlockParams<P>* nprm = nullptr;
  const int* ndone = nullptr;
  int* nflag = nullptr;

  __device__ bool next_ready() const { return nb >= 0 && (!ndone || *nflag); }

  template <int R>
  __device__ void settle(PrefT<R>& pf) {
    if constexpr (sizeof(S) == 2) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int n = 0; n < NTS; ++n) asm volatile("" : "+v"(pf.prev[r][n]));
    }
    asm volatile("" : "+v"(act_h));
  }
  __device__ void next_hook();

  __device__ bool row_ok(int p, int t) const {
    return p >= pos_lo && p < pos_hi && f_start + p < prm->a.F && t < kT;
  }

  template <int R>
  __device__ void prefetch(PrefT<R>& pf, int p0, int t, int g) const {
    const auto& a = prm->a;
    const bool need = mode == 0 || !first;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool ok = need && row_ok(p0 + r, t);
      // uniform plane base + 32-bit in-plane offset (no per-row 64-bit index chain)
      const S* src = (mode == 0 ? a.s_in : a.s_out) + srow(b, u, 0, 0, a.U, a.F) +
                     sre(ok ? f_start + p0 + r : 0, ok ? t : 0);
#pragma unroll
      for (int n = 0; n < NTS; ++n) {
        if constexpr (sizeof(S) == 2) {
          const int c0 = 16 * n + 4 * g;
          half4 h4 = half4{0, 0, 0, 0};
          if (ok && c0 < kDS) h4 = *reinterpret_cast<const half4*>(src + c0);
          pf.prev[r][n] = h4;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int co = 16 * n + P::co(g, j);
            pf.prev[r][n][j] = (ok && co < kDS) ? (Real)src[co] : (Real)0;
          }
        }
      }
    }
  }

  __device__ void pre() const {
    if constexpr (P::WLDS) {
      if constexpr (TAILM == TAIL_READOUT_WB) {
        __syncthreads();   // heads staged into WB by strip_block (one LLR head)
      } else if constexpr (TAILM == TAIL_READOUT) {
        // LLR head 0 and the ChEst head were prefetched during the conv3 math and stored
        // into X by strip_block; stage any further heads (Var-IO) now
        const auto& a = prm->a;
        for (int h = 1; h < a.H; ++h) {
          stage_dense<kDSP, kHID>(X + head_w1(h), reinterpret_cast<float*>(X + head_b1(h)), prm->llr[h][0]);
          stage_dense<kHID, 16>(X + head_w2(h), reinterpret_cast<float*>(X + head_b2(h)), prm->llr[h][1]);
        }
        __syncthreads();
      }
    }
  }

  // f16 state row (56 channels of one (f, t)) from the C layout of the 4 state tiles: lane
  // (t, g) holds channels 16n + 4g .. +3 of tile n.  v_permlane16_swap on the tile pairs
  // (0,1) and (2,3) exchanges the 16-lane rows g <-> g^1 so that every lane holds 16
  // contiguous bytes per pair (8-channel chunk 2n + 2(g&1) + (g>>1)): two 16-byte stores
  // per lane instead of four 8-byte ones (chunk 7, channels 56..63, is padding and not
  // stored).  The swaps run on every lane; only the stores are predicated.
  __device__ static void store_row16(S* dst, const Real (&v)[NTS][4], bool ok, int g) {
    unsigned w[NTS][2];
#pragma unroll
    for (int n = 0; n < NTS; ++n) {
      const half2 lo = half2{(S)v[n][0], (S)v[n][1]}, hi = half2{(S)v[n][2], (S)v[n][3]};
      w[n][0] = __builtin_bit_cast(unsigned, lo);
      w[n][1] = __builtin_bit_cast(unsigned, hi);
    }
#pragma unroll
    for (int n = 0; n < NTS; n += 2)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto x = __builtin_amdgcn_permlane16_swap(w[n][d], w[n + 1][d], false, false);
        w[n][d] = x[0];
        w[n + 1][d] = x[1];
      }
    if (!ok) return;
    const int ck = 2 * (g & 1) + (g >> 1);
#pragma unroll
    for (int n = 0; n < NTS; n += 2) {
      const int chunk = 2 * n + ck;
      if (chunk * 8 < kDS)
        *reinterpret_cast<intx4*>(dst + chunk * 8) = intx4{(int)w[n][0], (int)w[n][1], (int)w[n + 1][0], (int)w[n + 1][1]};
    }
  }

  // store NT16 tiles of f32 outputs for one row: channel co = 16 n + P::co(g, j) < nvalid
  template <int NT16>
  __device__ __forceinline__ void store_f32(float* dst, const Real (&o)[NT16][4], int g, int nvalid) const {
#pragma unroll
    for (int n = 0; n < NT16; ++n) {
      if constexpr (sizeof(S) == 2) {
        const int c0 = 16 * n + 4 * g;
        if (c0 + 3 < nvalid && (nvalid & 3) == 0) {
          *reinterpret_cast<floatx4*>(dst + c0) = floatx4{(float)o[n][0], (float)o[n][1], (float)o[n][2], (float)o[n][3]};
          continue;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = 16 * n + P::co(g, j);
        if (co < nvalid) dst[co] = (float)o[n][j];
      }
    }
  }

  // LDS images of readout head hh (hh == H: ChEst): X layout (head_w1 ..) or, paired, WB
  __device__ void head_lds(int hh, bool ch, const char*& w1, const float*& b1, const char*& w2,
                           const float*& b2) const {
    if constexpr (TAILM == TAIL_READOUT_WB) {
      w1 = WB + (ch ? kHW1C : 0);
      b1 = reinterpret_cast<const float*>(WB + kHB1 + (ch ? kHID * 4 : 0));
      b2 = reinterpret_cast<const float*>(WB + kHB2 + (ch ? 16 * 4 : 0));
      w2 = WB + kHW2 + (ch ? prm->a.bits_max * 256 : 0);
    } else {
      w1 = X + head_w1(hh);
      b1 = reinterpret_cast<const float*>(X + head_b1(hh));
      w2 = X + head_w2(hh);
      b2 = reinterpret_cast<const float*>(X + head_b2(hh));
    }
  }

  template <int NO, int RB, class W1, class W2>
  __device__ __forceinline__ void head_rows(const CFrag<P, NTS> (&sb)[RB], const W1& w1, const W2& w2, int lane,
                                            int g, Real (&o)[RB][NO][4]) const {
    Real hdn[RB][kHID / 16][4];
    using HF = CFrag<P, kHID / 16>;
    dense_rows<P, NTS, kHID, RB>(sb, w1, lane, g, hdn, !HF::kPackedRelu);
    HF hb[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      hb[r] = HF(hdn[r]);
      hb[r].relu();
    }
    dense_rows<P, kHID / 16, NO * 16, RB>(hb, w2, lane, g, o, false);
  }

  template <int R>
  __device__ void run(const typename P::Acc (&acc)[R][NTS], const PrefT<R>& pf, int p0, int t, int g,
                      int r_lo, int r_hi) const {
    if (r_lo >= r_hi) return;        // all R rows in one call
    stamp(6);
    const auto& a = prm->a;
    const int F = a.F, U = a.U;
    const int lane = nrx_tid() & 63;
    // ---- new state rows s (C layout, channels >= 56 forced to 0), rounded to S
    Real sv[R][NTS][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int n = 0; n < NTS; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = 16 * n + P::co(g, j);
          Real v = (Real)acc[r][n][j];
          if (mode == 1) v *= wm;
          v += (Real)pf.prev[r][n][j];
          if (co >= kDS) v = 0;
          sv[r][n][j] = (Real)(S)v;
        }
    size_t off[R];
    bool ok[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      ok[r] = row_ok(p0 + r, t) && !(NRX_ABLATE & 16);
      off[r] = srow(b, u, 0, 0, U, F) + (size_t)(unsigned)sre(ok[r] ? f_start + p0 + r : 0, ok[r] ? t : 0);
    }
    if constexpr (!readout_tail(TAILM)) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        S* dst = a.s_out + off[r];
        if constexpr (sizeof(S) == 2) {
          store_row16(dst, sv[r], ok[r] && !((NRX_ABLATE & 32) && a.B > 0), g);
        } else {
          if (!ok[r]) continue;
#pragma unroll
          for (int n = 0; n < NTS; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int co = 16 * n + P::co(g, j);
              if (co < kDS) dst[co] = (S)sv[r][n][j];
            }
        }
      }
    }
    if constexpr (TAILM == TAIL_NONE) return;
    CFrag<P, NTS> sb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sb[r] = CFrag<P, NTS>(sv[r]);
    if constexpr (TAILM == TAIL_AGG) {
      // sp_u = act_u * (W2 relu(W1 s + b1) + b2)  -> a_out (combined by the tail)
      Real hdn[R][kAGG / 16][4], sp[R][NTS][4];
      const Real act = act_h;
      CFrag<P, kAGG / 16> hb[R];
      if constexpr ((NRX_ABLATE & 128) != 0 && P::WLDS) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int n = 0; n < NTS; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) sp[r][n][j] = sv[r][n][j];
      } else if constexpr (P::WLDS) {
        DLds<P, kDSP> w1{WB + 16 * 1024, reinterpret_cast<const float*>(WB + kWTailBias)};
        DLds<P, kAGG> w2{WB + 24 * 1024, reinterpret_cast<const float*>(WB + kWTailBias + kAGG * 4)};
        dense_rows<P, NTS, kAGG, R>(sb, w1, lane, g, hdn, !CFrag<P, kAGG / 16>::kPackedRelu);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          hb[r] = CFrag<P, kAGG / 16>(hdn[r]);
          hb[r].relu();
        }
        dense_rows<P, kAGG / 16, kDSP, R>(hb, w2, lane, g, sp, false);
      } else {
        dense_rows<P, NTS, kAGG, R>(sb, DGlb<P, kDSP>{prm->agg[0]}, lane, g, hdn, !CFrag<P, kAGG / 16>::kPackedRelu);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          hb[r] = CFrag<P, kAGG / 16>(hdn[r]);
          hb[r].relu();
        }
        dense_rows<P, kAGG / 16, kDSP, R>(hb, DGlb<P, kAGG>{prm->agg[1]}, lane, g, sp, false);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        S* dst = a.a_out + off[r];
        if constexpr (sizeof(S) == 2) {
          Real spa[NTS][4];
#pragma unroll
          for (int n = 0; n < NTS; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) spa[n][j] = sp[r][n][j] * act;
          store_row16(dst, spa, ok[r] && !((NRX_ABLATE & 64) && a.B > 0), g);
        } else {
          if (!ok[r]) continue;
#pragma unroll
          for (int n = 0; n < NTS; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int co = 16 * n + P::co(g, j);
              if (co < kDS) dst[co] = (S)(sp[r][n][j] * act);
            }
        }
      }
    } else {
      // readouts: LLR head(s) then ChEst, RB rows at a time
      constexpr int RB = R % 2 == 0 ? 2 : (R == 3 ? 3 : 1);
#pragma unroll
      for (int r0 = 0; r0 < R; r0 += RB) {
        CFrag<P, NTS> sbr[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) sbr[r] = sb[r0 + r];
        // one head (hh < H: LLR head hh, hh == H: ChEst); straight-line for the common
        // single LLR head so the ChEst MFMAs can start under the LLR head's tail
        auto one_head = [&](int hh, bool ch) __attribute__((always_inline)) {
          if (!ch) {
            Real o[RB][1][4];
            if constexpr (P::WLDS) {
              const char *w1, *w2;
              const float *b1, *b2;
              head_lds(hh, false, w1, b1, w2, b2);
              head_rows<1, RB>(sbr, DLds<P, kDSP>{w1, b1}, DLds<P, kHID>{w2, b2}, lane, g, o);
            } else {
              head_rows<1, RB>(sbr, DGlb<P, kDSP>{prm->llr[hh][0]}, DGlb<P, kHID>{prm->llr[hh][1]}, lane, g, o);
            }
#pragma unroll
            for (int r = 0; r < RB; ++r) {
              if (!ok[r0 + r]) continue;
              const int f = f_start + p0 + r0 + r;
              float* dst = a.llr + ((((size_t)hh * a.B + b) * U + u) * F + f) * kT * a.bits_max + t * a.bits_max;
              // head bits beyond head_bits[hh] (masking: sliced later) are written as 0
              if constexpr (sizeof(S) == 2) {
                if (a.bits_max == 4) {
                  // 16-QAM: lanes g = 0 hold the 4 LLRs of their symbol, one 16-byte store
                  const int nb = a.head_bits[hh];
                  if (g == 0)
                    *reinterpret_cast<floatx4*>(dst) =
                        floatx4{nb > 0 ? (float)o[r][0][0] : 0.f, nb > 1 ? (float)o[r][0][1] : 0.f,
                                nb > 2 ? (float)o[r][0][2] : 0.f, nb > 3 ? (float)o[r][0][3] : 0.f};
                  continue;
                }
              }
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int co = P::co(g, j);
                if (co < a.bits_max) dst[co] = co < a.head_bits[hh] ? (float)o[r][0][j] : 0.f;
              }
            }
          } else {
            Real o[RB][CHP / 16][4];
            if constexpr (P::WLDS) {
              const char *w1, *w2;
              const float *b1, *b2;
              head_lds(hh, true, w1, b1, w2, b2);
              head_rows<CHP / 16, RB>(sbr, DLds<P, kDSP>{w1, b1}, DLds<P, kHID>{w2, b2}, lane, g, o);
            } else {
              head_rows<CHP / 16, RB>(sbr, DGlb<P, kDSP>{prm->chest[0]}, DGlb<P, kHID>{prm->chest[1]}, lane, g, o);
            }
            const int A2 = 2 * a.A;
#pragma unroll
            for (int r = 0; r < RB; ++r) {
              if (!ok[r0 + r]) continue;
              const int f = f_start + p0 + r0 + r;
              store_f32<CHP / 16>(a.h_ref + ((((size_t)b * U + u) * F + f) * kT + t) * A2, o[r], g, A2);
            }
          }
        };
        if (NRX_RO_STRAIGHT && a.H == 1) {
          one_head(0, false);
          if (a.h_ref) one_head(1, true);
        } else {
          for (int hh = 0; hh <= a.H; ++hh) {
            const bool ch = hh == a.H;
            if (ch && !a.h_ref) break;
            one_head(hh, ch);
          }
        }
      }
    }
  }
};

// Register prefetch of the next layer's weights during the current layer's math (off: they
// are fetched after it, latency exposed, registers free for the conv pipeline).
#ifndef NRX_PREFETCH_W
#define NRX_PREFETCH_W 1
#endif
constexpr bool kPrefetchW = NRX_PREFETCH_W != 0;

// Fused forward (k_forward): what an item needs to know about the workgroup's next item and
// its work queue (nullptr everywhere else).
template <class P>
struct FusedNext {
  const BlockParams<P>* nprm;   // the next item's stage (the sources of its z DMA)
  const int* ndone;             // its dependency counter (nullptr: no hook)
  int nneed;
  int* nflag;                   // LDS word: 1 when the next item's z DMA was issued
  int* head;                    // this queue's work counter
  int jnn;                      // thread 0: the item dequeued at the start of this block
};


// The three layers of a block, in place: conv1 over positions [1, R0-1), conv2 over
// [2, R0-2), conv3 over [3, R0-3) with the fused epilogue.  P16: conv1's weights are in
// WB on entry; each layer's global weight loads for the next layer (conv3: + the
// aggregation MLP) are issued before its math and stored to WB after it.
template <class P, int CINP, int CHP, int TAILM, bool GZIN = false>
__device__ __forceinline__ void strip_block(const BlockParams<P>& prm, char* X, char* WB, int b, int u,
                                            int f_start, int mode, typename P::Real wm, bool first, int nb = -1,
                                            int nu = 0, int nfs = 0, FusedNext<P>* fn = nullptr,
                                            const GZ* gz = nullptr, int* psig = nullptr, bool skip = false) {
  constexpr int R0 = strip_slots<P>();
  const int F = prm.a.F;
  // fused forward: dequeue the item after next here, past the item's prologue waits (an
  // older pending atomic would hold every vmcnt wait of wave 0); read at the item's end
  if (fn && nrx_tid() == 0) fn->jnn = atomicAdd(fn->head, 1);
  // skip (StateInit_m with MCS weight 0, f16): conv1 / conv2 are not run at all -- conv3's
  // weights (and the aggregation MLP) are staged directly and conv3 runs its epilogue on the
  // bias (0 * finite, like the skipped conv output)
  const bool fast = P::WLDS && skip;
  if (!fast) {
    SepStage<kHID, kHID> nx;
    if constexpr (P::WLDS && kPrefetchW) nx.load(prm.w[1]);
    run_layer<P, CINP, kHID, GZIN>(X, WB, prm.w[0], 0, 1, R0 - 1, [&](auto ws) {
      return EpiInPlace<P, kHID, decltype(ws), GZIN ? 0 : 2>{X, 0, R0 - 1, f_start, F, ws};
    }, [&]() {
      if constexpr (P::WLDS) {
        if constexpr (!kPrefetchW) nx.load(prm.w[1]);
        nx.store(WB);
      }
      // k_forward GZ items: the previous item's stores are drained here, where every wave has
      // consumed its loads anyway, and its counter is added after the layer barrier
      if (psig) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }, gz, skip);
  }
  if (psig && nrx_tid() == 0) __hip_atomic_fetch_add(psig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(2);
  if (fast) {
    if constexpr (P::WLDS) {
      SepStage<kHID, kDSP> nx;
      DenseStage<kDSP, kAGG> d1;
      DenseStage<kAGG, kDSP> d2;
      nx.load(prm.w[2]);
      if constexpr (TAILM == TAIL_AGG) {
        d1.load(prm.agg[0]);
        d2.load(prm.agg[1]);
      }
      int pv = 0;
      const bool poll = fn && fn->ndone && nrx_tid() == 0;
      if (poll) {
        pv = __hip_atomic_load(fn->ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("buffer_inv sc1" ::: "memory");
      }
      nx.store(WB);
      if constexpr (TAILM == TAIL_AGG) {
        d1.store(WB + 16 * 1024, reinterpret_cast<float*>(WB + kWTailBias));
        d2.store(WB + 24 * 1024, reinterpret_cast<float*>(WB + kWTailBias + kAGG * 4));
      }
      if (poll) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *fn->nflag = pv >= fn->nneed;
      }
      __syncthreads();
    }
  } else {
    SepStage<kHID, kDSP> nx;
    DenseStage<kDSP, kAGG> d1;
    DenseStage<kAGG, kDSP> d2;
    auto ld = [&]() {
      if constexpr (P::WLDS) {
        nx.load(prm.w[2]);
        if constexpr (TAILM == TAIL_AGG) {
          d1.load(prm.agg[0]);
          d2.load(prm.agg[1]);
        }
      }
    };
    if constexpr (P::WLDS && kPrefetchW) ld();
    // fused forward: thread 0 polls the next item's dependency counter (an sc1 load, L2-
    // served) and invalidates this CU's L1 -- no line of the next item's inputs this CU read
    // in an earlier stage (ping-pong buffers) may survive into its loads; both complete
    // behind the conv2 math.  The verdict goes to nflag for conv3's next_hook.
    int pv = 0;
    const bool poll = fn && fn->ndone && nrx_tid() == 0;
    if (poll) {
      pv = __hip_atomic_load(fn->ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("buffer_inv sc1" ::: "memory");
    }
    run_layer<P, kHID, kHID>(X, WB, prm.w[1], 1, 2, R0 - 2, [&](auto ws) {
      return EpiInPlace<P, kHID, decltype(ws)>{X, 1, R0 - 2, f_start, F, ws};
    }, [&]() {
      if (poll) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the poll and the invalidate
        *fn->nflag = pv >= fn->nneed;
      }
      if constexpr (P::WLDS) {
        if constexpr (!kPrefetchW) ld();
        nx.store(WB);
        if constexpr (TAILM == TAIL_AGG) {
          d1.store(WB + 16 * 1024, reinterpret_cast<float*>(WB + kWTailBias));
          d2.store(WB + 24 * 1024, reinterpret_cast<float*>(WB + kWTailBias + kAGG * 4));
        }
      }
    }, nullptr, skip);
  }
  stamp(3);
  {
    // readout tail: LLR head 0 and ChEst weights are fetched during the conv3 math and
    // stored into the strip image X once every wave is past its conv3 reads
    DenseStage<kDSP, kHID> l1, c1;
    DenseStage<kHID, 16> l2;
    DenseStage<kHID, CHP> c2;
    auto ld = [&]() {
      if constexpr (P::WLDS) {
        l1.load(prm.llr[0][0]);
        l2.load(prm.llr[0][1]);
        c1.load(prm.chest[0]);
        c2.load(prm.chest[1]);
      }
    };
    if constexpr (P::WLDS && readout_tail(TAILM) && kPrefetchW) ld();
    run_layer<P, kHID, kDSP>(X, WB, prm.w[2], 2, kHalo, R0 - kHalo, [&](auto ws) {
      EpiConv3<P, decltype(ws), CHP, TAILM> e{&prm, X, WB, ws, b, u, f_start, R0 - kHalo, mode, wm, first,
                                             (typename P::Real)prm.a.active[(size_t)b * prm.a.U + u],
                                             nb, nu, nfs};
      if (fn && fn->ndone) {
        e.nprm = fn->nprm;
        e.ndone = fn->ndone;
        e.nflag = fn->nflag;
      }
      return e;
    }, [&]() {
      if constexpr (P::WLDS && TAILM == TAIL_READOUT_WB) {
        // conv3's weights are dead (every wave is past its math): heads into WB
        if constexpr (!kPrefetchW) ld();
        const int nb2 = prm.a.bits_max;
        l1.store(WB, reinterpret_cast<float*>(WB + kHB1));
        c1.store(WB + kHW1C, reinterpret_cast<float*>(WB + kHB1 + kHID * 4));
        l2.store(WB + kHW2, reinterpret_cast<float*>(WB + kHB2), nb2);
        c2.store(WB + kHW2 + nb2 * 256, reinterpret_cast<float*>(WB + kHB2 + 16 * 4), 2 * prm.a.A);
      } else if constexpr (P::WLDS && TAILM == TAIL_READOUT) {
        if constexpr (!kPrefetchW) ld();
        const int H = prm.a.H;
        l1.store(X + head_w1(0), reinterpret_cast<float*>(X + head_b1(0)));
        l2.store(X + head_w2(0), reinterpret_cast<float*>(X + head_b2(0)));
        c1.store(X + head_w1(H), reinterpret_cast<float*>(X + head_b1(H)));
        c2.store(X + head_w2(H), reinterpret_cast<float*>(X + head_b2(H)));
      }
    }, nullptr, skip);
  }
}

// ---------------------------------------------------------------- per-user block bodies
// StateInit_m of user u on the strip.  z = [y*ns | h*ns | pe] with each antenna block
// padded to A2P channels (y at [0, 2A), h at [A2P, A2P+2A), pe at 2 A2P, 2 A2P + 1; the host
// packs conv1's weights to match, nrx_api.cpp build_model).  One thread per (slot, symbol)
// row of the z image: vector loads of the y / h rows and the pe pair, channel assembly in
// registers at compile-time positions, then 16-byte LDS stores.
template <int A2P>
constexpr int init_cinp(int kc) {
  int c = (2 * A2P + 2 + kc - 1) / kc * kc;
  int p = 32;
  while (p < c) p *= 2;
  return p;
}

// Slot normalisation (neural_rx.py:551-557): ns = 1/sqrt(mean(y^2)) over the whole grid
// given (F x 14 x 2A floats, nq float4s), divide-no-nan (an all-zero slot gets 0).  Every
// workgroup of the slot computes it (21 KB at nrx_rt, L2-resident after the first): no
// separate launch.  Double accumulation; `red` is 8 doubles of LDS.
// acc + v.v as an explicit fma chain: the contraction is fixed in the source, so the slot norm
// (and with it every later rounding of the slot) does not move with the surrounding codegen
__device__ __forceinline__ double sq4(double acc, floatx4 v) {
  acc = __builtin_fma((double)v[0], (double)v[0], acc);
  acc = __builtin_fma((double)v[1], (double)v[1], acc);
  acc = __builtin_fma((double)v[2], (double)v[2], acc);
  return __builtin_fma((double)v[3], (double)v[3], acc);
}

// The first kNormPre float4s of each thread are loaded up front (slot_norm_issue, from
// clamped addresses, unconditionally) so that their latency overlaps the z-row loads; the
// accumulation order is the plain strided loop's.
constexpr int kNormPre = 4;
struct NormPre {
  floatx4 v[kNormPre];
};
__device__ __forceinline__ NormPre slot_norm_issue(const float* y, int nq) {
  const floatx4* yq = reinterpret_cast<const floatx4*>(y);
  NormPre p;
#pragma unroll
  for (int k = 0; k < kNormPre; ++k) {
    const int i = nrx_tid() + 512 * k;
    p.v[k] = yq[i < nq ? i : nq - 1];
  }
  return p;
}
__device__ __forceinline__ double slot_norm(const NormPre& pre, const float* y, int nq, double* red) {
  const floatx4* yq = reinterpret_cast<const floatx4*>(y);
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < kNormPre; ++k)
    if (nrx_tid() + 512 * k < nq) acc = sq4(acc, pre.v[k]);
  for (int i = nrx_tid() + 512 * kNormPre; i < nq; i += 512) {
    const floatx4 v = yq[i];
    acc = sq4(acc, v);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((nrx_tid() & 63) == 0) red[nrx_tid() >> 6] = acc;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int w = 0; w < 8; ++w) tot += red[w];
  const double ms = tot / (double)(4 * nq);
  return ms > 0.0 ? 1.0 / sqrt(ms) : 0.0;
}

// Per-slot normalisation pass for large grids (one workgroup per slot, fixed striding and
// reduction order: deterministic).  norm[b] = 1/sqrt(mean(y^2)), 0 for an all-zero slot.
__global__ __launch_bounds__(1024) void k_norm(const float* __restrict__ y, int nq, double* __restrict__ norm) {
  __shared__ double red[16];
  const floatx4* yq = reinterpret_cast<const floatx4*>(y) + (size_t)blockIdx.x * nq;
  double acc = 0.0;
  for (int i = nrx_tid(); i < nq; i += 1024) {
    const floatx4 v = yq[i];
    acc = sq4(acc, v);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((nrx_tid() & 63) == 0) red[nrx_tid() >> 6] = acc;
  __syncthreads();
  if (nrx_tid() == 0) {
    double tot = 0.0;
    for (int w = 0; w < 16; ++w) tot += red[w];
    const double ms = tot / (double)(4 * nq);
    norm[blockIdx.x] = ms > 0.0 ? 1.0 / sqrt(ms) : 0.0;
  }
}

#ifndef NRX_INIT_ORDER
#define NRX_INIT_ORDER 1
#endif

// slot grids above this many float4s get the separate k_norm pass (nrx_rt: 1 344)
constexpr int kNormFusedMaxQ = 8192;

template <class P, int A2P, int CHP, int TAILM>
__device__ __forceinline__ void init_user(const BlockParams<P>& prm, char* smem, int b, int u,
                                          int strip, typename P::Real wm, bool first, int nb = -1, int nu = 0,
                                          int nfs = 0, FusedNext<P>* fn = nullptr) {
  __shared__ double red[8];
  using S = typename P::S;
  using Real = typename P::Real;
  constexpr int CINP = init_cinp<A2P>(P::KC);
  constexpr int R0 = strip_slots<P>();
  constexpr int NQZ = CINP * (int)sizeof(S) / 16;
  const auto& a = prm.a;
  const int F = a.F, U = a.U, A2 = 2 * a.A;
  const int f0 = strip * P::FO;
  const int f_start = f0 - kHalo;
  char* X = smem;
  char* WB = smem + R0 * slot_pitch<P>();
  auto pad_zero = [&]() __attribute__((always_inline)) {
    if constexpr (sizeof(S) == 2 && CINP < kHID) {
      // pad symbols t = 14, 15 of the 128-channel layout the conv layers write in place:
      // zero once (the z image below occupies the first CINP*32 bytes of each slot; its
      // own t = 14, 15 stores are zeros too, so the two may land in either order)
      constexpr int NQ = kHID * (int)sizeof(S) / 16;
      for (int idx = nrx_tid(); idx < R0 * 2 * NQ; idx += 512) {
        const int q = idx % NQ, tt = kT + (idx / NQ) % 2, lf = idx / (2 * NQ);
        *reinterpret_cast<intx4*>(X + xoff<P, NQ>(lf, tt, q)) = intx4{0, 0, 0, 0};
      }
    }
  };
  if (!a.masking && wm == (Real)0) {
    // Var-IO: this MCS does not apply to (b, u) (one-hot mask), so StateInit_m enters the
    // state as 0 * finite (neural_rx.py:562-569): no z image, no conv math; the block still
    // stages its layer weights and runs the epilogue (the first stage writes the zero state,
    // the last one the aggregation MLP of the accumulated state).  Bit-identical up to the
    // sign of zero states (the bias replaces the conv output in the 0 * finite product).
    // The pad symbols are zeroed whatever CINP is (a full item's z image would have).
    if constexpr (sizeof(S) == 2) {
      constexpr int NQ = kHID * (int)sizeof(S) / 16;
      for (int idx = nrx_tid(); idx < R0 * 2 * NQ; idx += 512) {
        const int q = idx % NQ, tt = kT + (idx / NQ) % 2, lf = idx / (2 * NQ);
        *reinterpret_cast<intx4*>(X + xoff<P, NQ>(lf, tt, q)) = intx4{0, 0, 0, 0};
      }
    }
    if constexpr (sizeof(S) == 2) {
      // one-launch forward: the pe16 rows of this item (every other user of the slot may skip too)
      const int lf = nrx_tid() / kTP, tt = nrx_tid() % kTP, f = f_start + lf;
      if (a.pe16 && lf >= kHalo && lf < kHalo + P::FO && lf < R0 && tt < kT && f >= 0 && f < F) {
        const float2 pv = *reinterpret_cast<const float2*>(a.pe + (((size_t)u * F + f) * kT + tt) * 2);
        S pe2[8] = {};
        pe2[0] = (S)pv.x;
        pe2[1] = (S)pv.y;
        *reinterpret_cast<intx4*>(a.pe16 + (((size_t)u * F + f) * kT + tt) * kDS) = *reinterpret_cast<const intx4*>(pe2);
      }
    }
    __syncthreads();
    strip_block<P, CINP, CHP, TAILM>(prm, X, WB, b, u, f_start, 1, wm, first, nb, nu, nfs, fn, nullptr, nullptr, true);
    return;
  }
  SepStage<CINP, kHID> w1;
  // NRX_INIT_ORDER: the y / h / pe loads (the norm -> z chain) go out first; the conv1
  // weights and the pad zeroing follow them
  if (!NRX_INIT_ORDER) {
    pad_zero();
    if constexpr (P::WLDS) w1.load(prm.w[0]);
  }
  // small grids: the slot norm's y loads go out first, beside the z-row loads below
  const float* yslot = a.y + (size_t)b * F * kT * A2;
  const int nqs = F * kT * A2 / 4;
  NormPre npre;
  if (!prm.norm_pre) npre = slot_norm_issue(yslot, nqs);
  static_assert(R0 * kTP <= 512, "one z row per thread");
  {
    const int lf = nrx_tid() / kTP, tt = nrx_tid() % kTP;
    const int f = f_start + lf;
    const bool ok = lf < R0 && tt < kT && f >= 0 && f < F;
    float yv[A2P], hv[A2P];
    const size_t re = ((size_t)b * F + (ok ? f : 0)) * kT + (ok ? tt : 0);
    const float* yp = a.y + re * A2;
    const float* hp = a.h_hat + (((size_t)b * U + u) * F * kT + (re - (size_t)b * F * kT)) * A2;
    // every load unconditional from a clamped address (row 0 / last pair of the row) and
    // masked afterwards: a load under a per-element runtime condition makes the compiler
    // branch around it and wait for each one in turn.  16-byte loads when 2A % 4 == 0.
    if ((A2 & 3) == 0) {
      const int nk = A2 / 4;
      float4 yl[A2P / 4], hl[A2P / 4];
#pragma unroll
      for (int k = 0; k < A2P / 4; ++k) yl[k] = reinterpret_cast<const float4*>(yp)[k < nk ? k : nk - 1];
#pragma unroll
      for (int k = 0; k < A2P / 4; ++k) hl[k] = float4{0.f, 0.f, 0.f, 0.f};
      if (a.use_h) {
#pragma unroll
        for (int k = 0; k < A2P / 4; ++k) hl[k] = reinterpret_cast<const float4*>(hp)[k < nk ? k : nk - 1];
      }
#pragma unroll
      for (int k = 0; k < A2P / 4; ++k) {
        const bool on = ok && k < nk;
        yv[4 * k] = on ? yl[k].x : 0.f;
        yv[4 * k + 1] = on ? yl[k].y : 0.f;
        yv[4 * k + 2] = on ? yl[k].z : 0.f;
        yv[4 * k + 3] = on ? yl[k].w : 0.f;
        hv[4 * k] = on ? hl[k].x : 0.f;
        hv[4 * k + 1] = on ? hl[k].y : 0.f;
        hv[4 * k + 2] = on ? hl[k].z : 0.f;
        hv[4 * k + 3] = on ? hl[k].w : 0.f;
      }
    } else {
      const int nk = A2 / 2;
      float2 yl[A2P / 2], hl[A2P / 2];
#pragma unroll
      for (int k = 0; k < A2P / 2; ++k) yl[k] = reinterpret_cast<const float2*>(yp)[k < nk ? k : nk - 1];
#pragma unroll
      for (int k = 0; k < A2P / 2; ++k) hl[k] = float2{0.f, 0.f};
      if (a.use_h) {
#pragma unroll
        for (int k = 0; k < A2P / 2; ++k) hl[k] = reinterpret_cast<const float2*>(hp)[k < nk ? k : nk - 1];
      }
#pragma unroll
      for (int k = 0; k < A2P / 2; ++k) {
        const bool on = ok && k < nk;
        yv[2 * k] = on ? yl[k].x : 0.f;
        yv[2 * k + 1] = on ? yl[k].y : 0.f;
        hv[2 * k] = on ? hl[k].x : 0.f;
        hv[2 * k + 1] = on ? hl[k].y : 0.f;
      }
    }
    float2 pv = *reinterpret_cast<const float2*>(a.pe + (((size_t)u * F + (ok ? f : 0)) * kT + (ok ? tt : 0)) * 2);
    if (!ok) pv = float2{0.f, 0.f};
    if constexpr (sizeof(S) == 2) {
      // one-launch forward: the pe16 chunk of this item's own rows for the update items' conv1
      // (every slot's StateInit items write the same bytes for a user's rows)
      if (a.pe16 && ok && lf >= kHalo && lf < kHalo + P::FO) {
        S pe2[8] = {};
        pe2[0] = (S)pv.x;
        pe2[1] = (S)pv.y;
        *reinterpret_cast<intx4*>(a.pe16 + (((size_t)u * F + f) * kT + tt) * kDS) = *reinterpret_cast<const intx4*>(pe2);
      }
    }
    stamp(33);
    if (NRX_INIT_ORDER) {
      if constexpr (P::WLDS) w1.load(prm.w[0]);
      pad_zero();
    }
    // large grids: the per-slot k_norm pass already reduced y (every workgroup of the slot
    // re-reading the whole grid costs O(strips x grid) there); small grids: fused here
    const Real ns = prm.norm_pre ? (Real)a.norm[b] : (Real)slot_norm(npre, yslot, nqs, red);
    stamp(36);
    if (lf < R0) {
#pragma unroll
      for (int q = 0; q < NQZ; ++q) {
        S o[P::EPC];
#pragma unroll
        for (int e = 0; e < P::EPC; ++e) {
          const int c = q * P::EPC + e;
          Real v = 0;
          if (c < A2P) v = f32_rounded((Real)yv[c] * ns);
          else if (c < 2 * A2P) v = f32_rounded((Real)hv[c - A2P] * ns);
          else if (c == 2 * A2P) v = (Real)pv.x;
          else if (c == 2 * A2P + 1) v = (Real)pv.y;
          o[e] = (S)v;
        }
        *reinterpret_cast<intx4*>(X + xoff<P, NQZ>(lf, tt, q)) = *reinterpret_cast<const intx4*>(o);
      }
    }
  }
  stamp(37);
  if constexpr (P::WLDS) w1.store(WB);
  stamp(39);
  __syncthreads();
  stamp(1);
  strip_block<P, CINP, CHP, TAILM>(prm, X, WB, b, u, f_start, 1, wm, first, nb, nu, nfs, fn);
  stamp(4);
}

// Zero the pad symbols t = 14, 15 of every slot of the 128-channel strip image (the conv
// layers never write them; their depthwise reads them as the T = 14 SAME padding).
template <class P>
__device__ __forceinline__ void zero_pad_symbols(char* X) {
  constexpr int NQ = kHID * (int)sizeof(typename P::S) / 16;
  for (int idx = nrx_tid(); idx < strip_slots<P>() * 2 * NQ; idx += 512) {
    const int q = idx % NQ, tt = kT + (idx / NQ) % 2, lf = idx / (2 * NQ);
    *reinterpret_cast<intx4*>(X + xoff<P, NQ>(lf, tt, q)) = intx4{0, 0, 0, 0};
  }
}

// Waves that issue the paired next item's z DMA: 0-3.  A burst of LDS-DMA issues stalls the
// issuing wave; with four issuing waves one wave of each SIMD pair issues while the other runs
// its epilogue (all eight: -1.5 %, after the item: -2.1 %, split before / after the epilogue:
// -1 %; profiles/r03/ab_fused_dma_placement.txt).
constexpr int kDmaWaves = 4;

// 16 zero bytes: the LDS-DMA source of every z chunk that is zero (pad symbols, rows
// outside the grid, channel padding, the missing other user of U = 1)
__device__ intx4 g_zero16[1];

#ifndef NRX_ZDMA
#define NRX_ZDMA 1
#endif

// f16 update z-load for U <= 2 as LDS-DMA (global_load_lds_dwordx4): with at most one
// other user the leave-one-out mean is a plain copy of that user's act*sp plane (p = 1 for
// any activity pattern of two users), so every 16-byte chunk of the z image is a copy of
// one global chunk or zero, and the image is filled with no VGPR round trip and no LDS
// store instructions.  One wave-instruction fills 1 KB of LDS linearly (4 symbols x 16
// chunks of one slot); the chunk swizzle is applied on the source address (the lane at
// physical chunk q' of symbol t loads logical chunk q' ^ swz(t)).  The pe chunk (2 values)
// is written by ds_write after the DMA has landed.  Every lane loads (zero chunks from
// g_zero16): EXEC-masking the pe / pad-symbol lanes was 0.9 % slower (profiles/r03/
// ab_zdma_skip.txt).
template <class P, int NW = 8>
__device__ __forceinline__ void zload_dma_u2(const BlockParams<P>& prm, char* X, int b, int u, int f_start) {
  using S = typename P::S;
  static_assert(sizeof(S) == 2 && kUPD_CINP * 2 / 16 == 16, "f16 z image with 16 chunks per symbol row");
  // the lane's symbol group is fixed at 4 (wave & 3) + tq and instruction k steps by NW: that
  // matches k's symbol group 4 (k & 3) + tq only when NW is a multiple of 4 and the issuing
  // waves 0 .. NW-1 cover every residue mod 4
  static_assert(NW % 4 == 0 && NW <= 8, "DMA-issuing wave count must be 4 or 8");
  constexpr int R0 = strip_slots<P>();
  constexpr int QS = kDS / P::EPC;   // 7 chunks of a, then 7 of s
  const auto& a = prm.a;
  const int F = a.F, U = a.U;
  const int lane = nrx_tid() & 63;
  const int wave = __builtin_amdgcn_readfirstlane(nrx_tid() >> 6);
  const int tq = lane >> 4, qp = lane & 15;
  const S* sp = a.s_in + srow(b, u, 0, 0, U, F);
  const S* ap = a.a + srow(b, U == 2 ? 1 - u : 0, 0, 0, U, F);
  const bool has_a = U == 2;
  typedef __attribute__((address_space(3))) void lds_void;
  typedef const __attribute__((address_space(1))) void glb_void;
  // instruction k = wave + 8 i covers slot r = (wave >> 2) + 2 i, symbols 4 (wave & 3) + tq:
  // the lane's symbol and chunk (hence its source plane and column) are loop-invariant, only
  // the slot advances, so the per-lane source is computed once and stepped by two grid rows
  const int t = 4 * (wave & 3) + tq;
  const int q = qp ^ swz<16>(t);
  const S* lsrc = nullptr;   // this lane's chunk in grid row 0 (null: always zero)
  if (t < kT) {
    if (q < QS) {
      if (has_a) lsrc = ap + t * kDS + P::EPC * q;
    } else if (q < 2 * QS) {
      lsrc = sp + t * kDS + P::EPC * (q - QS);
    }
  }
  if (wave >= NW) return;
  for (int k = wave; k < R0 * 4; k += NW) {
    const int f = f_start + (k >> 2);             // wave-uniform
    const S* src = reinterpret_cast<const S*>(g_zero16);
    if (f >= 0 && f < F && lsrc) src = lsrc + (size_t)f * (kT * kDS);
    __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(X + k * 1024), 16, 0, 0);
  }
}

template <class P, class WS, int CHP, int TAILM>
__device__ void EpiConv3<P, WS, CHP, TAILM>::next_hook() {
  if constexpr (kNextHook || kNextHookRO) {
    if (!next_ready()) return;   // fused forward: the next item's inputs were not complete
    zload_dma_u2<P, kDmaWaves>(nprm ? *nprm : *prm, X, nb, nu, nfs);
  }
}

// Rest of an update item whose z image is being filled by LDS-DMA (issued by the caller, or
// by the previous item's conv3 hook): conv1 weights, pe chunk once the DMA has landed, the
// block.  (nb, nu, nfs): the next item of a paired workgroup (nb < 0: none).
template <class P, int CHP, int TAILM>
__device__ __forceinline__ void dma_item_run(const BlockParams<P>& prm, char* X, char* WB, int b, int u, int f_start,
                                             int nb, int nu, int nfs, bool issue_z = false,
                                             FusedNext<P>* fn = nullptr) {
  using S = typename P::S;
  constexpr int R0 = strip_slots<P>();
  constexpr int NQ = kUPD_CINP * (int)sizeof(S) / 16;
  constexpr int QS = kDS / P::EPC;
  const auto& a = prm.a;
  const int F = a.F;
  SepStage<kUPD_CINP, kHID> w1;
  w1.load(prm.w[0]);
  const int pe_slot = nrx_tid() / kT, pe_t = nrx_tid() % kT;
  const int pe_f = f_start + pe_slot;
  const bool pe_ok = pe_slot < R0 && pe_f >= 0 && pe_f < F;
  const float2 pe_v = *reinterpret_cast<const float2*>(a.pe + (((size_t)u * F + (pe_ok ? pe_f : 0)) * kT + (pe_ok ? pe_t : 0)) * 2);
  // first item of a workgroup: its z DMA goes out behind the conv1-weight and pe loads, so
  // their latency hides under the DMA instead of following it
  if (issue_z) zload_dma_u2<P>(prm, X, b, u, f_start);
  stamp(24);
  stamp(25);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave's DMA has landed (and a previous item's epilogue is done)
  stamp(26);
  if (pe_slot < R0) {
    S pe2[P::EPC] = {};
    pe2[0] = pe_ok ? (S)pe_v.x : (S)0;
    pe2[1] = pe_ok ? (S)pe_v.y : (S)0;
    *reinterpret_cast<intx4*>(X + xoff<P, NQ>(pe_slot, pe_t, 2 * QS)) = *reinterpret_cast<const intx4*>(pe2);
  }
  w1.store(WB);
  stamp(27);
  __syncthreads();
  stamp(1);
  strip_block<P, kUPD_CINP, CHP, TAILM>(prm, X, WB, b, u, f_start, 0, 0, false, nb, nu, nfs, fn);
  stamp(4);
  if (nb >= 0) stamp(32);   // first item of a pair done
}


// A k_forward update item whose conv1 reads the z rows [a | s | pe] straight from memory
// (GZ): no z image in LDS, hence no z DMA and no pe chunk store; the prologue stages conv1's
// weights only, and conv1 writes all its output rows before its layer barrier.
template <class P, int CHP, int TAILM>
__device__ __forceinline__ void gz_item_run(const BlockParams<P>& prm, char* X, char* WB, int b, int u, int f_start,
                                            FusedNext<P>* fn, int* psig) {
  const auto& a = prm.a;
  SepStage<kUPD_CINP, kHID> w1;
  w1.load(prm.w[0]);
  GZ gz;
  gz.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(a.ws_base), 0, (int)a.ws_bytes, 0x00020000);
  gz.f_start = f_start;
  gz.F = a.F;
  const int lane = nrx_tid() & 63, t = lane & 15, g = lane >> 4;
  auto rel = [&](const void* p) { return (unsigned)(reinterpret_cast<const char*>(p) - a.ws_base); };
  const unsigned tb = (unsigned)(t * kDS * 2);
  const unsigned so = rel(a.s_in + srow(b, u, 0, 0, a.U, a.F)) + tb;
  // a: the other user's act*sp plane (U = 2, p = 1), none (U = 1), or the combined a_u plane
  // (U > 4: a combine stage ran in place)
  const unsigned ao = !prm.inline_combine ? rel(a.a + srow(b, u, 0, 0, a.U, a.F)) + tb
                      : a.U == 2          ? rel(a.a + srow(b, 1 - u, 0, 0, a.U, a.F)) + tb
                                          : kGzOob;
  const unsigned po = rel(a.pe16 + srow(0, u, 0, 0, a.U, a.F)) + tb;
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    const int q = 4 * kc + g;
    unsigned off = kGzOob;
    if (t < kT) {
      if (q < 7) off = ao == kGzOob ? kGzOob : ao + 16u * q;
      else if (q < 14) off = so + 16u * (q - 7);
      else if (q == 14) off = po;
    }
    gz.off[kc] = off;
  }
  // conv1's first K chunk for this wave's rows (conv_layer's split: 28 rows, waves 0-3 four,
  // 4-7 three), in flight during the weight staging and the barrier
  {
    constexpr int R0 = strip_slots<P>();
    static_assert(R0 - 2 - 24 == 4, "conv1 row split of the 24-row strip: 4 x 4 + 4 x 3");
    const int wave = __builtin_amdgcn_readfirstlane(nrx_tid() >> 6);
    const int p0 = 1 + 4 * (wave < 4 ? wave : 4) + 3 * (wave > 4 ? wave - 4 : 0);
#pragma unroll
    for (int i = 0; i < 6; ++i) gz.x0[i] = (i < 5 || wave < 4) ? gz.load(0, gz.row_soff(p0 - 1 + i)) : half8{};
  }
  // the previous item's stores drain during conv1 and its counter is added after conv1's
  // layer barrier (deferred signal, k_forward): the prologue waits for the conv1 weights only,
  // the z-row loads stay in flight across the barrier
  w1.store(WB);
  __syncthreads();
  stamp(1);
  strip_block<P, kUPD_CINP, CHP, TAILM, true>(prm, X, WB, b, u, f_start, 0, 0, false, -1, 0, 0, fn, &gz, psig);
  stamp(4);
}

#ifndef NRX_PAIR
#define NRX_PAIR 1
#endif
#ifndef NRX_W1_FIRST
#define NRX_W1_FIRST 1
#endif
#ifndef NRX_PAIR_RO
#define NRX_PAIR_RO 1
#endif

// Two update items (aggregation tail) per workgroup: item 1's z image is DMA'd into the
// strip image during item 0's epilogue (EpiConv3::next_hook), so its load overlaps that
// epilogue instead of stalling a chip-wide load phase of its own.
template <class P, int CHP, int TAILM>
__device__ __forceinline__ void update_pair(const BlockParams<P>& prm, char* smem, int b0, int u0, int s0, int b1,
                                            int u1, int s1) {
  constexpr int R0 = strip_slots<P>();
  char* X = smem;
  char* WB = smem + R0 * slot_pitch<P>();
  const int fs0 = s0 * P::FO - kHalo, fs1 = s1 * P::FO - kHalo;
  if (!NRX_W1_FIRST) zload_dma_u2<P>(prm, X, b0, u0, fs0);
  dma_item_run<P, CHP, TAILM>(prm, X, WB, b0, u0, fs0, b1, u1, fs1, NRX_W1_FIRST != 0);
  dma_item_run<P, CHP, TAILM>(prm, X, WB, b1, u1, fs1, -1, 0, 0);
}

// UpdateState of user u on the strip (z = [a, s, pe]).
// fn / psig: a k_forward item (U > 2: the z image with the inline leave-one-out combine is
// staged here, not read by conv1 from memory): the next item's dependency poll, and the
// previous item's deferred counter add (after this item's loads and the layer barrier).
template <class P, int CHP, int TAILM>
__device__ __forceinline__ void update_user(const BlockParams<P>& prm, char* smem, int b, int u, int strip,
                                            FusedNext<P>* fn = nullptr, int* psig = nullptr) {
  using S = typename P::S;
  constexpr int R0 = strip_slots<P>();
  constexpr int NQ = kUPD_CINP * (int)sizeof(S) / 16;  // chunks per z row
  constexpr int QS = kDS / P::EPC;                      // chunks of a (and of s) in z
  const auto& a = prm.a;
  const int F = a.F, U = a.U;
  const int f0 = strip * P::FO;
  const int f_start = f0 - kHalo;
  char* X = smem;
  char* WB = smem + R0 * slot_pitch<P>();
  if constexpr (sizeof(S) == 2 && NRX_ZDMA != 0) {
    if (prm.inline_combine && U <= 2 && !fn) {
      if (!NRX_W1_FIRST) zload_dma_u2<P>(prm, X, b, u, f_start);
      dma_item_run<P, CHP, TAILM>(prm, X, WB, b, u, f_start, -1, 0, 0, NRX_W1_FIRST != 0);
      return;
    }
  }
  // z chunks: [0,QS) <- a, [QS,2QS) <- s, 2QS <- pe (2 values), rest 0.
  // a_u = (sum_u' sp_u' - sp_u) * p is formed here from the producer's act*sp rows when
  // U <= kInlineUsers (AggregateUserStates' leave-one-out mean, neural_rx.py:191-204);
  // otherwise k_combine already wrote a_u in place.
  // The in-grid rows [lo, hi) of a (b, u) plane are one contiguous range of the compact
  // [F][14][56] layout (K = 14 * QS chunks per row).  Fixed thread -> (row phase, symbol,
  // chunk) mapping: thread tid handles chunk k = tid % K of image rows r = tid / K + RG * i,
  // so per iteration only the row advances (one add on the global and on the LDS offset; no
  // divisions) and rows outside the grid store zeros in the same pass.  All global loads are
  // issued first (32-bit offsets from wave-uniform bases), then the LDS stores.
  using Real = typename P::Real;
  constexpr int K = kT * QS;               // chunks per row of one plane
  constexpr int RG = 512 / K;              // image rows per iteration (P16: 5, P64: 2)
  constexpr int PV = (R0 + RG - 1) / RG;   // iterations (P16: 6, P64: 7)
  const int lo = f_start < 0 ? 0 : f_start;
  const int hi = f_start + R0 < F ? f_start + R0 : F;
  const int slot_lo = lo - f_start, nrow = hi - lo;
  const bool inl = prm.inline_combine != 0;
  // planes read for a: inline -> the U-1 other users' act*sp rows; else the combined a_u
  const int no = inl ? U - 1 : 1;
  SepStage<kUPD_CINP, kHID> w1;
  if constexpr (P::WLDS) w1.load(prm.w[0]);
  const intx4* sb = reinterpret_cast<const intx4*>(a.s_in + srow(b, u, lo, 0, U, F));
  const intx4* ab[kInlineUsers - 1];
#pragma unroll
  for (int k = 0; k < kInlineUsers - 1; ++k) {
    const int uu = inl ? (k < u ? k : k + 1) : u;
    ab[k] = reinterpret_cast<const intx4*>(a.a + srow(b, uu < U ? uu : 0, lo, 0, U, F));
  }
  const int kk = nrx_tid() % K, r0 = nrx_tid() / K;
  const bool lane_on = r0 < RG;
  const int tk = kk / QS, qk = kk % QS;
  intx4 vs[PV], va[PV][kInlineUsers - 1];
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int rr = r0 + RG * i - slot_lo;           // plane row of image row r0 + RG i
    const bool ld = lane_on && rr >= 0 && rr < nrow && !(NRX_ABLATE & 2);
    const unsigned c = ld ? (unsigned)(rr * K + kk) : 0u;   // clamped: chunk 0, not stored
    vs[i] = sb[c];
#pragma unroll
    for (int k = 0; k < kInlineUsers - 1; ++k) va[i][k] = k < no ? ab[k][c] : intx4{0, 0, 0, 0};
  }
  // pe chunk (2 values) of z row (slot, t < 14): one row per thread, loaded with the rest
  static_assert(R0 * kT <= 512, "one pe row per thread");
  const int pe_slot = nrx_tid() / kT, pe_t = nrx_tid() % kT;
  const int pe_f = f_start + pe_slot;
  const bool pe_ok = pe_slot < R0 && pe_f >= 0 && pe_f < F;
  // unconditional load from a clamped address (no branch around it: a conditional load
  // makes the compiler convert right after it, i.e. wait for every load issued above)
  const float2 pe_v = *reinterpret_cast<const float2*>(
      a.pe + (((size_t)u * F + (pe_ok ? pe_f : 0)) * kT + (pe_ok ? pe_t : 0)) * 2);
  stamp(24);
  // zero chunks while the loads fly: the pad symbols t = 14, 15 of every slot are one
  // contiguous 2 * NQ-chunk block at the end of the slot's symbol rows (whatever the swizzle)
  {
    constexpr int ZS = 2 * NQ;                       // chunks per slot (power of 2)
    static_assert((ZS & (ZS - 1)) == 0, "pad block size");
    for (int idx = nrx_tid(); idx < R0 * ZS; idx += 512)
      *reinterpret_cast<intx4*>(X + (idx / ZS) * slot_pitch<P>() + (kT * NQ + idx % ZS) * 16) = intx4{0, 0, 0, 0};
  }
  stamp(25);
  if (pe_slot < R0) {
    // pe chunk 2QS and the pad chunks (2QS, NQ) of symbol row (pe_slot, pe_t)
    S pe2[P::EPC] = {};
    pe2[0] = pe_ok ? (S)pe_v.x : (S)0;
    pe2[1] = pe_ok ? (S)pe_v.y : (S)0;
    *reinterpret_cast<intx4*>(X + xoff<P, NQ>(pe_slot, pe_t, 2 * QS)) = *reinterpret_cast<const intx4*>(pe2);
#pragma unroll
    for (int q = 2 * QS + 1; q < NQ; ++q)
      *reinterpret_cast<intx4*>(X + xoff<P, NQ>(pe_slot, pe_t, q)) = intx4{0, 0, 0, 0};
  }
  Real pf = 1;
  if (inl) {
    Real nact = 0;
    for (int uu = 0; uu < U; ++uu) nact += (Real)a.active[(size_t)b * U + uu];
    pf = nact - (Real)1;
    pf = pf > (Real)0 ? (Real)1 / pf : (Real)1;
  }
  // LDS offsets of this thread's a / s chunks in image row r0 (+ RG i rows per iteration)
  const int oa = xoff<P, NQ>(r0, tk, qk), os = xoff<P, NQ>(r0, tk, QS + qk);
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int r = r0 + RG * i;
    if (lane_on && r < R0) {
      const int rr = r - slot_lo;
      const bool in = rr >= 0 && rr < nrow;
      intx4 out = va[i][0];
      if (inl) {
        // a_u = p * sum of the other users' act*sp (packed f16 adds in the f16 policy; one
        // plane with p = 1, e.g. U = 2 with a 0/1 mask, stays exact)
        if constexpr (sizeof(S) == 2) {
          half8 sm = __builtin_bit_cast(half8, va[i][0]);
#pragma unroll
          for (int k = 1; k < kInlineUsers - 1; ++k)
            if (k < no) sm += __builtin_bit_cast(half8, va[i][k]);
          if (pf != (Real)1) sm *= (_Float16)pf;
          out = no > 0 ? __builtin_bit_cast(intx4, sm) : intx4{0, 0, 0, 0};
        } else {
          S o[P::EPC];
#pragma unroll
          for (int e = 0; e < P::EPC; ++e) {
            Real sum = 0;
#pragma unroll
            for (int k = 0; k < kInlineUsers - 1; ++k)
              if (k < no) sum += (Real)reinterpret_cast<const S*>(&va[i][k])[e];
            o[e] = (S)(sum * pf);
          }
          out = *reinterpret_cast<const intx4*>(o);
        }
      }
      *reinterpret_cast<intx4*>(X + oa + RG * i * slot_pitch<P>()) = in ? out : intx4{0, 0, 0, 0};
      *reinterpret_cast<intx4*>(X + os + RG * i * slot_pitch<P>()) = in ? vs[i] : intx4{0, 0, 0, 0};
    }
  }
  stamp(26);
  if constexpr (P::WLDS) w1.store(WB);
  stamp(27);
  if (psig) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the previous item's stores
  __syncthreads();
  if (psig && nrx_tid() == 0) __hip_atomic_fetch_add(psig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(1);
  strip_block<P, kUPD_CINP, CHP, TAILM>(prm, X, WB, b, u, f_start, 0, 0, false, -1, 0, 0, fn);
  stamp(4);
}

// ------------------------------------------------------------ work-item placement
// 1-D grid of B * U * strips workgroups.  Workgroups are dispatched to the 8 XCDs round-
// robin by linear id (cdna_hip_programming.md T1: id % 8 labels the XCD), so the items of
// one slot -- which exchange users' aggregates and strip halos through HBM between
// launches -- are given ids with one residue mod 8: everything a workgroup reads was
// written on its own XCD, through its L2.  Consecutive launches alternate the order within
// an XCD (order_rev) so that the items written last, the most likely still in L2, are
// read first.  Slots beyond the last complete group of 8 keep the plain order.
__device__ __forceinline__ void work_item(int i, int B, int U, int S, int rev, int& b, int& u, int& strip) {
  const int ips = U * S;
  const int per_xcd = (B / 8) * ips;
  int k;
  if (i < 8 * per_xcd) {
    const int x = i % 8;
    int j = i / 8;
    if (rev) j = per_xcd - 1 - j;
    b = 8 * (j / ips) + x;
    k = j % ips;
  } else {
    b = i / ips;
    k = i % ips;
  }
  u = k / S;
  strip = k % S;
}

// ------------------------------------------------------------ user combine (U > 4)
// Leave-one-out mean over users (neural_rx.py:191-204) in place: a_u = (sum_u' sp_u' -
// sp_u) * p, sp_u already scaled by act_u, p = 1/max(#active - 1) (1 when <= 1 active).
// For U <= kInlineUsers the update kernel's z-load forms a_u itself and this is not run.
// grid = (ceil(F*14*QS / 256), B), 256 threads, one 16-byte chunk of a row per thread.
template <class P>
__global__ __launch_bounds__(256) void k_combine(typename P::S* __restrict__ buf, const float* __restrict__ active,
                                                 int U, int F) {
  using S = typename P::S;
  using Real = typename P::Real;
  constexpr int QS = kDS / P::EPC;
  const int b = blockIdx.y;
  const int idx = blockIdx.x * 256 + nrx_tid();
  if (idx >= F * kT * QS) return;
  const size_t ustride = (size_t)F * kT * kDS;
  S* base = buf + (size_t)b * U * ustride + (size_t)(idx / QS) * kDS + (idx % QS) * P::EPC;
  Real nact = 0;
  for (int u = 0; u < U; ++u) nact += (Real)active[(size_t)b * U + u];
  Real p = nact - (Real)1;
  p = p > (Real)0 ? (Real)1 / p : (Real)1;
  Real sum[P::EPC];
#pragma unroll
  for (int e = 0; e < P::EPC; ++e) sum[e] = 0;
  for (int u = 0; u < U; ++u) {
    const intx4 v = *reinterpret_cast<const intx4*>(base + u * ustride);
    const S* sv = reinterpret_cast<const S*>(&v);
#pragma unroll
    for (int e = 0; e < P::EPC; ++e) sum[e] += (Real)sv[e];
  }
  for (int u = 0; u < U; ++u) {
    const intx4 v = *reinterpret_cast<const intx4*>(base + u * ustride);
    const S* sv = reinterpret_cast<const S*>(&v);
    S o[P::EPC];
#pragma unroll
    for (int e = 0; e < P::EPC; ++e) o[e] = (S)f32_rounded((sum[e] - (Real)sv[e]) * p);
    *reinterpret_cast<intx4*>(base + u * ustride) = *reinterpret_cast<const intx4*>(o);
  }
}

// StateInit_m (+ Var-IO mix: one launch per m, m > 0 accumulating) of one (slot, user,
// strip); the last launch applies the aggregation MLP of iteration 0 (stores act * sp).
// grid = (strips, U, B).
template <class P, int A2P, int TAILM>
__global__ __launch_bounds__(512) void k_init(BlockParams<P> prm) {
  using Real = typename P::Real;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const auto& a = prm.a;
  int b, u, strip;
  work_item(blockIdx.x, prm.a.B, prm.a.U, prm.strips, prm.order_rev, b, u, strip);
  const int U = a.U;
  const int m = prm.m;
  Real wm = (Real)1;
  if (!a.masking)
    wm = a.mcs_mask ? (Real)a.mcs_mask[((size_t)b * U + u) * a.M + m] : (Real)(m == 0 ? 1 : 0);
  // wm == 0: this MCS contributes exactly 0 * finite; the conv math is still run (the
  // m = 0 launch defines s, the last launch applies the aggregation MLP).
  stamp(0);
  init_user<P, A2P, 16, TAILM>(prm, smem, b, u, strip, wm, m == 0);
  stamp(5);
}

#ifndef NRX_UPDATE_GZ
#define NRX_UPDATE_GZ 1
#endif
// UpdateState of one (slot, user, strip) with the fused tail.  grid = (strips, U, B).
template <class P, int CHP, int TAILM>
__global__ __launch_bounds__(512) void k_update(BlockParams<P> prm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int b, u, strip;
  work_item(blockIdx.x, prm.a.B, prm.a.U, prm.strips, prm.order_rev, b, u, strip);
  stamp(0);
  if constexpr (std::is_same<P, P16>::value) {
    if (prm.gz) {
      // conv1 reads its z rows [a | s | pe] from L2 / HBM (GZ, as k_forward's update items): no
      // z image, so neither the first item's chip-wide z load nor the paired item's DMA
      constexpr int R0 = strip_slots<P>();
      char* X = smem;
      char* WB = smem + R0 * slot_pitch<P>();
      zero_pad_symbols<P>(X);
      gz_item_run<P, CHP, TAILM>(prm, X, WB, b, u, strip * P::FO - kHalo, nullptr, nullptr);
      if (prm.pair) {
        int b1, u1, s1;
        work_item(blockIdx.x + gridDim.x, prm.a.B, prm.a.U, prm.strips, prm.order_rev, b1, u1, s1);
        __syncthreads();   // every wave is past the first item's epilogue (WB, X)
        gz_item_run<P, CHP, TAILM>(prm, X, WB, b1, u1, s1 * P::FO - kHalo, nullptr, nullptr);
      }
      stamp(5);
      return;
    }
  }
  if constexpr ((TAILM == TAIL_AGG || TAILM == TAIL_READOUT_WB) && P::WLDS && NRX_PAIR != 0 && NRX_ZDMA != 0) {
    if (prm.pair) {
      int b1, u1, s1;
      work_item(blockIdx.x + gridDim.x, prm.a.B, prm.a.U, prm.strips, prm.order_rev, b1, u1, s1);
      update_pair<P, CHP, TAILM>(prm, smem, b, u, strip, b1, u1, s1);
      stamp(5);
      return;
    }
  }
  update_user<P, CHP, TAILM>(prm, smem, b, u, strip);
  stamp(5);
}

// ================================================================ fused forward (one launch)
// The whole forward -- StateInit, the num_it state updates and the readouts (neural_rx.py:
// 544-595) -- as ONE persistent launch, one 512-thread workgroup per CU.  The launch
// boundaries of the three-launch forward cost every update launch a chip-wide lockstep
// z-load of its first item (~10 k of ~90 k cycles per CU: all CUs fetch at once) plus the
// drain/fill of the launch; here a workgroup runs a stream of items and the z image of its
// next update item is DMA'd during the current item's conv3 epilogue, whatever stage that
// item belongs to.
//
// Work queues.  One queue per XCD (the workgroup reads its XCC id from the hardware), holding
// the items of the slots b with b % nq == queue in stage-major order: stage 0 (StateInit),
// then each update; inside a stage slot by slot, (user, strip) within the slot.  A workgroup
// dequeues with one atomic per item (one item ahead, so the next item is known during the
// current one's conv3).  An item of stage s >= 1 reads the stage s-1 outputs of its slot
// (its own and the other user's rows, both strips through the halo), so it waits for the
// slot's counter done[s-1][b] to reach U * strips.  Items are dequeued in that topological
// order, and an item only waits for items dequeued before it, i.e. held by workgroups that
// are running: no deadlock whatever the residency.  The bounded spin (~0.5 s) is a guard
// only; a timeout sets a sticky error word (nrx_fused_status).
//
// Visibility.  Producer and consumer of a hand-off run on the same XCD by construction (the
// queue is chosen by the XCC id read at run time, not by dispatch order), so the plain
// 16-byte state stores are in the shared L2 once the storing wave's vmcnt has drained; the
// producer then signals after a workgroup barrier (one agent-scope atomic add per item).
// The consumer polls with an sc1 (L1-bypassing) load and invalidates its CU's L1 (buffer_inv
// sc1) before any load of the handed-off rows: the ping-pong state buffers were read by this
// CU two stages earlier (MI355X_MICROARCH.md, inter-workgroup visibility).  The counters
// live in a handle-owned buffer and are reset by the last workgroup to leave.
struct FusedSync {
  int head[8];   // per-queue work counters
  int exits;     // workgroups that left the loop
  int err;       // sticky: a dependency wait timed out
  int waited;    // update items whose z image was not prefetched (dependency not met in time)
  int spins;     // dependency-wait polls of those items
  int pad[4];
  // int done[kFusedMaxStages][B] follows
};
constexpr int kFusedMaxStages = 12;  // StateInit (x M for Var-IO) + the updates (8 for nrx_large);
                                     // FusedParams ~7.5 KB of kernel arguments (16 KB measured to
                                     // pass, tools/ubench/kernarg.hip)
// dynamic LDS of k_forward: the paired-readout layout minus room for the static __shared__
// words (the slot-norm reduction of StateInit, the queue words); the readout heads must fit
constexpr int kFusedLds = 160 * 1024 - 256;
// dynamic LDS of k_forward per strip tier: the 24-row tier's paired-readout layout fills the
// LDS, so it gives up 256 bytes of WB; the small-grid tiers (8 / 16-row strips) fit whole
template <class P>
constexpr int fused_lds() {
  return strip_lds_bytes<P>(true) > kFusedLds ? kFusedLds : strip_lds_bytes<P>(true);
}
constexpr int kFusedMaxB = 65536;
// logical stages: the StateInit stages, then per iteration (U > kInlineUsers) a combine stage
// and the update stage; one dependency counter row each
constexpr int kFusedMaxLS = 20;
constexpr size_t kFusedSyncBytes = sizeof(FusedSync) + (size_t)kFusedMaxLS * kFusedMaxB * sizeof(int);

template <class P>
struct FusedParams {
  BlockParams<P> st[kFusedMaxStages];   // 0..ninit-1: StateInit m, ninit..nst-1: updates
  FusedSync* sync;
  int nst;                              // ninit + num_it
  int ninit;                            // StateInit stages (M for Var-IO, else 1)
  int nls;                              // logical stages (GEN)
  int kind[kFusedMaxLS];                // GEN: 0 StateInit, 1 update, 2 leave-one-out combine
  int pidx[kFusedMaxLS];                // GEN: the stage's st[] entry (combine: its update's)
  int heads_x;                          // readout heads staged in the strip image (H > 1)
  int gz;                               // update items: conv1 reads z from memory (U <= 2, the
                                        // workspace within the 32-bit buffer range); else
                                        // the z image is staged in LDS (update_user)
  int nq;                               // queues (XCDs)
  int spin_limit;                       // dependency-wait polls before the timeout error
  int dbg_err;                          // debug: error bits workgroup 0 sets (nrx_debug_fused)
};

__device__ __forceinline__ int xcc_id() {
  return (int)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // hwreg(HW_REG_XCC_ID, 0, 4)
}

// Thread 0 waits for *cnt >= need (bounded), then invalidates this CU's L1 before the
// workgroup loads the handed-off rows.
__device__ __forceinline__ void fused_wait(const int* cnt, int need, FusedSync* sy, int limit) {
  if (nrx_tid() == 0) {
    int it = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
      __builtin_amdgcn_s_sleep(4);
      if (++it > limit) {
        __hip_atomic_fetch_or(&sy->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (it) {
      __hip_atomic_fetch_add(&sy->waited, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&sy->spins, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("buffer_inv sc1" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// A combine item of k_forward (U > kInlineUsers): the leave-one-out mean of one (slot, strip),
// in place over the act*sp rows of every user -- k_combine's arithmetic (f32 sum over u in
// order, then (sum - sp_u) * p), so the outputs equal the three-launch forward's.  Its rows
// are its own strip's (no halo); the next update stage waits for all strips of the slot.  It
// runs no conv2, so the next item's dependency poll is done at its end.
constexpr int kFusedMaxUsers = 8;
template <class P>
__device__ __forceinline__ void combine_item(const BlockParams<P>& prm, int b, int strip, FusedNext<P>* fn) {
  using S = typename P::S;
  using Real = typename P::Real;
  constexpr int QS = kDS / P::EPC;
  if (nrx_tid() == 0) fn->jnn = atomicAdd(fn->head, 1);
  const auto& a = prm.a;
  const int U = a.U, F = a.F;
  const int f0 = strip * P::FO, f1 = f0 + P::FO < F ? f0 + P::FO : F;
  const size_t ustride = (size_t)F * kT * kDS;
  S* buf = const_cast<S*>(a.a) + (size_t)b * U * ustride + (size_t)f0 * kT * kDS;
  Real nact = 0;
  for (int uu = 0; uu < U; ++uu) nact += (Real)a.active[(size_t)b * U + uu];
  Real p = nact - (Real)1;
  p = p > (Real)0 ? (Real)1 / p : (Real)1;
  const int n = (f1 - f0) * kT * QS;
  for (int idx = nrx_tid(); idx < n; idx += 512) {
    S* base = buf + (size_t)(idx / QS) * kDS + (idx % QS) * P::EPC;
    // every user's chunk in flight at once (one workgroup per CU: a load-use chain per user
    // would leave the CU waiting U memory latencies per chunk)
    intx4 vv[kFusedMaxUsers];
#pragma unroll
    for (int uu = 0; uu < kFusedMaxUsers; ++uu)
      vv[uu] = uu < U ? *reinterpret_cast<const intx4*>(base + uu * ustride) : intx4{0, 0, 0, 0};
    Real sum[P::EPC];
#pragma unroll
    for (int e = 0; e < P::EPC; ++e) sum[e] = 0;
#pragma unroll
    for (int uu = 0; uu < kFusedMaxUsers; ++uu) {
      if (uu >= U) break;
      const S* sv = reinterpret_cast<const S*>(&vv[uu]);
#pragma unroll
      for (int e = 0; e < P::EPC; ++e) sum[e] += (Real)sv[e];
    }
#pragma unroll
    for (int uu = 0; uu < kFusedMaxUsers; ++uu) {
      if (uu >= U) break;
      const S* sv = reinterpret_cast<const S*>(&vv[uu]);
      S o[P::EPC];
#pragma unroll
      // rounded to f32 before the storage conversion (as k_combine: no fused single-rounding
      // multiply-convert in one kernel family and not in the other)
      for (int e = 0; e < P::EPC; ++e) o[e] = (S)f32_rounded((sum[e] - (Real)sv[e]) * p);
      *reinterpret_cast<intx4*>(base + uu * ustride) = *reinterpret_cast<const intx4*>(o);
    }
  }
  if (nrx_tid() == 0) {
    int v = 0;
    if (fn->ndone) {
      v = __hip_atomic_load(fn->ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= fn->nneed;
      asm volatile("buffer_inv sc1" ::: "memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *fn->nflag = v;
  }
}

// MODE 0: one StateInit, one head in WB, GZ updates (the bench shape); 1: the general stage
// list with GZ updates (Var-IO StateInit stages, readout heads in the strip image); 2: staged
// z images (U > 2 or a workspace beyond GZ's offsets) with combine stages for U > 4.  Each
// kernel carries only its own item code: compiling the general list into the bench kernel grew
// it from 141 KB to 237 KB and cost 3.5 % (profiles/r04/ab_fused_gen.txt).
template <class P, int A2P, int CHP, int MODE>
__global__ __launch_bounds__(512) void k_forward(FusedParams<P> fp_arg) {
  constexpr bool GEN = MODE != 0;
  constexpr bool STAGED = MODE == 2;
  // the stage parameters are read through the kernarg segment pointer: indexing the by-value
  // parameter with the (dynamic) stage made the compiler copy the whole struct to scratch
  typedef const __attribute__((address_space(4))) FusedParams<P> KFP;
  const FusedParams<P>& fp = *(const FusedParams<P>*)(KFP*)__builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int sh[4];   // 0, 1: dequeued items; 2: next z DMA issued; 3: last workgroup
  constexpr int R0 = strip_slots<P>();
  char* X = smem;
  char* WB = smem + R0 * slot_pitch<P>();
  FusedSync* sy = fp_arg.sync;   // scalars straight from the parameter (keeps it in the kernarg list)
  int* done = reinterpret_cast<int*>(sy + 1);
  const int nst = fp_arg.nst, ninit = fp_arg.ninit, nqs = fp_arg.nq, spin_limit = fp_arg.spin_limit;
  const auto& a0 = fp.st[0].a;
  const int B = a0.B, U = a0.U, strips = fp.st[0].strips;
  const int ips = U * strips;   // items per (stage, slot) = a slot's dependency count
  const int q = xcc_id() % nqs;
  const int nbq = (B - q + nqs - 1) / nqs;
  const int per_stage = nbq * ips;
  // logical stages: the plain kernel has StateInit stages then updates, ips items per slot
  // each; GEN adds a combine stage (one item per (slot, strip)) before each update when U > 4
  const int nls = GEN ? fp_arg.nls : nst;
  auto kind_of = [&](int ls) -> int {
    if constexpr (GEN) return fp.kind[ls];
    else return ls < ninit ? 0 : 1;
  };
  auto pidx_of = [&](int ls) -> int {
    if constexpr (GEN) return fp.pidx[ls];
    else return ls;
  };
  auto ips_of = [&](int ls) -> int {
    if constexpr (GEN) return fp.kind[ls] == 2 ? strips : ips;
    else return ips;
  };
  int total = nst * per_stage;
  if constexpr (GEN) {
    total = 0;
    for (int ls = 0; ls < nls; ++ls) total += nbq * ips_of(ls);
  }
  int* head = &sy->head[q];
  if (nrx_tid() == 0) {
    // two separate dequeues: with one atomic for both (round 3, d1f0f90) a workgroup's first
    // two items were consecutive, so a slot's StateInit items all ran as second items and the
    // first update item of every workgroup found its slot incomplete (1 of 4 update items
    // un-prefetched)
    sh[0] = atomicAdd(head, 1);
    sh[1] = atomicAdd(head, 1);
    if (fp_arg.dbg_err && blockIdx.x == 0)
      __hip_atomic_fetch_or(&sy->err, fp_arg.dbg_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  int j = sh[0], jn = sh[1];
  bool have_z = false;      // item j's inputs were complete and acquired during the previous item
  bool pads_zero = false;   // the strip image's pad symbols were zeroed (by an earlier item)
  int* psig = nullptr;      // the previous item's dependency counter, not yet added
  auto decode = [&](int jj, int& s, int& b, int& u, int& strip) {
    int k = jj, ip = ips;
    if constexpr (GEN) {
      s = 0;
      for (;;) {
        ip = ips_of(s);
        if (k < nbq * ip || s == nls - 1) break;
        k -= nbq * ip;
        ++s;
      }
    } else {
      s = jj / per_stage;
      k = jj - s * per_stage;
    }
    b = q + nqs * (k / ip);
    const int r = k % ip;
    u = GEN && kind_of(s) == 2 ? 0 : r / strips;
    strip = r % strips;
  };
#ifdef NRX_STAMPS
  int n_item = 0;
#endif
  while (j < total) {
    int s, b, u, strip;
    decode(j, s, b, u, strip);
#ifdef NRX_STAMPS
    if (nrx_tid() == 0 && blockIdx.x < 4096) {
      g_fstamp_item[blockIdx.x] = n_item;
      if (n_item < 8 && g_nrx_stamp_on == 100) g_nrx_rr_stamps[blockIdx.x][8 * n_item + 7] = s + 1;
    }
    ++n_item;
    fstamp(0);
#endif
    int sn = 0, bn = 0, un = 0, stn = 0;
    if (jn < total) decode(jn, sn, bn, un, stn);
    // poll: the next item's dependency counter is read (and this CU's L1 invalidated) during
    // this item's conv2, so that a satisfied next item skips its prologue wait and acquire
    const bool poll = jn < total && sn >= 1;
    FusedNext<P> fn{&fp.st[poll ? pidx_of(sn) : 0], poll ? done + (sn - 1) * B + bn : nullptr,
                    poll ? ips_of(sn - 1) : ips, &sh[2], head, 0};
    const int kd = kind_of(s), ps = pidx_of(s);
    // deferred signal of the previous item: an update item whose inputs were acquired during
    // the previous item (no wait) drains and adds it in its prologue, behind its own loads;
    // otherwise first -- an item that waits must never wait on its own predecessor's signal
    if (psig && !(kd == 1 && have_z)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (nrx_tid() == 0) __hip_atomic_fetch_add(psig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      psig = nullptr;
    }
    if (s >= 1 && !have_z) fused_wait(done + (s - 1) * B + b, ips_of(s - 1), sy, spin_limit);
    if (kd == 0) {
      // StateInit m = s (Var-IO: one stage per MCS, accumulating s = sum_m mask_m SI_m,
      // neural_rx.py:562-569; the last one applies iteration 0's aggregation MLP)
      const auto& a = fp.st[s].a;
      float wm = 1.f;
      if (!a.masking) wm = a.mcs_mask ? a.mcs_mask[((size_t)b * U + u) * a.M + s] : (s == 0 ? 1.f : 0.f);
      if (!GEN || s == ninit - 1) init_user<P, A2P, 16, TAIL_AGG>(fp.st[s], smem, b, u, strip, wm, s == 0, -1, 0, 0, &fn);
      else if constexpr (GEN) init_user<P, A2P, 16, TAIL_NONE>(fp.st[s], smem, b, u, strip, wm, s == 0, -1, 0, 0, &fn);
    } else if (STAGED && kd == 2) {
      // U > 4: the leave-one-out combine of the slot's strip rows, in place (k_combine's pass)
      if constexpr (STAGED) combine_item<P>(fp.st[ps], b, strip, &fn);
    } else if (STAGED) {
      // U > 2 (or a workspace beyond GZ's 32-bit offsets): the z image is staged in the strip
      // image by update_user, as in the three-launch forward -- U = 3, 4 with the inline
      // leave-one-out combine of the U - 1 other users' act*sp rows, U > 4 from the combined
      // a_u plane (combine stage)
      if constexpr (STAGED) {
        if (ps < nst - 1) update_user<P, CHP, TAIL_AGG>(fp.st[ps], smem, b, u, strip, &fn, psig);
        else if (fp_arg.heads_x) update_user<P, CHP, TAIL_READOUT>(fp.st[ps], smem, b, u, strip, &fn, psig);
        else update_user<P, CHP, TAIL_READOUT_WB>(fp.st[ps], smem, b, u, strip, &fn, psig);
      }
      psig = nullptr;
    } else {
      if constexpr (!STAGED) {
        const int fs = strip * P::FO - kHalo;
        if (!pads_zero) zero_pad_symbols<P>(X);   // first item of the workgroup
        if (ps < nst - 1) gz_item_run<P, CHP, TAIL_AGG>(fp.st[ps], X, WB, b, u, fs, &fn, psig);
        else if (GEN && fp_arg.heads_x) {
          if constexpr (GEN) gz_item_run<P, CHP, TAIL_READOUT>(fp.st[ps], X, WB, b, u, fs, &fn, psig);
        } else gz_item_run<P, CHP, TAIL_READOUT_WB>(fp.st[ps], X, WB, b, u, fs, &fn, psig);
      }
      psig = nullptr;
    }
    fstamp(5);
    // item done: one add on the slot's counter once every wave's stores have reached L2 --
    // deferred to the next item (above / its prologue), so that the store drain overlaps that
    // item's first loads
    if (nrx_tid() == 0) sh[1] = fn.jnn;
    __syncthreads();
    have_z = poll && sh[2] != 0;   // the next item's inputs are complete and acquired
    fstamp(6);
    psig = done + s * B + b;
    // a readout item with its heads in the strip image (TAIL_READOUT, H > 1) overwrote the pad
    // symbols: the next item zeroes them again
    pads_zero = !(GEN && kd == 1 && ps == nst - 1 && fp_arg.heads_x);
    j = jn;
    jn = sh[1];
  }
  if (psig) {   // the last item's deferred signal
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (nrx_tid() == 0) __hip_atomic_fetch_add(psig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the last workgroup to leave resets the counters for the next forward
  if (nrx_tid() == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's last counter add has landed
    sh[3] = atomicAdd(&sy->exits, 1) == (int)(gridDim.x * gridDim.y) - 1;
  }
  __syncthreads();
  if (sh[3]) {
    // every item ran (a queue whose XCD never received a workgroup would leave its slots
    // undone: error word 2), then the reset
    for (int i = nrx_tid(); i < nls * B; i += 512)
      if (__hip_atomic_load(done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ips_of(i / B))
        __hip_atomic_fetch_or(&sy->err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (int i = nrx_tid(); i < nls * B; i += 512) done[i] = 0;
    if (nrx_tid() < 8) sy->head[nrx_tid()] = 0;
    if (nrx_tid() == 0) sy->exits = 0;
  }
}


// ======================================================================= launchers

// CUs of the current device for the pairing / strip-tier heuristics, queried once per
// device on first use (a single cached value was wrong for other devices)
constexpr int kMaxDevices = 64;
static int g_cu_count[kMaxDevices];
static int cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  if (g_cu_count[dev] <= 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    g_cu_count[dev] = cus;
  }
  return g_cu_count[dev];
}

template <class P>
struct Launch {
  using A = FwdArgs<typename P::WT, typename P::BT, typename P::S>;
  using MW = ModelW<typename P::WT, typename P::BT>;

  static hipError_t setup() {
    hipError_t e = hipSuccess;
    auto set = [&](const void* f, bool heads_wb = false) {
      hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, strip_lds_bytes<P>(heads_wb));
      if (r != hipSuccess) e = r;
    };
#define NRX_SET_INIT(A2P)                                     \
    set((const void*)k_init<P, A2P, TAIL_NONE>);              \
    set((const void*)k_init<P, A2P, TAIL_AGG>);
    NRX_SET_INIT(8) NRX_SET_INIT(16) NRX_SET_INIT(32)
#undef NRX_SET_INIT
    set((const void*)k_update<P, 16, TAIL_AGG>);
    set((const void*)k_update<P, 16, TAIL_READOUT>);
    set((const void*)k_update<P, 32, TAIL_AGG>);
    set((const void*)k_update<P, 32, TAIL_READOUT>);
    if constexpr (P::WLDS) {
      set((const void*)k_update<P, 16, TAIL_READOUT_WB>, true);
      set((const void*)k_update<P, 32, TAIL_READOUT_WB>, true);
    }
    return e;
  }

  template <int A2P>
  static void launch_init(dim3 grid, int L, hipStream_t st, const BlockParams<P>& bp, bool tail) {
    static_assert(init_cinp<A2P>(P::KC) <= kHID, "StateInit input wider than the strip image");
    if (tail) k_init<P, A2P, TAIL_AGG><<<grid, 512, L, st>>>(bp);
    else k_init<P, A2P, TAIL_NONE><<<grid, 512, L, st>>>(bp);
  }

  static hipError_t run(const A& args0, const MW& W, int num_it, hipStream_t st, Prof* prof) {
    A args = args0;
    const int strips = (args.F + P::FO - 1) / P::FO;
    constexpr int L = strip_lds_bytes<P>();
    const bool ch32 = 2 * args.A > 16;
    auto B_ = [&](int k) { if (prof) prof->begin(k, st); };
    auto E_ = [&](int k) { if (prof) prof->end(k, st); };
    BlockParams<P> bp;
    bp.a = args;
    bp.inline_combine = args.U <= kInlineUsers;
    bp.pair = 0;
    bp.gz = 0;
    if constexpr (std::is_same<P, P16>::value)   // 24-row strips, U <= 2, the workspace within GZ's offsets
      bp.gz = NRX_UPDATE_GZ != 0 && args.U <= 2 && args.ws_bytes < kGzOob && args.pe16 != nullptr;
    bp.strips = strips;
    const int nq = args.F * kT * 2 * args.A / 4;
    bp.norm_pre = nq > kNormFusedMaxQ;
    if (bp.norm_pre) {
      B_(K_NORM);
      k_norm<<<args.B, 1024, 0, st>>>(args.y, nq, args.norm);
      E_(K_NORM);
    }
    int launch_no = 0;
    // U > kInlineUsers: the leave-one-out combine runs as its own launch on the sp rows
    auto combine = [&](typename P::S* sp) {
      if (bp.inline_combine) return;
      dim3 g((args.F * kT * (kDS / P::EPC) + 255) / 256, args.B);
      k_combine<P><<<g, 256, 0, st>>>(sp, args.active, args.U, args.F);
    };
    for (int h = 0; h < args.H; ++h) {
      bp.llr[h][0] = W.llr[h][0];
      bp.llr[h][1] = W.llr[h][1];
    }
    bp.chest[0] = W.chest[0];
    bp.chest[1] = W.chest[1];
    // StateInit -> s_out; tail of the last StateInit launch: aggregation of iteration 0
    const dim3 grid(strips * args.U * args.B);
    B_(K_INIT);
    for (int m = 0; m < args.num_init; ++m) {
      for (int l = 0; l < 3; ++l) bp.w[l] = W.init[m][l];
      bp.m = m;
      bp.tail = m == args.num_init - 1 ? TAIL_AGG : TAIL_NONE;
      bp.agg[0] = W.agg[0][0];
      bp.agg[1] = W.agg[0][1];
      const bool tl = bp.tail == TAIL_AGG;
      bp.order_rev = launch_no++ & 1;
#ifdef NRX_STAMPS
      {
        static const int sel = getenv("NRX_STAMP_LAUNCH") ? atoi(getenv("NRX_STAMP_LAUNCH")) : 0;
        const int on = sel == -1 - m;
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_nrx_stamp_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, st);
        (void)hipStreamSynchronize(st);
      }
#endif
      // antenna block padding A2P (must match nrx_api.cpp init_a2p)
      if (2 * args.A <= 8) launch_init<8>(grid, L, st, bp, tl);
      else if (2 * args.A <= 16) launch_init<16>(grid, L, st, bp, tl);
      else launch_init<32>(grid, L, st, bp, tl);
    }
    E_(K_INIT);
    combine(bp.a.a_out);
    for (int i = 0; i < num_it; ++i) {
      std::swap(bp.a.s_in, bp.a.s_out);
      std::swap(bp.a.a, bp.a.a_out);
      for (int l = 0; l < 3; ++l) bp.w[l] = W.upd[i][l];
      const bool last = i == num_it - 1;
      bp.tail = last ? TAIL_READOUT : TAIL_AGG;
      if (!last) {
        bp.agg[0] = W.agg[i + 1][0];
        bp.agg[1] = W.agg[i + 1][1];
      }
      bp.order_rev = launch_no++ & 1;
      B_(K_UPDATE);
#ifdef NRX_STAMPS
      {
        static const int sel = getenv("NRX_STAMP_LAUNCH") ? atoi(getenv("NRX_STAMP_LAUNCH")) : 0;
        const int on = i == sel;
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_nrx_stamp_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, st);
        (void)hipStreamSynchronize(st);
      }
#endif
      if (last) {
        // paired readout items (heads staged into WB) under the same conditions as the
        // aggregation pairing below, for one LLR head that fits WB
        bool pair_ro = false;
        if constexpr (P::WLDS) {
          const int items = (int)grid.x;
          pair_ro = NRX_PAIR != 0 && NRX_ZDMA != 0 && NRX_PAIR_RO != 0 && args.U <= 2 && bp.inline_combine &&
                    items % 16 == 0 && items >= 2 * cu_count() && args.H == 1 &&
                    heads_fit_wb(args.bits_max, ch32 ? 32 : 16, 2 * args.A);
          if (pair_ro) {
            constexpr int L_wb = strip_lds_bytes<P>(true);
            bp.pair = 1;
            const dim3 g2(items / 2);
            if (ch32) k_update<P, 32, TAIL_READOUT_WB><<<g2, 512, L_wb, st>>>(bp);
            else k_update<P, 16, TAIL_READOUT_WB><<<g2, 512, L_wb, st>>>(bp);
            bp.pair = 0;
          }
        }
        if (!pair_ro) {
          if (ch32) k_update<P, 32, TAIL_READOUT><<<grid, 512, L, st>>>(bp);
          else k_update<P, 16, TAIL_READOUT><<<grid, 512, L, st>>>(bp);
        }
      } else {
        // two items per workgroup when there are at least two per CU (CU count of the
        // device, one workgroup per CU by LDS) and the halves keep the XCD grouping of
        // work_item (items % 16 == 0)
        const int items = (int)grid.x;
        bp.pair = P::WLDS && NRX_PAIR != 0 && NRX_ZDMA != 0 && args.U <= 2 && bp.inline_combine &&
                  items % 16 == 0 && items >= 2 * cu_count();
        const dim3 g2(bp.pair ? items / 2 : items);
        if (ch32) k_update<P, 32, TAIL_AGG><<<g2, 512, L, st>>>(bp);
        else k_update<P, 16, TAIL_AGG><<<g2, 512, L, st>>>(bp);
        bp.pair = 0;
      }
      E_(K_UPDATE);
      if (!last) combine(bp.a.a_out);
    }
    return hipGetLastError();
  }
};

#ifndef NRX_SMALL_STRIPS
#define NRX_SMALL_STRIPS 1
#endif
// Small grids: the forward is latency-bound and a workgroup's time scales with its rows, so
// the narrowest strips whose items all get a CU of their own are taken (24-row strips
// otherwise).  The readout heads must fit the strip image (X layout: H LLR heads + ChEst,
// 25 KB each).
template <class P>
static bool small_strips_fit(const FwdArgs<_Float16, float, _Float16>& a) {
  const long items = (long)a.B * a.U * ((a.F + P::FO - 1) / P::FO);
  return items <= cu_count() && (a.H + 1) * (kHeadSlot + 1024) <= strip_slots<P>() * slot_pitch<P>();
}
// XCDs (XCCs) of the current device, queried once per device: k_forward keeps one work
// queue per XCD and needs every XCD to hold the same number of CUs (32 per XCD
// was assumed)
static int g_xcc_count[kMaxDevices];
static int xcc_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 0;
  if (g_xcc_count[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || n <= 0) n = -1;
    g_xcc_count[dev] = n;
  }
  return g_xcc_count[dev];
}

// k_forward covers: U <= 8 (U <= 2 with a workspace under 1 GB: conv1 reads z from memory, GZ;
// otherwise the z image is staged in LDS, U = 3, 4 with the inline leave-one-out combine),
// 1..M StateInit stages (Var-IO), up to three LLR heads,
// 2A <= 32, num_init + num_it <= kFusedMaxStages; 24-row strips with at least two items per
// CU (the small-grid tiers keep the three launches: through k_forward they were slower for
// batch-1 latency, profiles/r03/ab_fused_small_latency.txt); a device whose XCDs hold equal CU
// counts (1..8 XCDs, the queue is picked by the hardware XCC id).  U = 5..8: a combine stage
// (k_combine's f32 pass, one item per (slot, strip)) before each update, whose z image then
// takes the combined a_u plane.
// one LLR head whose readout fits the paired-readout WB layout (TAIL_READOUT_WB)
template <class P>
static bool heads_in_wb(const FwdArgs<_Float16, float, _Float16>& a) {
  const int chp = 2 * a.A <= 16 ? 16 : 32;
  return a.H == 1 && heads_fit_wb(a.bits_max, chp, 2 * a.A) &&
         strip_slots<P>() * slot_pitch<P>() + kHW2 + 256 * (a.bits_max + chp) <= fused_lds<P>();
}

template <class P>
static bool fused_gz(const FwdArgs<_Float16, float, _Float16>& a) {
  return a.U <= 2 && a.ws_bytes < kGzOob && a.pe16;
}
template <class P>
static int fused_mode(const FwdArgs<_Float16, float, _Float16>& a) {
  return !fused_gz<P>(a) ? 2 : (a.num_init > 1 || !heads_in_wb<P>(a) ? 1 : 0);
}

template <class P>
static bool fused_applicable(const FwdArgs<_Float16, float, _Float16>& a, int num_it, const FusedCtl& fc) {
  if (!fc.sync || !fc.enabled) return false;
  const int cus = cu_count(), nx = xcc_count();
  if (nx < 1 || nx > 8 || cus % nx != 0) return false;
  const long items = (long)a.B * a.U * ((a.F + P::FO - 1) / P::FO);
  // readout heads: one LLR head in WB (TAIL_READOUT_WB), or up to three + ChEst in the strip
  // image (TAIL_READOUT, X layout)
  const bool heads = heads_in_wb<P>(a) || (a.H <= 3 && (a.H + 1) * (kHeadSlot + 1024) <= strip_slots<P>() * slot_pitch<P>());
  const int nls = a.num_init + num_it * (a.U > kInlineUsers ? 2 : 1);
  // the default (enabled == 1) takes the GZ schedules (MODE 0, 1) with at least four stages
  // (cfg4, cfg4'): the staged-z kernel (cfg3, cfg5) and the three-stage bench forward (cfg2)
  // measured slower than the three launches on most boxes (DESIGN.md section 12,
  // profiles/r04/ab_cfg2_fused_vs_three.txt)
  if (fc.enabled == 1 && (fused_mode<P>(a) == 2 || a.num_init + num_it < 4)) return false;
  return items >= 2L * cus && a.U <= kFusedMaxUsers && a.num_init + num_it <= kFusedMaxStages &&
         nls <= kFusedMaxLS && 2 * a.A <= 32 && a.B <= kFusedMaxB && a.bits_max <= 16 && heads;
}

template <class P>
static hipError_t run_fused(const FwdArgs<_Float16, float, _Float16>& args, const ModelW<_Float16, float>& W,
                            int num_it, hipStream_t st, Prof* prof, const FusedCtl& fc) {
  FusedParams<P> fp{};
  fp.sync = reinterpret_cast<FusedSync*>(fc.sync);
  fp.ninit = args.num_init;
  fp.nst = args.num_init + num_it;
  fp.heads_x = !heads_in_wb<P>(args);
  fp.gz = fused_gz<P>(args);
  const bool comb = args.U > kInlineUsers;
  fp.nls = 0;
  for (int s = 0; s < fp.ninit; ++s) {
    fp.kind[fp.nls] = 0;
    fp.pidx[fp.nls++] = s;
  }
  for (int i = 0; i < num_it; ++i) {
    if (comb) {
      fp.kind[fp.nls] = 2;
      fp.pidx[fp.nls++] = fp.ninit + i;
    }
    fp.kind[fp.nls] = 1;
    fp.pidx[fp.nls++] = fp.ninit + i;
  }
  const int cus = cu_count();
  fp.nq = xcc_count();
  fp.spin_limit = fc.spin_limit;
  fp.dbg_err = fc.dbg_err;
  const int nq = args.F * kT * 2 * args.A / 4;
  const bool norm_pre = nq > kNormFusedMaxQ;
  auto B_ = [&](int k) { if (prof) prof->begin(k, st); };
  auto E_ = [&](int k) { if (prof) prof->end(k, st); };
  if (norm_pre) {
    B_(K_NORM);
    k_norm<<<args.B, 1024, 0, st>>>(args.y, nq, args.norm);
    E_(K_NORM);
  }
  FwdArgs<_Float16, float, _Float16> a = args;
  for (int s = 0; s < fp.nst; ++s) {
    BlockParams<P>& bp = fp.st[s];
    bp.inline_combine = comb ? 0 : 1;   // U > 4: the combine stages write a_u in place
    bp.pair = 0;
    bp.order_rev = 0;
    bp.norm_pre = norm_pre;
    bp.strips = (args.F + P::FO - 1) / P::FO;
    bp.m = 0;
    for (int h = 0; h < args.H; ++h) {
      bp.llr[h][0] = W.llr[h][0];
      bp.llr[h][1] = W.llr[h][1];
    }
    bp.chest[0] = W.chest[0];
    bp.chest[1] = W.chest[1];
    if (s < fp.ninit) {
      // StateInit m = s into s_out (m > 0 accumulating); the last one runs iteration 0's
      // aggregation MLP
      for (int l = 0; l < 3; ++l) bp.w[l] = W.init[s][l];
      bp.m = s;
      bp.tail = s == fp.ninit - 1 ? TAIL_AGG : TAIL_NONE;
      bp.agg[0] = W.agg[0][0];
      bp.agg[1] = W.agg[0][1];
    } else {
      std::swap(a.s_in, a.s_out);
      std::swap(a.a, a.a_out);
      const int i = s - fp.ninit;
      for (int l = 0; l < 3; ++l) bp.w[l] = W.upd[i][l];
      const bool last = i == num_it - 1;
      bp.tail = last ? (fp.heads_x ? TAIL_READOUT : TAIL_READOUT_WB) : TAIL_AGG;
      if (!last) {
        bp.agg[0] = W.agg[i + 1][0];
        bp.agg[1] = W.agg[i + 1][1];
      }
    }
    bp.a = a;
  }
  constexpr int L = fused_lds<P>();
#ifdef NRX_STAMPS
  {
    const int on = getenv("NRX_STAMP_FUSED") ? 100 : 0;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_nrx_stamp_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
  }
#endif
  B_(K_FUSED);
  const int mode = fused_mode<P>(args);
  if (2 * args.A > 16) {
    if (mode == 2) k_forward<P, 32, 32, 2><<<cus, 512, L, st>>>(fp);
    else k_forward<P, 32, 32, 1><<<cus, 512, L, st>>>(fp);
  } else if (2 * args.A <= 8) {
    if (mode == 2) k_forward<P, 8, 16, 2><<<cus, 512, L, st>>>(fp);
    else if (mode == 1) k_forward<P, 8, 16, 1><<<cus, 512, L, st>>>(fp);
    else k_forward<P, 8, 16, 0><<<cus, 512, L, st>>>(fp);
  } else {
    if (mode == 2) k_forward<P, 16, 16, 2><<<cus, 512, L, st>>>(fp);
    else if (mode == 1) k_forward<P, 16, 16, 1><<<cus, 512, L, st>>>(fp);
    else k_forward<P, 16, 16, 0><<<cus, 512, L, st>>>(fp);
  }
  E_(K_FUSED);
  return hipGetLastError();
}

hipError_t launch_forward_f16(const FwdArgs<_Float16, float, _Float16>& args,
                              const ModelW<_Float16, float>& W, int num_it, hipStream_t st,
                              Prof* prof, const FusedCtl& fc) {
  if (NRX_SMALL_STRIPS != 0) {
    if (small_strips_fit<P16S>(args)) return Launch<P16S>::run(args, W, num_it, st, prof);
    if (small_strips_fit<P16M>(args)) return Launch<P16M>::run(args, W, num_it, st, prof);
  }
  if (fused_applicable<P16>(args, num_it, fc)) return run_fused<P16>(args, W, num_it, st, prof, fc);
  return Launch<P16>::run(args, W, num_it, st, prof);
}

bool fused_would_run(const FwdArgs<_Float16, float, _Float16>& args, int num_it, const FusedCtl& fc) {
  if (NRX_SMALL_STRIPS != 0 && (small_strips_fit<P16S>(args) || small_strips_fit<P16M>(args))) return false;
  return fused_applicable<P16>(args, num_it, fc);
}

size_t fused_sync_bytes() { return kFusedSyncBytes; }

// {error word, items that waited, polls} of the fused forward since the last reset.  Blocking:
// the stream the forwards ran on is synchronised first, so the read and the reset never race
// with a k_forward in flight; reset clears the three words.
hipError_t fused_sync_status(void* sync, int* st, bool reset, hipStream_t stream) {
  FusedSync* sy = reinterpret_cast<FusedSync*>(sync);
  hipError_t e = hipStreamSynchronize(stream);
  if (e != hipSuccess) e = hipDeviceSynchronize();   // that stream is gone: wait for everything
  if (e == hipSuccess) e = hipMemcpy(st, &sy->err, 3 * sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) e = hipMemset(&sy->err, 0, 3 * sizeof(int));
  if (e == hipSuccess && reset) e = hipDeviceSynchronize();
  return e;
}

hipError_t launch_forward_f64(const FwdArgs<double, double, float>& args,
                              const ModelW<double, double>& W, int num_it, hipStream_t st,
                              Prof* prof) {
  return Launch<P64>::run(args, W, num_it, st, prof);
}

hipError_t setup_kernels() {
  (void)cu_count();
  (void)xcc_count();
  hipError_t e = Launch<P16>::setup();
  hipError_t e1 = Launch<P16S>::setup();
  if (e1 == hipSuccess) e1 = Launch<P16M>::setup();
  hipError_t e2 = Launch<P64>::setup();
  auto set_fused = [&](const void* f, int lds) {
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (r != hipSuccess && e2 == hipSuccess) e2 = r;
  };
  set_fused((const void*)k_forward<P16, 8, 16, 0>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 16, 16, 0>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 8, 16, 1>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 16, 16, 1>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 8, 16, 2>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 16, 16, 2>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 32, 32, 1>, fused_lds<P16>());
  set_fused((const void*)k_forward<P16, 32, 32, 2>, fused_lds<P16>());
  return e != hipSuccess ? e : (e1 != hipSuccess ? e1 : e2);
}

int strip_width(int precision) { return precision == 0 ? P16::FO : P64::FO; }

#ifdef NRX_STAMPS
extern "C" int nrx_debug_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nrx_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
extern "C" int nrx_debug_fused_stamps(void* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nrx_rr_stamps), (size_t)n * 64 * 8, 0, hipMemcpyDeviceToHost);
}
#endif

}  // namespace nrx
