// nrx_kernels.hip -- CDNA4 (gfx950) kernels of the CGNN neural-receiver forward pass.
//
// Reference semantics: CGNN.forward, neural_rx.py:544-595, with
// the TF structure of "neural_rx copy_pytorch.py" (StateInit :82-188, AggregateUserStates
// :191-231, UpdateState :234-287, ReadoutLLRs/ChEst :324-362).
//
// Kernel map (one launch each, per forward):
//   k_norm      per-slot 1/sqrt(mean(y^2))                       (neural_rx.py:551-557)
//   k_init      StateInit: z=[y,pe,h] -> 3 separable convs       (copy_pytorch.py:160-188)
//               fused with the Var-IO mcs mix                    (neural_rx.py:562-569)
//   k_agg       per-RE user aggregation MLP + leave-one-out mean (neural_rx.py:135-207)
//   k_update    z=[a,s,pe] -> 3 separable convs + skip           (copy_pytorch.py:267-287)
//   k_readout   LLR head(s) + ChEst head                          (neural_rx.py:309-404)
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

#include <utility>

#include "nrx_internal.h"

namespace nrx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef int intx4 __attribute__((ext_vector_type(4)));
typedef int intx8 __attribute__((ext_vector_type(8)));

// DPP: lane l receives lane l-1 (row_shr:1) / lane l+1 (row_shl:1) inside its 16-lane
// row; the lane without a source gets 0 (bound_ctrl).
__device__ __forceinline__ int dpp_shr1(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ int dpp_shl1(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true);
}

struct P16 {
  using S = _Float16;
  using WT = _Float16;
  using BT = float;
  using DV = half8;
  using Acc = floatx4;
  using Real = float;
  static constexpr int KC = 32;   // channels per K chunk (one MFMA K)
  static constexpr int CPL = 8;   // channels per lane per chunk
  static constexpr int EPC = 8;   // storage elements per 16-byte LDS chunk
  static constexpr int FO = 12;   // output subcarriers per strip
  __device__ static DV ld_lds(const char* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static DV ld_glb(const S* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static DV ld_w(const WT* p) { return *reinterpret_cast<const half8*>(p); }
  __device__ static Acc zero() { return Acc{0.f, 0.f, 0.f, 0.f}; }
  __device__ static Acc mma(const WT* a, DV b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const half8*>(a), b, c, 0, 0, 0);
  }
  __device__ static int co(int g, int j) { return 4 * g + j; }
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
  static constexpr int FO = 4;
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
  __device__ static int co(int g, int j) { return g + 4 * j; }
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

// ------------------------------------------------ depthwise 3x3 + pointwise on MFMA
// Output row `row` (buffer index in `in`, rows row-1..row+1 must exist), all COUTP
// channels, pre-bias.  acc[n][j] = out[co = 16 n + P::co(g, j)][t].
template <class P, int CINP, int COUTP>
__device__ __forceinline__ void sep_tile(const char* in, int row, int t, int g, int lane,
                                         const SepW<typename P::WT, typename P::BT>& w,
                                         typename P::Acc (&acc)[COUTP / 16]) {
  using DV = typename P::DV;
  constexpr int NQ = CINP * (int)sizeof(typename P::S) / 16;
  constexpr int NKC = CINP / P::KC;
#pragma unroll
  for (int n = 0; n < COUTP / 16; ++n) acc[n] = P::zero();
  const int sw = swz<NQ>(t);
  const char* rm = in + ((row - 1) * kTP + t) * NQ * 16;
  const char* r0 = rm + kTP * NQ * 16;
  const char* rp = r0 + kTP * NQ * 16;
  const typename P::WT* pwrow = w.pw + (lane & 15) * CINP + g * P::CPL;
#pragma unroll 2
  for (int kc = 0; kc < NKC; ++kc) {
    const int off = ((kc * 4 + g) ^ sw) * 16;
    const DV xm = P::ld_lds(rm + off);
    const DV x0 = P::ld_lds(r0 + off);
    const DV xp = P::ld_lds(rp + off);
    const typename P::WT* dw = w.dw + kc * P::KC + g * P::CPL;
    const DV w0 = P::ld_w(dw + 0 * CINP), w1 = P::ld_w(dw + 1 * CINP), w2 = P::ld_w(dw + 2 * CINP);
    const DV w3 = P::ld_w(dw + 3 * CINP), w4 = P::ld_w(dw + 4 * CINP), w5 = P::ld_w(dw + 5 * CINP);
    const DV w6 = P::ld_w(dw + 6 * CINP), w7 = P::ld_w(dw + 7 * CINP), w8 = P::ld_w(dw + 8 * CINP);
    // column sums per symbol offset dt = j - 1 (tap = i*3 + j, i along subcarriers)
    const DV cm = w0 * xm + w3 * x0 + w6 * xp;
    const DV c0 = w1 * xm + w4 * x0 + w7 * xp;
    const DV cp = w2 * xm + w5 * x0 + w8 * xp;
    const DV d = c0 + P::shr(cm) + P::shl(cp);
#pragma unroll
    for (int n = 0; n < COUTP / 16; ++n)
      acc[n] = P::mma(pwrow + n * 16 * CINP + kc * P::KC, d, acc[n]);
  }
}

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

// ======================================================================== k_norm
// ns[b] = 1/sqrt(mean(y[b]^2)) over the whole provided grid (F x T x 2A);
// divide-no-nan: an all-zero slot gets 0.
__global__ __launch_bounds__(256) void k_norm(const float* __restrict__ y, int n_per_slot,
                                              double* __restrict__ ns) {
  __shared__ double red[256];
  const float* p = y + (size_t)blockIdx.x * n_per_slot;
  double acc = 0.0;
  for (int i = threadIdx.x * 4; i < n_per_slot; i += 256 * 4) {
    if (i + 3 < n_per_slot) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(p + i);
      acc += (double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2] + (double)v[3] * v[3];
    } else {
      for (int k = i; k < n_per_slot; ++k) acc += (double)p[k] * p[k];
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double ms = red[0] / (double)n_per_slot;
    ns[blockIdx.x] = ms > 0.0 ? 1.0 / sqrt(ms) : 0.0;
  }
}

// ===================================================== separable-conv strip kernels
template <class P>
struct InitParams {
  FwdArgs<typename P::WT, typename P::BT, typename P::S> a;
  SepW<typename P::WT, typename P::BT> w[kMaxInit][3];
};

template <class P>
struct UpdParams {
  FwdArgs<typename P::WT, typename P::BT, typename P::S> a;
  SepW<typename P::WT, typename P::BT> w[3];
};

template <class P>
constexpr int strip_lds_bytes(int cinp0) {
  // X: FO+6 rows of max(cinp0, 128) channels; Y: FO+4 rows of 128 channels
  return (P::FO + 2 * kHalo) * kTP * (cinp0 > kHID ? cinp0 : kHID) * (int)sizeof(typename P::S) +
         (P::FO + 2 * kHalo - 2) * kTP * kHID * (int)sizeof(typename P::S);
}

// conv1 (X rows [1,R0-1) -> Y rows shifted by 1) and conv2 (Y -> X rows [2,R0-2)).
template <class P, int CINP>
__device__ __forceinline__ void strip_conv12(char* X, char* Y, int f_start, int F,
                                             const SepW<typename P::WT, typename P::BT>* w) {
  constexpr int R0 = P::FO + 2 * kHalo;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  typename P::Acc acc[kHID / 16];
  for (int lf = 1 + wave; lf < R0 - 1; lf += 8) {
    const int f = f_start + lf;
    const bool valid = f >= 0 && f < F;
    if (valid) sep_tile<P, CINP, kHID>(X, lf, t, g, lane, w[0], acc);
    else {
#pragma unroll
      for (int n = 0; n < kHID / 16; ++n) acc[n] = P::zero();
    }
    epi_lds<P, kHID>(Y, lf - 1, t, g, acc, w[0].b, true, !valid);
  }
  __syncthreads();
  for (int lf = 2 + wave; lf < R0 - 2; lf += 8) {
    const int f = f_start + lf;
    const bool valid = f >= 0 && f < F;
    if (valid) sep_tile<P, kHID, kHID>(Y, lf - 1, t, g, lane, w[1], acc);
    else {
#pragma unroll
      for (int n = 0; n < kHID / 16; ++n) acc[n] = P::zero();
    }
    epi_lds<P, kHID>(X, lf, t, g, acc, w[1].b, true, !valid);
  }
  __syncthreads();
}

// StateInit (+ Var-IO mix).  grid = (strips, U, B), block = 512.
template <class P, int CINP>
__global__ __launch_bounds__(512) void k_init(InitParams<P> prm) {
  using S = typename P::S;
  using Real = typename P::Real;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int R0 = P::FO + 2 * kHalo;
  const auto& a = prm.a;
  const int strip = blockIdx.x, u = blockIdx.y, b = blockIdx.z;
  const int F = a.F, U = a.U, A2 = 2 * a.A;
  const int f0 = strip * P::FO;
  const int f_start = f0 - kHalo;
  char* X = smem;
  char* Y = smem + R0 * kTP * (CINP > kHID ? CINP : kHID) * (int)sizeof(S);
  const Real ns = (Real)a.norm[b];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  bool wrote = false;
  for (int m = 0; m < a.num_init; ++m) {
    Real wm = (Real)1;
    if (!a.masking) {
      wm = a.mcs_mask ? (Real)a.mcs_mask[((size_t)b * U + u) * a.M + m] : (Real)(m == 0 ? 1 : 0);
      if (wm == (Real)0) continue;   // exact: contributes 0 * finite
    }
    // z = [y*ns (2A), pe (2), h*ns (2A), 0...] on rows [0,R0) x 16
    for (int idx = threadIdx.x; idx < R0 * kTP * CINP; idx += 512) {
      const int c = idx % CINP;
      const int tt = (idx / CINP) % kTP;
      const int lf = idx / (CINP * kTP);
      const int f = f_start + lf;
      Real v = 0;
      if (f >= 0 && f < F && tt < kT) {
        if (c < A2) v = (Real)a.y[(((size_t)b * F + f) * kT + tt) * A2 + c] * ns;
        else if (c < A2 + 2) v = (Real)a.pe[(((size_t)u * F + f) * kT + tt) * 2 + (c - A2)];
        else if (a.use_h && c < 2 * A2 + 2)
          v = (Real)a.h_hat[((((size_t)b * U + u) * F + f) * kT + tt) * A2 + (c - A2 - 2)] * ns;
      }
      lds_store<P>(X, lds_elem_off<P, CINP>(lf, tt, c), v);
    }
    __syncthreads();
    strip_conv12<P, CINP>(X, Y, f_start, F, prm.w[m]);
    // conv3: X rows [3, R0-3) -> global s (d_s channels, padded to 64)
    typename P::Acc acc[kDSP / 16];
    for (int lf = kHalo + wave; lf < R0 - kHalo; lf += 8) {
      const int f = f_start + lf;
      if (f >= F) continue;
      sep_tile<P, kHID, kDSP>(X, lf, t, g, lane, prm.w[m][2], acc);
      S* dst = a.s_out + ((((size_t)b * U + u) * F + f) * kTP + t) * kDSP;
#pragma unroll
      for (int n = 0; n < kDSP / 16; ++n) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = 16 * n + P::co(g, j);
          Real v = ((Real)acc[n][j] + (Real)prm.w[m][2].b[co]) * wm;
          if (wrote) v += (Real)dst[co];
          if (t >= kT || co >= kDS) v = 0;
          dst[co] = (S)v;
        }
      }
    }
    wrote = true;
    __syncthreads();
  }
  if (!wrote) {
    for (int idx = threadIdx.x; idx < P::FO * kTP * kDSP; idx += 512) {
      const int f = f0 + idx / (kTP * kDSP);
      if (f < F) a.s_out[(((size_t)b * U + u) * F + f0) * kTP * kDSP + idx] = (S)0;
    }
  }
}

// UpdateState: z = [a, s, pe] -> 3 sep convs + skip.  grid = (strips, U, B), block 512.
template <class P>
__global__ __launch_bounds__(512) void k_update(UpdParams<P> prm) {
  using S = typename P::S;
  using Real = typename P::Real;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int R0 = P::FO + 2 * kHalo;
  constexpr int CINP = kUPD_CINP;
  constexpr int NQ = CINP * (int)sizeof(S) / 16;      // chunks per z row
  constexpr int QS = kDS / P::EPC;                     // chunks of a (and of s) in z
  const auto& a = prm.a;
  const int strip = blockIdx.x, u = blockIdx.y, b = blockIdx.z;
  const int F = a.F, U = a.U;
  const int f0 = strip * P::FO;
  const int f_start = f0 - kHalo;
  char* X = smem;
  char* Y = smem + R0 * kTP * kHID * (int)sizeof(S);
  const size_t bu = (size_t)b * U + u;
  // z chunks: [0,QS) <- a, [QS,2QS) <- s, 2QS <- pe (2 values), rest 0
  for (int idx = threadIdx.x; idx < R0 * kTP * NQ; idx += 512) {
    const int q = idx % NQ;
    const int tt = (idx / NQ) % kTP;
    const int lf = idx / (NQ * kTP);
    const int f = f_start + lf;
    floatx4 zero4 = {0.f, 0.f, 0.f, 0.f};
    char* dst = X + lds_off<NQ>(lf, tt, q);
    if (f >= 0 && f < F && tt < kT) {
      const size_t row = ((bu * F + f) * kTP + tt) * kDSP;
      if (q < QS) {
        *reinterpret_cast<floatx4*>(dst) = *reinterpret_cast<const floatx4*>(a.a + row + q * P::EPC);
      } else if (q < 2 * QS) {
        *reinterpret_cast<floatx4*>(dst) = *reinterpret_cast<const floatx4*>(a.s_in + row + (q - QS) * P::EPC);
      } else {
        *reinterpret_cast<floatx4*>(dst) = zero4;
        if (q == 2 * QS) {
          const float* pp = a.pe + (((size_t)u * F + f) * kT + tt) * 2;
          S* d = reinterpret_cast<S*>(dst);
          d[0] = (S)pp[0];
          d[1] = (S)pp[1];
        }
      }
    } else {
      *reinterpret_cast<floatx4*>(dst) = zero4;
    }
  }
  __syncthreads();
  strip_conv12<P, CINP>(X, Y, f_start, F, prm.w);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  typename P::Acc acc[kDSP / 16];
  for (int lf = kHalo + wave; lf < R0 - kHalo; lf += 8) {
    const int f = f_start + lf;
    if (f >= F) continue;
    sep_tile<P, kHID, kDSP>(X, lf, t, g, lane, prm.w[2], acc);
    const size_t row = ((bu * F + f) * kTP + t) * kDSP;
    const S* skip = a.s_in + row;
    S* dst = a.s_out + row;
#pragma unroll
    for (int n = 0; n < kDSP / 16; ++n) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = 16 * n + P::co(g, j);
        Real v = (Real)acc[n][j] + (Real)prm.w[2].b[co] + (Real)skip[co];
        if (t >= kT || co >= kDS) v = 0;
        dst[co] = (S)v;
      }
    }
  }
}

// ========================================================================= k_agg
// Per RE, all users: sp_u = W2 relu(W1 s_u + b1) + b2, masked by active; a_u = (sum -
// sp_u) * p, p = 1/max(#active-1) (1 when <= 1 active).  grid = (ceil(F/4), B), block 256:
// one wave per subcarrier row (16 symbols).
template <class P>
struct AggParams {
  FwdArgs<typename P::WT, typename P::BT, typename P::S> a;
  DenseW<typename P::WT, typename P::BT> w[2];
};

template <class P>
__device__ __forceinline__ void agg_mlp(const typename P::S* srow, char* hid, int t, int g, int lane,
                                        const DenseW<typename P::WT, typename P::BT>* w,
                                        typename P::Acc (&out)[kDSP / 16]) {
  constexpr int NQ_H = kAGG * (int)sizeof(typename P::S) / 16;
  typename P::Acc h[kAGG / 16];
  dense_tile<P, kDSP, kAGG>([&](int q) { return P::ld_glb(srow + q * P::EPC); }, lane, g, w[0], h);
  wave_lds_sync();
  epi_lds<P, kAGG>(hid, 0, t, g, h, w[0].b, true, false);
  wave_lds_sync();
  dense_tile<P, kAGG, kDSP>([&](int q) { return P::ld_lds(hid + lds_off<NQ_H>(0, t, q)); }, lane, g,
                            w[1], out);
}

template <class P>
__global__ __launch_bounds__(256) void k_agg(AggParams<P> prm) {
  using S = typename P::S;
  using Real = typename P::Real;
  __shared__ __attribute__((aligned(16))) char smem[4][kTP * kAGG * sizeof(S)];
  const auto& a = prm.a;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  const int f = blockIdx.x * 4 + wave;
  const int b = blockIdx.y;
  const int F = a.F, U = a.U;
  if (f >= F) return;
  char* hid = smem[wave];
  Real nact = 0;
  for (int u = 0; u < U; ++u) nact += (Real)a.active[(size_t)b * U + u];
  Real p = nact - (Real)1;
  p = p > (Real)0 ? p : (Real)0;
  p = p == (Real)0 ? (Real)1 : (Real)1 / p;
  typename P::Acc sum[kDSP / 16], sp[kDSP / 16];
#pragma unroll
  for (int n = 0; n < kDSP / 16; ++n) sum[n] = P::zero();
  for (int u = 0; u < U; ++u) {
    const Real act = (Real)a.active[(size_t)b * U + u];
    const S* srow = a.s_in + ((((size_t)b * U + u) * F + f) * kTP + t) * kDSP;
    agg_mlp<P>(srow, hid, t, g, lane, prm.w, sp);
#pragma unroll
    for (int n = 0; n < kDSP / 16; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        sum[n][j] += ((Real)sp[n][j] + (Real)prm.w[1].b[16 * n + P::co(g, j)]) * act;
  }
  for (int u = 0; u < U; ++u) {
    const Real act = (Real)a.active[(size_t)b * U + u];
    const size_t row = ((((size_t)b * U + u) * F + f) * kTP + t) * kDSP;
    agg_mlp<P>(a.s_in + row, hid, t, g, lane, prm.w, sp);
    S* dst = a.a + row;
#pragma unroll
    for (int n = 0; n < kDSP / 16; ++n) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = 16 * n + P::co(g, j);
        const Real own = ((Real)sp[n][j] + (Real)prm.w[1].b[co]) * act;
        Real v = ((Real)sum[n][j] - own) * p;
        if (t >= kT || co >= kDS) v = 0;
        dst[co] = (S)v;
      }
    }
  }
}

// ===================================================================== k_readout
// Per (b, u, subcarrier row): LLR head(s) 56->128->bits and ChEst 56->128->2A.
template <class P>
struct ReadParams {
  FwdArgs<typename P::WT, typename P::BT, typename P::S> a;
  DenseW<typename P::WT, typename P::BT> llr[kMaxHeads][2];
  DenseW<typename P::WT, typename P::BT> chest[2];
};

template <class P, int COUTP>
__device__ __forceinline__ void head(const typename P::S* srow, char* hid, int t, int g, int lane,
                                     const DenseW<typename P::WT, typename P::BT>* w,
                                     typename P::Acc (&out)[COUTP / 16]) {
  constexpr int NQ_H = kHID * (int)sizeof(typename P::S) / 16;
  typename P::Acc h[kHID / 16];
  dense_tile<P, kDSP, kHID>([&](int q) { return P::ld_glb(srow + q * P::EPC); }, lane, g, w[0], h);
  wave_lds_sync();
  epi_lds<P, kHID>(hid, 0, t, g, h, w[0].b, true, false);
  wave_lds_sync();
  dense_tile<P, kHID, COUTP>([&](int q) { return P::ld_lds(hid + lds_off<NQ_H>(0, t, q)); }, lane, g,
                             w[1], out);
}

template <class P, int CHP>
__global__ __launch_bounds__(256) void k_readout(ReadParams<P> prm) {
  using S = typename P::S;
  using Real = typename P::Real;
  __shared__ __attribute__((aligned(16))) char smem[4][kTP * kHID * sizeof(S)];
  const auto& a = prm.a;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 15, g = lane >> 4;
  const int f = blockIdx.x * 4 + wave;
  const int u = blockIdx.y, b = blockIdx.z;
  const int F = a.F, U = a.U, B = a.B;
  if (f >= F) return;
  char* hid = smem[wave];
  const size_t bu = (size_t)b * U + u;
  const S* srow = a.s_in + ((bu * F + f) * kTP + t) * kDSP;
  for (int hh = 0; hh < a.H; ++hh) {
    typename P::Acc o[1];
    head<P, 16>(srow, hid, t, g, lane, prm.llr[hh], o);
    if (t < kT) {
      float* dst = a.llr + ((((size_t)hh * B + b) * U + u) * F + f) * kT * a.bits_max + t * a.bits_max;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = P::co(g, j);
        if (co < a.bits_max)
          dst[co] = co < a.head_bits[hh] ? (float)((Real)o[0][j] + (Real)prm.llr[hh][1].b[co]) : 0.f;
      }
    }
    wave_lds_sync();
  }
  if (a.h_ref) {
    typename P::Acc o[CHP / 16];
    head<P, CHP>(srow, hid, t, g, lane, prm.chest, o);
    if (t < kT) {
      const int A2 = 2 * a.A;
      float* dst = a.h_ref + ((bu * F + f) * kT + t) * A2;
#pragma unroll
      for (int n = 0; n < CHP / 16; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = 16 * n + P::co(g, j);
          if (co < A2) dst[co] = (float)((Real)o[n][j] + (Real)prm.chest[1].b[co]);
        }
    }
  }
}

// ======================================================================= launchers
template <class P>
struct Launch {
  using A = FwdArgs<typename P::WT, typename P::BT, typename P::S>;
  using MW = ModelW<typename P::WT, typename P::BT>;

  static hipError_t setup() {
    hipError_t e = hipSuccess;
    auto set = [&](const void* f, int bytes) {
      hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
      if (r != hipSuccess) e = r;
    };
    set((const void*)k_init<P, 32>, strip_lds_bytes<P>(32));
    set((const void*)k_init<P, 64>, strip_lds_bytes<P>(64));
    set((const void*)k_init<P, 128>, strip_lds_bytes<P>(128));
    set((const void*)k_update<P>, strip_lds_bytes<P>(kUPD_CINP));
    return e;
  }

  static hipError_t run(const A& args0, const MW& W, int num_it, hipStream_t st, Prof* prof) {
    A args = args0;
    const int strips = (args.F + P::FO - 1) / P::FO;
    auto B_ = [&](int k) { if (prof) prof->begin(k, st); };
    auto E_ = [&](int k) { if (prof) prof->end(k, st); };
    B_(K_NORM);
    k_norm<<<args.B, 256, 0, st>>>(args.y, args.F * kT * 2 * args.A, args.norm);
    E_(K_NORM);
    B_(K_INIT);
    {
      InitParams<P> ip;
      ip.a = args;
      for (int m = 0; m < args.num_init; ++m)
        for (int l = 0; l < 3; ++l) ip.w[m][l] = W.init[m][l];
      dim3 grid(strips, args.U, args.B);
      if (args.init_cinp <= 32) {
        constexpr int L = strip_lds_bytes<P>(32);
        k_init<P, 32><<<grid, 512, L, st>>>(ip);
      } else if (args.init_cinp <= 64) {
        constexpr int L = strip_lds_bytes<P>(64);
        k_init<P, 64><<<grid, 512, L, st>>>(ip);
      } else {
        constexpr int L = strip_lds_bytes<P>(128);
        k_init<P, 128><<<grid, 512, L, st>>>(ip);
      }
    }
    E_(K_INIT);
    constexpr int LU = strip_lds_bytes<P>(kUPD_CINP);
    for (int i = 0; i < num_it; ++i) {
      // s_out of the previous stage is this iteration's input
      std::swap(args.s_in, args.s_out);
      AggParams<P> ap;
      ap.a = args;
      ap.w[0] = W.agg[i][0];
      ap.w[1] = W.agg[i][1];
      B_(K_AGG);
      k_agg<P><<<dim3((args.F + 3) / 4, args.B), 256, 0, st>>>(ap);
      E_(K_AGG);
      UpdParams<P> up;
      up.a = args;
      for (int l = 0; l < 3; ++l) up.w[l] = W.upd[i][l];
      B_(K_UPDATE);
      k_update<P><<<dim3(strips, args.U, args.B), 512, LU, st>>>(up);
      E_(K_UPDATE);
    }
    std::swap(args.s_in, args.s_out);
    ReadParams<P> rp;
    rp.a = args;
    for (int h = 0; h < args.H; ++h) {
      rp.llr[h][0] = W.llr[h][0];
      rp.llr[h][1] = W.llr[h][1];
    }
    rp.chest[0] = W.chest[0];
    rp.chest[1] = W.chest[1];
    dim3 grid((args.F + 3) / 4, args.U, args.B);
    B_(K_READOUT);
    if (2 * args.A <= 16) k_readout<P, 16><<<grid, 256, 0, st>>>(rp);
    else k_readout<P, 32><<<grid, 256, 0, st>>>(rp);
    E_(K_READOUT);
    return hipGetLastError();
  }
};

hipError_t launch_forward_f16(const FwdArgs<_Float16, float, _Float16>& args,
                              const ModelW<_Float16, float>& W, int num_it, hipStream_t st,
                              Prof* prof) {
  return Launch<P16>::run(args, W, num_it, st, prof);
}

hipError_t launch_forward_f64(const FwdArgs<double, double, float>& args,
                              const ModelW<double, double>& W, int num_it, hipStream_t st,
                              Prof* prof) {
  return Launch<P64>::run(args, W, num_it, st, prof);
}

hipError_t setup_kernels() {
  hipError_t e = Launch<P16>::setup();
  hipError_t e2 = Launch<P64>::setup();
  return e != hipSuccess ? e : e2;
}

int strip_width(int precision) { return precision == 0 ? P16::FO : P64::FO; }

}  // namespace nrx
