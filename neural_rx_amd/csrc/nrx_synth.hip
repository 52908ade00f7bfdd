// nrx_synth.hip -- seeded PUSCH slot generator and uncoded error counters on the GPU
// (SURVEY.md 8(f) f3): the stand-in for the reference's transmitter + channel + LS chain
// (E2E_Model.forward, utils/e2e_model.py:219-344) and sim_ber's error counting
// (scripts/evaluate.py:193-202), so that an evaluation loop never leaves the device.
// The algorithm is stated once, in oracle/synth_ref.py; these kernels compute the same
// function (f64 arithmetic, one f32 rounding at the end).
//
//   k_gen_params   per slot: active ports (Fisher-Yates, e2e_model.py:187-193), MCS per
//                  user, TDL delays (sorted, first = 0) and the exponential PDP
//   k_gen_taps     per (slot, user, antenna, tap, symbol): sum-of-sinusoids tap gain g(t)
//   k_gen_tx       per (slot, user, RE): Philox bits, Gray QAM / DMRS QPSK x sqrt(2), x *= active
//   k_gen_rx       per (slot, subcarrier): the user/tap phasors of that subcarrier in LDS,
//                  then y[a][t] = sum_u H_u x_u + AWGN (and the true channel, optional)
//   k_gen_ls       per (slot, user, RE, antenna): LS at the nearest own pilot (closed form
//                  of the Manhattan argmin), and the Aerial pilot list (optional)
//   k_count_errors per (slot group, user): hard decisions of the LLR head vs the sent bits on
//                  the data REs, block reductions, 4 int64 atomics per workgroup
//
// Random draws: Philox4x32-10 with key = seed and counter = (element, slot lo, slot hi,
// stream), slot = slot_offset + b -- a pure function of the global slot index, so any split
// of slots over launches or ranks generates the same slots.  All HBM-bound or
// latency-trivial next to the CGNN (a few bytes per RE); one pass each, coalesced along the
// fastest output axis.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nrx.h"
#include "nrx_internal.h"

namespace nrx {

struct GenWs {
  double2* x;        // [B][U][F][T]
  double2* gt;       // [B][U][A][L][T]
  double* tau;       // [B][U][L]
  double* spdp;      // [B][U][L]
  uint8_t* mcs;      // [B][U]
  float* active;     // [B][U]
};

namespace {

enum { ST_RE = 0, ST_ACTIVE = 1, ST_MCS = 2, ST_DELAY = 3, ST_TAP = 4, ST_NOISE = 5 };

constexpr double kPi = 3.14159265358979323846;
constexpr double kCP = 1.07;      // symbol time = 1.07 / scs (normal cyclic prefix)
constexpr double kPDP = 3.0;      // PDP decay constant = max_delay / 3

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                     uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ U4 draw(const nrx_gen_desc& d, int64_t b, int stream, uint32_t idx) {
  const uint64_t g = (uint64_t)(d.slot_offset + b);
  return philox(idx, (uint32_t)g, (uint32_t)(g >> 32), (uint32_t)stream, (uint32_t)d.seed,
                (uint32_t)(d.seed >> 32));
}

__device__ __forceinline__ double uni(uint32_t w) { return ((double)w + 0.5) * 0x1p-32; }

__device__ __forceinline__ double2 box_muller(uint32_t w0, uint32_t w1) {
  const double r = sqrt(-2.0 * log(uni(w0)));
  const double th = 2.0 * kPi * uni(w1);
  return make_double2(r * cos(th), r * sin(th));
}

// Gray QAM of TS 38.211 5.1 (unit energy): bit k of `w`, k < m
__device__ __forceinline__ double2 qam(uint32_t w, int m) {
  auto s = [&](int k) { return 1.0 - 2.0 * (double)((w >> k) & 1u); };
  if (m == 2) return make_double2(s(0) / sqrt(2.0), s(1) / sqrt(2.0));
  if (m == 4) return make_double2(s(0) * (2.0 - s(2)) / sqrt(10.0), s(1) * (2.0 - s(3)) / sqrt(10.0));
  return make_double2(s(0) * (4.0 - s(2) * (2.0 - s(4))) / sqrt(42.0),
                      s(1) * (4.0 - s(3) * (2.0 - s(5))) / sqrt(42.0));
}

__global__ __launch_bounds__(64) void k_gen_params(nrx_gen_desc d, GenWs w, float* __restrict__ active_out,
                                                    float* __restrict__ mcs_mask, uint8_t* __restrict__ mcs_out) {
  const int b = blockIdx.x;
  const int U = d.num_tx, L = d.num_taps, M = d.num_mcs;
  const int i = threadIdx.x;
  if (i == 0) {
    uint32_t wd[16];
    for (int q = 0; q < 4; ++q) {
      const U4 r = draw(d, b, ST_ACTIVE, q);
      wd[4 * q] = r.x;
      wd[4 * q + 1] = r.y;
      wd[4 * q + 2] = r.z;
      wd[4 * q + 3] = r.w;
    }
    int arr[kMaxUsers];
    for (int u = 0; u < U; ++u) arr[u] = u < d.num_active ? 1 : 0;
    for (int k = U - 1; k > 0; --k) {
      const int j = (int)(wd[k] % (uint32_t)(k + 1));
      const int t = arr[k];
      arr[k] = arr[j];
      arr[j] = t;
    }
    for (int u = 0; u < U; ++u) {
      w.active[b * U + u] = (float)arr[u];
      if (active_out) active_out[b * U + u] = (float)arr[u];
    }
  }
  if (i < U) {
    const int u = i;
    int m = d.mcs_of_user[u];
    if (m < 0) m = (int)(draw(d, b, ST_MCS, u).x % (uint32_t)M);
    w.mcs[b * U + u] = (uint8_t)m;
    if (mcs_out) mcs_out[b * U + u] = (uint8_t)m;
    if (mcs_mask)
      for (int k = 0; k < M; ++k) mcs_mask[((size_t)b * U + u) * M + k] = k == m ? 1.0f : 0.0f;
  }
  // delays: one thread per (u, l) (U * L <= 128 = 2 passes of 64); ascending order by rank
  // (ties by index, as a stable sort), the smallest set to 0; PDP normalised per user
  __shared__ double tau[kMaxUsers * 8];
  __shared__ double pw[kMaxUsers * 8];
  for (int j = i; j < U * L; j += 64) tau[j] = uni(draw(d, b, ST_DELAY, j).x) * d.max_delay_s;
  __syncthreads();
  double tr[2], pr[2];
  int rk[2];
  for (int q = 0; q < 2; ++q) {
    const int j = i + 64 * q;
    if (j >= U * L) break;
    const int u = j / L, l = j % L;
    int r = 0;
    for (int k = 0; k < L; ++k) {
      const double o = tau[u * L + k];
      r += (o < tau[j]) || (o == tau[j] && k < l);
    }
    rk[q] = r;
    tr[q] = r == 0 ? 0.0 : tau[j];
    pr[q] = exp(-tr[q] / (d.max_delay_s / kPDP + 1e-12));
  }
  __syncthreads();
  for (int q = 0; q < 2; ++q) {
    const int j = i + 64 * q;
    if (j >= U * L) break;
    const int u = j / L;
    tau[u * L + rk[q]] = tr[q];
    pw[u * L + rk[q]] = pr[q];
  }
  __syncthreads();
  for (int q = 0; q < 2; ++q) {
    const int j = i + 64 * q;
    if (j >= U * L) break;
    const int u = j / L;
    double ps = 0.0;
    for (int k = 0; k < L; ++k) ps += pw[u * L + k];
    w.tau[(size_t)b * U * L + j] = tau[j];
    w.spdp[(size_t)b * U * L + j] = sqrt(pw[j] / ps);
  }
}

// g(t) = sqrt(pdp_l) sum_s g0_s exp(j 2 pi fd_s t Tsym).  A block owns kTapGroups
// (b, u, a, l) groups: the NS sinusoid draws of each group (Philox + Box-Muller + Doppler
// cosine, the f64 transcendentals) are made once into LDS, then one thread per (group, t)
// sums the NS rotations -- the same operations per value as drawing them per thread (the
// taps are unchanged bit for bit) at 1/T of the draw work.
constexpr int kTapGroups = 16;
constexpr int kMaxSinusoids = 16;   // nrx_generate_slots validates num_sinusoids <= 16

__global__ __launch_bounds__(kTapGroups * kT) void k_gen_taps(nrx_gen_desc d, GenWs w) {
  __shared__ double sg[kTapGroups * kMaxSinusoids][3];
  const int U = d.num_tx, A = d.num_rx_ant, L = d.num_taps, NS = d.num_sinusoids;
  const int64_t ngrp = (int64_t)d.batch * U * A * L;
  const int64_t g0 = (int64_t)blockIdx.x * kTapGroups;
  const double tsym = kCP / d.subcarrier_spacing;
  const double sc = 1.0 / sqrt(2.0 * NS);
  for (int j = threadIdx.x; j < kTapGroups * NS; j += kTapGroups * kT) {
    const int64_t g = g0 + j / NS;
    const int s = j % NS;
    if (g >= ngrp) continue;
    const int l = (int)(g % L);
    const int a = (int)((g / L) % A);
    const int u = (int)((g / ((int64_t)L * A)) % U);
    const int64_t b = g / ((int64_t)L * A * U);
    const U4 r = draw(d, b, ST_TAP, (uint32_t)((((u * A + a) * L + l) * NS) + s));
    const double2 z = box_muller(r.x, r.y);
    sg[j][0] = z.x * sc;
    sg[j][1] = z.y * sc;
    sg[j][2] = d.max_doppler_hz * cos(2.0 * kPi * uni(r.z));
  }
  __syncthreads();
  const int gl = threadIdx.x / kT, t = threadIdx.x % kT;
  const int64_t g = g0 + gl;
  if (g >= ngrp) return;
  double ar = 0.0, ai = 0.0;
  for (int s = 0; s < NS; ++s) {
    const double g0r = sg[gl * NS + s][0], g0i = sg[gl * NS + s][1], fd = sg[gl * NS + s][2];
    const double ph = 2.0 * kPi * (fd * (t * tsym));
    const double c = cos(ph), sn = sin(ph);
    ar += g0r * c - g0i * sn;
    ai += g0r * sn + g0i * c;
  }
  const int l = (int)(g % L);
  const int64_t bu = g / ((int64_t)L * A);
  const double sp = w.spdp[bu * L + l];
  w.gt[g * kT + t] = make_double2(ar * sp, ai * sp);
}

// one thread per (b, u, f, t)
__global__ __launch_bounds__(256) void k_gen_tx(nrx_gen_desc d, GenWs w, uint8_t* __restrict__ bits,
                                                int bits_stride) {
  const int U = d.num_tx, F = d.num_subcarriers, T = d.num_symbols;
  const int64_t n = (int64_t)d.batch * U * F * T;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int t = (int)(i % T);
  const int f = (int)((i / T) % F);
  const int u = (int)((i / ((int64_t)T * F)) % U);
  const int64_t b = i / ((int64_t)T * F * U);
  const U4 r = draw(d, b, ST_RE, (uint32_t)((u * F + f) * T + t));
  const bool dmrs = (d.dmrs_symbol_mask >> t) & 1;
  const int m = d.mcs_bits[w.mcs[b * U + u]];
  double2 x;
  if (dmrs) {
    const double2 q = qam(r.y, 2);
    x = (f & 1) == d.cdm_group[u] ? make_double2(q.x * sqrt(2.0), q.y * sqrt(2.0)) : make_double2(0.0, 0.0);
  } else {
    x = qam(r.x, m);
  }
  const double act = w.active[b * U + u];
  w.x[i] = make_double2(x.x * act, x.y * act);
  if (bits) {
    uint8_t* dst = bits + i * bits_stride;
    for (int k = 0; k < bits_stride; ++k) dst[k] = (!dmrs && k < m) ? (uint8_t)((r.x >> k) & 1u) : (uint8_t)0;
  }
}

// block = FB subcarriers x (A * T) threads; grid = (ceil(F / FB), B)
__global__ __launch_bounds__(256) void k_gen_rx(nrx_gen_desc d, GenWs w, int FB, float* __restrict__ y,
                                                float* __restrict__ h, float* __restrict__ y_re,
                                                float* __restrict__ y_im) {
  __shared__ double2 e[4][kMaxUsers * 8];   // phasor of (u, l) at the block's subcarriers
  const int U = d.num_tx, A = d.num_rx_ant, L = d.num_taps, F = d.num_subcarriers, T = d.num_symbols;
  const int b = blockIdx.y;
  const int fl = threadIdx.x / (A * T);
  const int f = blockIdx.x * FB + fl;
  for (int j = threadIdx.x; j < FB * U * L; j += blockDim.x) {
    const int ff = blockIdx.x * FB + j / (U * L);
    const int ul = j % (U * L);
    if (ff < F) {
      const double fa = 2.0 * kPi * (((double)ff * d.subcarrier_spacing) * w.tau[(size_t)b * U * L + ul]);
      e[j / (U * L)][ul] = make_double2(cos(fa), -sin(fa));
    }
  }
  __syncthreads();
  if (fl >= FB || f >= F) return;
  const int at = threadIdx.x % (A * T);
  const int a = at / T, t = at % T;
  double yr = 0.0, yi = 0.0;
  for (int u = 0; u < U; ++u) {
    const double2* g = w.gt + ((((size_t)b * U + u) * A + a) * L) * T + t;
    double hr = 0.0, hi = 0.0;
    for (int l = 0; l < L; ++l) {
      const double2 gl = g[(size_t)l * T], el = e[fl][u * L + l];
      hr += gl.x * el.x - gl.y * el.y;
      hi += gl.x * el.y + gl.y * el.x;
    }
    const double2 x = w.x[(((size_t)b * U + u) * F + f) * T + t];
    yr += hr * x.x - hi * x.y;
    yi += hr * x.y + hi * x.x;
    if (h) {
      float* dst = h + ((((size_t)b * U + u) * F + f) * T + t) * 2 * A;
      dst[a] = (float)hr;
      dst[A + a] = (float)hi;
    }
  }
  const U4 r = draw(d, b, ST_NOISE, (uint32_t)((a * F + f) * T + t));
  const double2 z = box_muller(r.x, r.y);
  const double sd = sqrt(d.no / 2.0);
  yr += sd * z.x;
  yi += sd * z.y;
  const size_t ft = ((size_t)b * F + f) * T + t;
  y[ft * 2 * A + a] = (float)yr;
  y[ft * 2 * A + A + a] = (float)yi;
  if (y_re) {
    y_re[ft * A + a] = (float)yr;
    y_im[ft * A + a] = (float)yi;
  }
}

// Nearest own pilot of RE (f, t) in Manhattan distance, first in the pilot order
// (subcarrier-major, then DMRS symbol): the distance is separable over the Cartesian pilot
// grid, so it is the smallest own-group subcarrier nearest f and the first listed DMRS
// symbol nearest t (oracle: synth_ref.nearest_pilot, the general argmin).
__device__ __forceinline__ void nearest_pilot(const nrx_gen_desc& d, int u, int f, int t, int& fp, int& tp) {
  const int c = d.cdm_group[u];
  if ((f & 1) == c) fp = f;
  else fp = f - 1 >= 0 ? f - 1 : f + 1;
  int best = 1 << 30;
  tp = d.dmrs_symbols[0];
  for (int k = 0; k < d.num_dmrs_symbols; ++k) {
    const int dt = abs(t - d.dmrs_symbols[k]);
    if (dt < best) {
      best = dt;
      tp = d.dmrs_symbols[k];
    }
  }
}

__device__ __forceinline__ double2 ls(const float* y, const GenWs& w, const nrx_gen_desc& d, int64_t b, int u,
                                      int fp, int tp, int a) {
  const int U = d.num_tx, F = d.num_subcarriers, T = d.num_symbols, A = d.num_rx_ant;
  const double2 x = w.x[(((size_t)b * U + u) * F + fp) * T + tp];
  if (x.x == 0.0 && x.y == 0.0) return make_double2(0.0, 0.0);
  const size_t ft = ((size_t)b * F + fp) * T + tp;
  const double yr = y[ft * 2 * A + a], yi = y[ft * 2 * A + A + a];
  const double den = x.x * x.x + x.y * x.y;
  return make_double2((yr * x.x + yi * x.y) / den, (yi * x.x - yr * x.y) / den);
}

// one thread per (b, u, f, t, a)
__global__ __launch_bounds__(256) void k_gen_ls(nrx_gen_desc d, GenWs w, const float* __restrict__ y,
                                                float* __restrict__ h_hat) {
  const int U = d.num_tx, F = d.num_subcarriers, T = d.num_symbols, A = d.num_rx_ant;
  const int64_t n = (int64_t)d.batch * U * F * T * A;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int a = (int)(i % A);
  const int64_t r = i / A;
  const int t = (int)(r % T);
  const int f = (int)((r / T) % F);
  const int u = (int)((r / ((int64_t)T * F)) % U);
  const int64_t b = r / ((int64_t)T * F * U);
  int fp, tp;
  nearest_pilot(d, u, f, t, fp, tp);
  const double2 v = ls(y, w, d, b, u, fp, tp, a);
  h_hat[r * 2 * A + a] = (float)v.x;
  h_hat[r * 2 * A + A + a] = (float)v.y;
}

// Aerial pilot list [B][Npil][U][A], p = (k * nprb + prb) * 6 + j, subcarrier prb*12 + cdm + 2j
// (nrx.h nrx_aerial_io); one thread per element.
__global__ __launch_bounds__(256) void k_gen_ls_aerial(nrx_gen_desc d, GenWs w, const float* __restrict__ y,
                                                       float* __restrict__ h_re, float* __restrict__ h_im) {
  const int U = d.num_tx, F = d.num_subcarriers, A = d.num_rx_ant;
  const int nprb = F / 12, npl = d.num_dmrs_symbols * nprb * 6;
  const int64_t n = (int64_t)d.batch * npl * U * A;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int a = (int)(i % A);
  const int u = (int)((i / A) % U);
  const int p = (int)((i / ((int64_t)A * U)) % npl);
  const int64_t b = i / ((int64_t)A * U * npl);
  const int j = p % 6, prb = (p / 6) % nprb, k = p / (6 * nprb);
  const double2 v = ls(y, w, d, b, u, prb * 12 + d.cdm_group[u] + 2 * j, d.dmrs_symbols[k], a);
  h_re[i] = (float)v.x;
  h_im[i] = (float)v.y;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// grid (G, U): workgroup (g, u) walks the slots b = g, g + G, ... of user u; per (b, u) a
// block reduction gives the bit errors (and whether the grid has any), accumulated in
// registers; 3 int64 atomics per workgroup at the end (G <= 32 keeps same-address atomics
// few: the per-(b, u) atomics of a one-block-per-grid layout serialised at L2)
__global__ __launch_bounds__(256) void k_count_errors(nrx_count_io c, int G) {
  __shared__ unsigned red[4];
  const int U = c.num_tx, F = c.num_subcarriers, T = c.num_symbols, BS = c.bits_stride;
  const int u = blockIdx.y;
  unsigned long long err_tot = 0, bits_tot = 0, blk_err = 0, blks = 0;
  int ndata = 0;
  for (int t = 0; t < T; ++t) ndata += !((c.dmrs_symbol_mask >> t) & 1);
  for (int b = blockIdx.x; b < c.batch; b += G) {
    const int64_t bu = (int64_t)b * U + u;
    if (c.active[bu] <= 0.0f) continue;        // uniform per block
    const int m = c.mcs ? c.mcs[bu] : 0;
    const int nb = c.mcs_bits[m];
    const int head = c.num_heads > 1 ? m : 0;
    const float* l = c.llr + ((size_t)head * c.batch * U + bu) * (size_t)F * T * BS;
    const uint8_t* sb = c.bits + (size_t)bu * F * T * BS;
    unsigned err = 0;
    for (int i = threadIdx.x; i < F * T; i += 256) {
      if ((c.dmrs_symbol_mask >> (i % T)) & 1) continue;
      for (int k = 0; k < nb; ++k) err += (uint8_t)(l[(size_t)i * BS + k] > 0.0f) != sb[(size_t)i * BS + k];
    }
    err = wave_sum(err);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = err;
    __syncthreads();
    const unsigned e = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    err_tot += e;
    bits_tot += (unsigned long long)ndata * F * nb;
    blk_err += e ? 1 : 0;
    blks += 1;
  }
  if (threadIdx.x == 0 && blks) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(c.counts) + 4 * u;
    atomicAdd(o + 0, err_tot);
    atomicAdd(o + 1, bits_tot);
    atomicAdd(o + 2, blk_err);
    atomicAdd(o + 3, blks);
  }
}

// Same counters for the common LLR widths (bits_stride 2, 4, 6, 8), one (slot, RE) unit
// per thread: a workgroup (g, u) walks the units of its slots as one flat index space,
// kCntUnroll units per thread per step with every load issued unconditionally (clamped
// index, masked afterwards) before any compare; per-slot bit errors gather in LDS.  nrx_rt,
// 128 slots: 10.2 us vs 13.4 us for the slot loop above.  Measured flat in the layout
// (profiles/r02/ab_count_errors.txt): 4 or 12 units per step, G = 8 / 16 / 32 slot groups
// of 1024 / 512 / 256 threads all 9.5-11.7 us; G = 128 (four times the same-address int64
// atomics) 16.4 us.
#ifndef NRX_CNT_UNROLL
#define NRX_CNT_UNROLL 4
#endif
#ifndef NRX_CNT_T
#define NRX_CNT_T 256
#endif
#ifndef NRX_CNT_G
#define NRX_CNT_G 32
#endif
constexpr int kCntSlots = 64;
constexpr int kCntUnroll = NRX_CNT_UNROLL;

template <int BSC>
__global__ __launch_bounds__(NRX_CNT_T) void k_count_errors_re(nrx_count_io c, int G) {
  __shared__ unsigned s_err[kCntSlots];
  __shared__ int s_nb[kCntSlots];          // bits of the slot's MCS, 0 when the user is inactive
  __shared__ long long s_l[kCntSlots];     // element offset of the slot's LLR grid (its head)
  __shared__ long long s_b[kCntSlots];     // element offset of the slot's bit grid
  const int U = c.num_tx, F = c.num_subcarriers, T = c.num_symbols;
  const int u = blockIdx.y;
  const int FT = F * T;
  unsigned long long err_tot = 0, bits_tot = 0, blk_err = 0, blks = 0;
  int ndata = 0;
  for (int t = 0; t < T; ++t) ndata += !((c.dmrs_symbol_mask >> t) & 1);
  const int nslots = (c.batch - (int)blockIdx.x + G - 1) / G;
  for (int j0 = 0; j0 < nslots; j0 += kCntSlots) {
    const int nj = nslots - j0 < kCntSlots ? nslots - j0 : kCntSlots;
    if ((int)threadIdx.x < nj) {
      const long long bu = (long long)((int)blockIdx.x + G * (j0 + (int)threadIdx.x)) * U + u;
      int nb = 0, head = 0;
      if (c.active[bu] > 0.0f) {
        const int m = c.mcs ? c.mcs[bu] : 0;
        nb = c.mcs_bits[m];
        head = c.num_heads > 1 ? m : 0;
      }
      s_nb[threadIdx.x] = nb;
      s_l[threadIdx.x] = ((long long)head * c.batch * U + bu) * FT * BSC;
      s_b[threadIdx.x] = bu * FT * BSC;
      s_err[threadIdx.x] = 0;
    }
    __syncthreads();
    const int n = nj * FT;
    for (int e0 = 0; e0 < n; e0 += NRX_CNT_T * kCntUnroll) {
      float lv[kCntUnroll][BSC];
      uint8_t sv[kCntUnroll][BSC];
      int jl[kCntUnroll], ii[kCntUnroll];
#pragma unroll
      for (int q = 0; q < kCntUnroll; ++q) {
        int e = e0 + q * NRX_CNT_T + (int)threadIdx.x;
        e = e < n ? e : n - 1;
        jl[q] = e / FT;
        ii[q] = e - jl[q] * FT;
        const float* lp = c.llr + s_l[jl[q]] + (long long)ii[q] * BSC;
        const uint8_t* bp = c.bits + s_b[jl[q]] + (long long)ii[q] * BSC;
#pragma unroll
        for (int k = 0; k < BSC; ++k) {
          lv[q][k] = lp[k];
          sv[q][k] = bp[k];
        }
      }
#pragma unroll
      for (int q = 0; q < kCntUnroll; ++q) {
        const int e = e0 + q * NRX_CNT_T + (int)threadIdx.x;
        const int nb = s_nb[jl[q]];
        if (e >= n || !nb || ((c.dmrs_symbol_mask >> (ii[q] % T)) & 1)) continue;
        unsigned er = 0;
#pragma unroll
        for (int k = 0; k < BSC; ++k) er += (k < nb && (uint8_t)(lv[q][k] > 0.0f) != sv[q][k]) ? 1u : 0u;
        if (er) atomicAdd(&s_err[jl[q]], er);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int j = 0; j < nj; ++j) {
        if (!s_nb[j]) continue;
        err_tot += s_err[j];
        bits_tot += (unsigned long long)ndata * F * s_nb[j];
        blk_err += s_err[j] ? 1 : 0;
        blks += 1;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && blks) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(c.counts) + 4 * u;
#ifdef NRX_CNT_NOATOM
    if (err_tot == 12345678) o[0] = 0;
#else
    atomicAdd(o + 0, err_tot);
    atomicAdd(o + 1, bits_tot);
    atomicAdd(o + 2, blk_err);
    atomicAdd(o + 3, blks);
#endif
  }
}

size_t al(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace

size_t gen_workspace_bytes(const nrx_gen_desc& d, GenWs* w, char* base) {
  const size_t B = d.batch, U = d.num_tx, F = d.num_subcarriers, T = d.num_symbols, A = d.num_rx_ant,
               L = d.num_taps;
  size_t o = 0;
  auto take = [&](size_t n) {
    char* p = base ? base + o : nullptr;
    o += al(n);
    return p;
  };
  GenWs v;
  v.x = (double2*)take(B * U * F * T * sizeof(double2));
  v.gt = (double2*)take(B * U * A * L * T * sizeof(double2));
  v.tau = (double*)take(B * U * L * sizeof(double));
  v.spdp = (double*)take(B * U * L * sizeof(double));
  v.mcs = (uint8_t*)take(B * U);
  v.active = (float*)take(B * U * sizeof(float));
  if (w) *w = v;
  return o;
}

hipError_t launch_generate(const nrx_gen_desc& d, const nrx_gen_out& o, void* ws, hipStream_t st) {
  GenWs w;
  gen_workspace_bytes(d, &w, (char*)ws);
  const int64_t B = d.batch, U = d.num_tx, F = d.num_subcarriers, T = d.num_symbols, A = d.num_rx_ant,
                L = d.num_taps;
  auto blocks = [](int64_t n) { return (unsigned)((n + 255) / 256); };
  k_gen_params<<<(unsigned)B, 64, 0, st>>>(d, w, o.active, o.mcs_mask, o.mcs);
  k_gen_taps<<<(unsigned)((B * U * A * L + kTapGroups - 1) / kTapGroups), kTapGroups * kT, 0, st>>>(d, w);
  k_gen_tx<<<blocks(B * U * F * T), 256, 0, st>>>(d, w, o.bits, o.bits_stride);
  const int at = (int)(A * T);
  int FB = 256 / at;
  if (FB > 4) FB = 4;
  k_gen_rx<<<dim3((unsigned)((F + FB - 1) / FB), (unsigned)B), FB * at, 0, st>>>(d, w, FB, o.y, o.h, o.y_real,
                                                                                o.y_imag);
  if (o.h_hat) k_gen_ls<<<blocks(B * U * F * T * A), 256, 0, st>>>(d, w, o.y, o.h_hat);
  if (o.h_ls_real)
    k_gen_ls_aerial<<<blocks(B * d.num_dmrs_symbols * (F / 12) * 6 * U * A), 256, 0, st>>>(d, w, o.y, o.h_ls_real,
                                                                                          o.h_ls_imag);
  return hipGetLastError();
}

hipError_t launch_count_errors(const nrx_count_io& c, hipStream_t st) {
  const int G = c.batch < NRX_CNT_G ? c.batch : NRX_CNT_G;
  const dim3 grid(G, c.num_tx);
  switch (c.bits_stride) {
    case 2: k_count_errors_re<2><<<grid, NRX_CNT_T, 0, st>>>(c, G); break;
    case 4: k_count_errors_re<4><<<grid, NRX_CNT_T, 0, st>>>(c, G); break;
    case 6: k_count_errors_re<6><<<grid, NRX_CNT_T, 0, st>>>(c, G); break;
    case 8: k_count_errors_re<8><<<grid, NRX_CNT_T, 0, st>>>(c, G); break;
    default: {
      const int G32 = c.batch < 32 ? c.batch : 32;
      k_count_errors<<<dim3(G32, c.num_tx), 256, 0, st>>>(c, G32);
    }
  }

  return hipGetLastError();
}

}  // namespace nrx
