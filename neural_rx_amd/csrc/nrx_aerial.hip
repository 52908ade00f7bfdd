// nrx_aerial.hip -- the Aerial (cuPHY / TensorRT) front- and back-end of the engine:
// the NeuralReceiverONNX contract (neural_rx.py:1773-1812, NRPreprocessing 1614-1711;
// TF structure in "neural_rx copy_pytorch.py" 959-1092) on the GPU.
//
//   k_aerial_tables   per user: nearest-DMRS-pilot index of every RE of one PRB and the
//                     positional encoding pe[U][F][T][2]     (_calculate_nn_indices)
//   k_aerial_inputs   y = cat(y_re, y_im); h_hat = FOCC pair average of the LS pilots,
//                     gathered per PRB by the NN index     (_focc_removal, _nn_interpolation)
//   k_aerial_llr      llr[B][U][F][T][bits] -> Aerial [B][bits][U][F][T], negated
//                     (Sionna LLR = log p1/p0, Aerial = log p0/p1; neural_rx.py:1808-1811)
//   k_llr_demap       grid LLRs -> per-user coded-bit vector of the data REs
//
// All four are gathers / transposes over a few MB: HBM-bound, one pass, coalesced along
// the fastest output axis.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nrx_internal.h"

namespace nrx {

// One workgroup per user.  RE list of a PRB: (t, sc), t-major (TF 'xy' meshgrid of
// (arange(12), arange(T))); pilot list: (k, j) symbol-major, i = k * npil + j.  The NN index
// is the first pilot at minimal Manhattan distance; the PE components are the minimal
// |t - t_k| and |sc - sc_j| over all pilots, each normalised over the 12 x T REs of the PRB
// with the population std (where std > 0), stacked [time, freq] and repeated over PRBs.
__global__ __launch_bounds__(256) void k_aerial_tables(const int32_t* __restrict__ ofdm_pos,
                                                        const int32_t* __restrict__ sc_pos, int nsym,
                                                        int npil, int T, int F, int32_t* __restrict__ nn,
                                                        float* __restrict__ pe) {
  __shared__ double red[2][256];
  __shared__ float dtf[2][12 * 16];
  const int u = blockIdx.x;
  const int i = threadIdx.x;
  const int nre = 12 * T;
  double st = 0.0, sf = 0.0;
  if (i < nre) {
    const int t = i / 12, sc = i % 12;
    int best = 0, bestd = 1 << 30, dt = 1 << 30, df = 1 << 30;
    for (int k = 0; k < nsym; ++k) {
      const int pt = ofdm_pos[u * nsym + k];
      for (int j = 0; j < npil; ++j) {
        const int ps = sc_pos[u * npil + j];
        const int a = abs(t - pt), c = abs(sc - ps);
        if (a + c < bestd) {
          bestd = a + c;
          best = k * npil + j;
        }
        dt = a < dt ? a : dt;
        df = c < df ? c : df;
      }
    }
    nn[(u * T + t) * 12 + sc] = best;
    dtf[0][i] = (float)dt;
    dtf[1][i] = (float)df;
    st = dt;
    sf = df;
  }
  // means
  red[0][i] = st;
  red[1][i] = sf;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (i < s) {
      red[0][i] += red[0][i + s];
      red[1][i] += red[1][i + s];
    }
    __syncthreads();
  }
  const double mt = red[0][0] / nre, mf = red[1][0] / nre;
  __syncthreads();
  // population variances
  double vt = 0.0, vf = 0.0;
  if (i < nre) {
    vt = (dtf[0][i] - mt) * (dtf[0][i] - mt);
    vf = (dtf[1][i] - mf) * (dtf[1][i] - mf);
  }
  red[0][i] = vt;
  red[1][i] = vf;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (i < s) {
      red[0][i] += red[0][i + s];
      red[1][i] += red[1][i + s];
    }
    __syncthreads();
  }
  const double sdt = sqrt(red[0][0] / nre), sdf = sqrt(red[1][0] / nre);
  if (i < nre) {
    const int t = i / 12, sc = i % 12;
    double pt = dtf[0][i] - mt, pf = dtf[1][i] - mf;
    if (sdt > 0.0) pt /= sdt;
    if (sdf > 0.0) pf /= sdf;
    for (int prb = 0; prb * 12 < F; ++prb) {
      float* dst = pe + (((size_t)u * F + prb * 12 + sc) * T + t) * 2;
      dst[0] = (float)pt;
      dst[1] = (float)pf;
    }
  }
}

// One thread per (b, f, t, a) of y and per (b, u, f, t, a) of h_hat; grid.y = B.
// h_ls pilot p = (k * nprb + prb) * npil + j (symbol k, PRB, pilot j); its FOCC partner is
// p ^ 1 (adjacent pilot of the same PRB and symbol; npil even).
__global__ __launch_bounds__(256) void k_aerial_inputs(const float* __restrict__ y_re, const float* __restrict__ y_im,
                                                        const float* __restrict__ h_re, const float* __restrict__ h_im,
                                                        const int32_t* __restrict__ nn, int U, int F, int T, int A,
                                                        int nsym, int npil, float* __restrict__ y,
                                                        float* __restrict__ h) {
  const int b = blockIdx.y;
  const int nprb = F / 12;
  const int npl = nsym * nprb * npil;       // pilots per (b, u, a)
  const int per_y = F * T * A;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < per_y) {
    const int a = idx % A, ft = idx / A;    // (f, t) flattened
    const size_t src = (size_t)b * per_y + idx;
    float* dst = y + ((size_t)b * F * T + ft) * 2 * A;
    dst[a] = y_re[src];
    dst[A + a] = y_im[src];
  }
  const int hidx = idx - ((per_y + 255) / 256) * 256;   // second range of blocks: h_hat
  if (hidx >= 0 && hidx < U * per_y) {
    const int a = hidx % A;
    int r = hidx / A;
    const int t = r % T;
    r /= T;
    const int f = r % F;
    const int u = r / F;
    const int prb = f / 12, sc = f % 12;
    const int i = nn[(u * T + t) * 12 + sc];
    const int k = i / npil, j = i % npil;
    const int p = (k * nprb + prb) * npil + j, q = p ^ 1;
    const size_t bp = (((size_t)b * npl + p) * U + u) * A + a;
    const size_t bq = (((size_t)b * npl + q) * U + u) * A + a;
    float* dst = h + ((((size_t)b * U + u) * F + f) * T + t) * 2 * A;
    dst[a] = (h_re[bp] + h_re[bq]) / 2.0f;
    dst[A + a] = (h_im[bp] + h_im[bq]) / 2.0f;
  }
}

// out[b][k][u][f][t] = -llr[b][u][f][t][k], k < bits (one thread per output element).
__global__ __launch_bounds__(256) void k_aerial_llr(const float* __restrict__ llr, int U, int F, int T, int bits_max,
                                                     int bits, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int n = bits * U * F * T;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= n) return;
  const int uft = idx % (U * F * T);
  const int k = idx / (U * F * T);
  out[(size_t)b * n + idx] = -llr[((size_t)b * U * F * T + uft) * bits_max + k];
}

// Coded-bit layout: out[b][u][i * bits + k] = llr[b][u][f][t][k] for the
// i-th data RE (t * F + f = data_re[i], symbol-major as Sionna's ResourceGridDemapper and
// DataEvaluator.post_process_llrs gather it: CGNNOFDM.forward neural_rx.py:843-852,
// onnx_utils.py:473-516); one thread per output element.
__global__ __launch_bounds__(256) void k_llr_demap(const float* __restrict__ llr, int F, int T, int bits_stride,
                                                    int bits, const int32_t* __restrict__ data_re, int n_data,
                                                    size_t total, float* __restrict__ out) {
  const size_t n = (size_t)n_data * bits;   // per (b, u)
  for (size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
    const size_t bu = idx / n;
    const int r = (int)(idx - bu * n);
    const int i = r / bits, k = r % bits;
    const int re = data_re[i];
    const int t = re / F, f = re % F;
    out[idx] = llr[((bu * F + f) * T + t) * bits_stride + k];
  }
}

hipError_t launch_llr_demap(const float* llr, int B, int U, int F, int T, int bits_stride, int bits,
                            const int32_t* data_re, int n_data, float* out, hipStream_t st) {
  const size_t total = (size_t)B * U * n_data * bits;
  size_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  k_llr_demap<<<(unsigned)blocks, 256, 0, st>>>(llr, F, T, bits_stride, bits, data_re, n_data, total, out);
  return hipGetLastError();
}

hipError_t launch_aerial_tables(const int32_t* ofdm_pos, const int32_t* sc_pos, int U, int nsym, int npil, int T,
                                int F, int32_t* nn, float* pe, hipStream_t st) {
  k_aerial_tables<<<U, 256, 0, st>>>(ofdm_pos, sc_pos, nsym, npil, T, F, nn, pe);
  return hipGetLastError();
}

hipError_t launch_aerial_inputs(const float* y_re, const float* y_im, const float* h_re, const float* h_im,
                                const int32_t* nn, int B, int U, int F, int T, int A, int nsym, int npil, float* y,
                                float* h, hipStream_t st) {
  const int per_y = F * T * A;
  const int blocks = (per_y + 255) / 256 + (U * per_y + 255) / 256;
  k_aerial_inputs<<<dim3(blocks, B), 256, 0, st>>>(y_re, y_im, h_re, h_im, nn, U, F, T, A, nsym, npil, y, h);
  return hipGetLastError();
}

hipError_t launch_aerial_llr(const float* llr, int B, int U, int F, int T, int bits_max, int bits, float* out,
                             hipStream_t st) {
  const int n = bits * U * F * T;
  k_aerial_llr<<<dim3((n + 255) / 256, B), 256, 0, st>>>(llr, U, F, T, bits_max, bits, out);
  return hipGetLastError();
}

// ------------------------------------------------------------ y input layouts
// CGNN channel order [Re a0..a(A-1), Im a0..a(A-1)] from the wrappers' input layouts:
//   layout 1: Sionna resource grid y[B][1][A][T][F] complex64 (CGNNOFDM.forward,
//             neural_rx.py:831-833: y[:,0].permute(0,3,2,1), cat(real, imag))
//   layout 2: split rx_slot_real / rx_slot_imag [B][F][T][A] (NeuralReceiverONNX.forward,
//             neural_rx.py:1787: cat([y_real, y_imag], -1))
// One thread per (b, t, f), f fastest: the complex grid is read coalesced along F.
__global__ __launch_bounds__(256) void k_y_layout(const float* __restrict__ y0, const float* __restrict__ y1,
                                                  int layout, int F, int T, int A, float* __restrict__ y) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= F * T) return;
  const int t = i / F, f = i % F;
  float* o = y + (((size_t)b * F + f) * T + t) * 2 * A;
  if (layout == 1) {
    const float2* g = reinterpret_cast<const float2*>(y0) + (size_t)b * A * T * F + (size_t)t * F + f;
    for (int a = 0; a < A; ++a) {
      const float2 v = g[(size_t)a * T * F];
      o[a] = v.x;
      o[A + a] = v.y;
    }
  } else {
    const size_t q = (((size_t)b * F + f) * T + t) * A;
    for (int a = 0; a < A; ++a) {
      o[a] = y0[q + a];
      o[A + a] = y1[q + a];
    }
  }
}

hipError_t launch_y_layout(const float* y0, const float* y1, int layout, int B, int F, int T, int A, float* y,
                           hipStream_t st) {
  k_y_layout<<<dim3((F * T + 255) / 256, B), 256, 0, st>>>(y0, y1, layout, F, T, A, y);
  return hipGetLastError();
}

}  // namespace nrx
