// nrx_api.cpp -- host side of libnrx.so: C ABI (include/nrx.h), weight validation and
// packing, workspace sizing, forward dispatch, and the product-side positional encoding.
//
// Weight order = Keras get_weights() of the reference CGNN:
//   StateInit x num_init : 3 x (dw[3,3,Cin,1], pw[1,1,Cin,Cout], b[Cout])
//   num_it x [ Agg: (W[ds,64], b), (W[64,ds], b) ; Update: 3 x sep ]
//   LLR heads x H : (W[ds,128], b), (W[128,bits], b)
//   ChEst : (W[ds,128], b), (W[128,2A], b)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/nrx.h"
#include "nrx_internal.h"

namespace nrx {
hipError_t launch_forward_f16(const FwdArgs<_Float16, float, _Float16>& args, const ModelW<_Float16, float>& W,
                              int num_it, hipStream_t st, Prof* prof, const FusedCtl& fc);
bool fused_would_run(const FwdArgs<_Float16, float, _Float16>& args, int num_it, const FusedCtl& fc);
size_t fused_sync_bytes();
hipError_t fused_sync_status(void* sync, int* st, bool reset, hipEvent_t last);
hipError_t launch_forward_f64(const FwdArgs<double, double, float>& args,
                              const ModelW<double, double>& W, int num_it, hipStream_t st,
                              Prof* prof);
hipError_t setup_kernels();
int strip_width(int precision);
}  // namespace nrx

using namespace nrx;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(NRX_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct LayerShape {
  enum Kind { SEP, DENSE } kind;
  int cin, cout;
};

// Topology checks: the kernels are specialised for the in-scope configs.
int check_desc(const nrx_desc* d) {
  if (!d) return fail(NRX_ERR_INVALID_ARG, "desc is NULL");
  if (d->d_s != kDS) return fail(NRX_ERR_UNSUPPORTED, "kernels are built for d_s = 56");
  if (d->init_units[0] != kHID || d->init_units[1] != kHID || d->state_units[0] != kHID ||
      d->state_units[1] != kHID || d->readout_units != kHID || d->agg_units != kAGG)
    return fail(NRX_ERR_UNSUPPORTED, "kernels are built for 128/128 convs, 64 agg, 128 readout");
  if (d->num_rx_ant < 1 || 4 * d->num_rx_ant + 2 > 128 || 2 * d->num_rx_ant > 32)
    return fail(NRX_ERR_UNSUPPORTED, "num_rx_ant must be 1..16");
  if (d->num_it < 1 || d->num_it > kMaxIt) return fail(NRX_ERR_UNSUPPORTED, "num_it must be 1..8");
  if (d->num_mcs < 1 || d->num_mcs > kMaxHeads) return fail(NRX_ERR_UNSUPPORTED, "num_mcs must be 1..8");
  for (int m = 0; m < d->num_mcs; ++m)
    if (d->bits[m] < 1 || d->bits[m] > 8) return fail(NRX_ERR_UNSUPPORTED, "bits must be 1..8");
  if (!d->var_mcs_masking && d->num_mcs > 3)
    return fail(NRX_ERR_UNSUPPORTED, "at most 3 LLR heads (fused readout staging)");
  if (d->use_h_hat != 0 && d->use_h_hat != 1) return fail(NRX_ERR_INVALID_ARG, "use_h_hat must be 0/1");
  return NRX_OK;
}

int num_init(const nrx_desc* d) { return d->var_mcs_masking ? 1 : d->num_mcs; }
int num_heads(const nrx_desc* d) { return d->var_mcs_masking ? 1 : d->num_mcs; }
int bits_max(const nrx_desc* d) {
  int b = 0;
  for (int m = 0; m < d->num_mcs; ++m) b = d->bits[m] > b ? d->bits[m] : b;
  return b;
}
int init_cin(const nrx_desc* d) { return (d->use_h_hat ? 4 : 2) * d->num_rx_ant + 2; }
int init_a2p(int num_rx_ant) { return 2 * num_rx_ant <= 8 ? 8 : (2 * num_rx_ant <= 16 ? 16 : 32); }

std::vector<LayerShape> layer_list(const nrx_desc* d) {
  std::vector<LayerShape> L;
  for (int m = 0; m < num_init(d); ++m) {
    L.push_back({LayerShape::SEP, init_cin(d), kHID});
    L.push_back({LayerShape::SEP, kHID, kHID});
    L.push_back({LayerShape::SEP, kHID, kDS});
  }
  for (int i = 0; i < d->num_it; ++i) {
    L.push_back({LayerShape::DENSE, kDS, kAGG});
    L.push_back({LayerShape::DENSE, kAGG, kDS});
    L.push_back({LayerShape::SEP, 2 * kDS + 2, kHID});
    L.push_back({LayerShape::SEP, kHID, kHID});
    L.push_back({LayerShape::SEP, kHID, kDS});
  }
  const int nh = num_heads(d);
  for (int h = 0; h < nh; ++h) {
    L.push_back({LayerShape::DENSE, kDS, kHID});
    L.push_back({LayerShape::DENSE, kHID, d->var_mcs_masking ? bits_max(d) : d->bits[h]});
  }
  L.push_back({LayerShape::DENSE, kDS, kHID});
  L.push_back({LayerShape::DENSE, kHID, 2 * d->num_rx_ant});
  return L;
}

std::vector<int64_t> weight_sizes(const nrx_desc* d) {
  std::vector<int64_t> s;
  for (const auto& l : layer_list(d)) {
    if (l.kind == LayerShape::SEP) {
      s.push_back(9LL * l.cin);
      s.push_back((int64_t)l.cin * l.cout);
      s.push_back(l.cout);
    } else {
      s.push_back((int64_t)l.cin * l.cout);
      s.push_back(l.cout);
    }
  }
  return s;
}

int round_up(int x, int m) { return (x + m - 1) / m * m; }
int pow2_at_least(int x, int lo) {
  int p = lo;
  while (p < x) p *= 2;
  return p;
}
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Host-side packing into one contiguous blob per precision; pointers are patched to the
// device copy after upload.
template <class WT, class BT>
struct Packer {
  std::vector<char> blob;
  size_t put_w(const std::vector<WT>& v) {
    size_t off = align256(blob.size());
    blob.resize(off + v.size() * sizeof(WT));
    memcpy(blob.data() + off, v.data(), v.size() * sizeof(WT));
    return off;
  }
  size_t put_b(const std::vector<BT>& v) {
    size_t off = align256(blob.size());
    blob.resize(off + v.size() * sizeof(BT));
    memcpy(blob.data() + off, v.data(), v.size() * sizeof(BT));
    return off;
  }
  // offsets relative to blob start, fixed up later
  struct SepOff { size_t dw, pw, b; };
  struct DenOff { size_t w, b; };
  // `pos` (optional) places input channel c at packed position pos[c] (StateInit conv1:
  // the kernel's z image is [y | pe | h] with the antenna blocks padded to A2P).
  SepOff sep(const float* dw, const float* pw, const float* b, int cin, int cout, int cinp, int coutp,
             const std::vector<int>* pos = nullptr) {
    std::vector<WT> dwp((size_t)9 * cinp, WT(0)), pwp((size_t)coutp * cinp, WT(0));
    std::vector<BT> bp(coutp, BT(0));
    auto P = [&](int c) { return pos ? (*pos)[c] : c; };
    for (int tap = 0; tap < 9; ++tap)
      for (int c = 0; c < cin; ++c) dwp[(size_t)tap * cinp + P(c)] = (WT)dw[(size_t)tap * cin + c];
    for (int c = 0; c < cin; ++c)
      for (int o = 0; o < cout; ++o) pwp[(size_t)o * cinp + P(c)] = (WT)pw[(size_t)c * cout + o];
    for (int o = 0; o < cout; ++o) bp[o] = (BT)b[o];
    SepOff r;
    r.dw = put_w(dwp);
    r.pw = put_w(pwp);
    r.b = put_b(bp);
    return r;
  }
  // kperm: 0 = natural K order; 32 / 16 = K permuted so that the MFMA C layout of the
  // producing layer (lane (t,g) holds channels 16n + 4g + j (f16) / 16n + g + 4j (f64))
  // is directly the B fragment (kernels: CFrag).
  static int kperm_channel(int p, int kperm) {
    if (kperm == 32) return 32 * (p / 32) + 16 * ((p % 8) / 4) + 4 * ((p % 32) / 8) + (p % 4);
    if (kperm == 16) return 16 * (p / 16) + (p % 16) / 4 + 4 * (p % 4);
    return p;
  }
  DenOff dense(const float* w, const float* b, int cin, int cout, int cinp, int coutp, int kperm = 0) {
    std::vector<WT> wp((size_t)coutp * cinp, WT(0));
    std::vector<BT> bp(coutp, BT(0));
    for (int pk = 0; pk < cinp; ++pk) {
      const int c = kperm_channel(pk, kperm);
      if (c >= cin) continue;
      for (int o = 0; o < cout; ++o) wp[(size_t)o * cinp + pk] = (WT)w[(size_t)c * cout + o];
    }
    for (int o = 0; o < cout; ++o) bp[o] = (BT)b[o];
    return DenOff{put_w(wp), put_b(bp)};
  }
};

template <class WT, class BT>
struct DeviceModel {
  ModelW<WT, BT> W{};
  void* dev = nullptr;
  int init_cinp = 0;
};

template <class WT, class BT>
int build_model(const nrx_desc* d, const float* const* w, int kc, DeviceModel<WT, BT>* out) {
  Packer<WT, BT> pk;
  using SO = typename Packer<WT, BT>::SepOff;
  using DO = typename Packer<WT, BT>::DenOff;
  SO init[kMaxInit][3];
  DO agg[kMaxIt][2];
  SO upd[kMaxIt][3];
  DO llr[kMaxHeads][2];
  DO ch[2];
  const int icin = init_cin(d);
  // StateInit input z = [y (2A), pe (2), h (2A)] (copy_pytorch.py:175-183) is laid out
  // with each antenna block padded to A2P = init_a2p(A): y at [0, 2A), h at [A2P, A2P+2A),
  // pe at 2 A2P, 2 A2P + 1 (so that an 8-channel lane chunk is all y, all h or pe: the
  // one-launch forward's conv1 loads them straight from y / h_hat / pe); the padded channels
  // carry zero weights.
  const int a2p = init_a2p(d->num_rx_ant);
  std::vector<int> ipos(icin);
  for (int c = 0; c < icin; ++c) {
    const int a2 = 2 * d->num_rx_ant;
    ipos[c] = c < a2 ? c : (c < a2 + 2 ? 2 * a2p + (c - a2) : a2p + (c - a2 - 2));
  }
  const int icinp = pow2_at_least(round_up(2 * a2p + 2, kc), 32);
  out->init_cinp = icinp;
  int k = 0;
  auto sep = [&](int cin, int cout, int cinp, int coutp, const std::vector<int>* pos = nullptr) {
    SO r = pk.sep(w[k], w[k + 1], w[k + 2], cin, cout, cinp, coutp, pos);
    k += 3;
    return r;
  };
  // every dense layer of the engine consumes an MFMA accumulator tile: K permuted
  auto den = [&](int cin, int cout, int cinp, int coutp) {
    DO r = pk.dense(w[k], w[k + 1], cin, cout, cinp, coutp, kc);
    k += 2;
    return r;
  };
  // f16: conv2 / conv3 read the strip image the previous layer's in-place epilogue wrote
  // straight from its accumulators (lane (t, g) stores tiles 2kc, 2kc+1 as one 16-byte
  // chunk 4kc + g), i.e. their input channels sit in the K-permuted order of the dense
  // layers: channel c at packed position kperm^-1(c)
  std::vector<int> hpos(kHID);
  for (int p = 0; p < kHID; ++p) hpos[Packer<WT, BT>::kperm_channel(p, kc == 32 ? 32 : 0)] = p;
  const std::vector<int>* hp = kc == 32 ? &hpos : nullptr;
  for (int m = 0; m < num_init(d); ++m) {
    init[m][0] = sep(icin, kHID, icinp, kHID, &ipos);
    init[m][1] = sep(kHID, kHID, kHID, kHID, hp);
    init[m][2] = sep(kHID, kDS, kHID, kDSP, hp);
  }
  for (int i = 0; i < d->num_it; ++i) {
    agg[i][0] = den(kDS, kAGG, kDSP, kAGG);
    agg[i][1] = den(kAGG, kDS, kAGG, kDSP);
    upd[i][0] = sep(2 * kDS + 2, kHID, kUPD_CINP, kHID);
    upd[i][1] = sep(kHID, kHID, kHID, kHID, hp);
    upd[i][2] = sep(kHID, kDS, kHID, kDSP, hp);
  }
  for (int h = 0; h < num_heads(d); ++h) {
    const int nb = d->var_mcs_masking ? bits_max(d) : d->bits[h];
    llr[h][0] = den(kDS, kHID, kDSP, kHID);
    llr[h][1] = den(kHID, nb, kHID, 16);
  }
  const int a2 = 2 * d->num_rx_ant;
  ch[0] = den(kDS, kHID, kDSP, kHID);
  ch[1] = den(kHID, a2, kHID, a2 <= 16 ? 16 : 32);

  hipError_t e = hipMalloc(&out->dev, pk.blob.size());
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(weights)");
  e = hipMemcpy(out->dev, pk.blob.data(), pk.blob.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy(weights)");
  char* base = (char*)out->dev;
  auto fs = [&](const SO& o) {
    return SepW<WT, BT>{(const WT*)(base + o.dw), (const WT*)(base + o.pw), (const BT*)(base + o.b)};
  };
  auto fd = [&](const DO& o) { return DenseW<WT, BT>{(const WT*)(base + o.w), (const BT*)(base + o.b)}; };
  for (int m = 0; m < num_init(d); ++m)
    for (int l = 0; l < 3; ++l) out->W.init[m][l] = fs(init[m][l]);
  for (int i = 0; i < d->num_it; ++i) {
    out->W.agg[i][0] = fd(agg[i][0]);
    out->W.agg[i][1] = fd(agg[i][1]);
    for (int l = 0; l < 3; ++l) out->W.upd[i][l] = fs(upd[i][l]);
  }
  for (int h = 0; h < num_heads(d); ++h) {
    out->W.llr[h][0] = fd(llr[h][0]);
    out->W.llr[h][1] = fd(llr[h][1]);
  }
  out->W.chest[0] = fd(ch[0]);
  out->W.chest[1] = fd(ch[1]);
  return NRX_OK;
}

}  // namespace

// Event-pair recorder behind nrx_profile_enable / nrx_profile_read.
struct EventProf : Prof {
  struct Rec { int kid; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  void begin(int kid, void* st) override {
    Rec r{kid, get(), nullptr};
    (void)hipEventRecord(r.a, (hipStream_t)st);
    recs.push_back(r);
  }
  void end(int, void* st) override {
    hipEvent_t e = get();
    (void)hipEventRecord(e, (hipStream_t)st);
    recs.back().b = e;
  }
  // fold finished records into totals
  int64_t launches[K_COUNT] = {0};
  double total_ms[K_COUNT] = {0};
  hipError_t collect() {
    for (auto& r : recs) {
      hipError_t e = hipEventSynchronize(r.b);
      if (e != hipSuccess) return e;
      float ms = 0.f;
      e = hipEventElapsedTime(&ms, r.a, r.b);
      if (e != hipSuccess) return e;
      launches[r.kid] += 1;
      total_ms[r.kid] += ms;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
    return hipSuccess;
  }
  void reset() {
    for (int k = 0; k < K_COUNT; ++k) {
      launches[k] = 0;
      total_ms[k] = 0;
    }
  }
  ~EventProf() override {
    for (auto& r : recs) {
      (void)hipEventDestroy(r.a);
      if (r.b) (void)hipEventDestroy(r.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct nrx_handle {
  nrx_desc desc;
  int device;
  DeviceModel<_Float16, float> m16;
  DeviceModel<double, double> m64;
  EventProf* prof = nullptr;
  void* fused_sync = nullptr;   // k_forward's work queues and dependency counters (zeroed)
  int fused_enabled = 1;    // NRX_FUSED (environment, read once at nrx_create)
  int spin_limit = kFusedSpinLimit;
  int dbg_err = 0;
  int update_rr = kSchedDefault;   // nrx_update_schedule (NRX_UPDATE_RR at nrx_create)
  // one-stream rule of the one-launch forward: an event the handle owns, recorded
  // behind every eager one-launch forward, stands for "that forward is done" -- the caller's
  // stream itself is never kept (it may be destroyed between calls).  last_stream is compared,
  // never used.  Forwards captured into a hipGraph record no event: graph replays are outside
  // the guard (the caller keeps replays of one handle on one stream).
  hipEvent_t last_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool have_last = false;
  FusedCtl fused_ctl() const { return FusedCtl{fused_sync, fused_enabled, spin_limit, dbg_err, update_rr}; }
};

static size_t state_bytes(const nrx_shape* s, int precision) {
  const size_t es = precision == NRX_PREC_F16 ? 2 : 4;
  return align256((size_t)s->batch * s->num_tx * s->num_subcarriers * kT * kDS * es);
}
// pe16 plane [U][F][14][56] f16 of the one-launch forward (f16 workspaces only)
static size_t pe16_bytes(const nrx_shape* s, int precision) {
  return precision == NRX_PREC_F16 ? align256((size_t)s->num_tx * s->num_subcarriers * kT * kDS * 2) : 0;
}

static int check_shape(const nrx_shape* s) {
  if (!s) return fail(NRX_ERR_INVALID_ARG, "shape is NULL");
  if (s->num_symbols != kT) return fail(NRX_ERR_SHAPE, "num_symbols must be 14");
  if (s->batch < 1 || s->batch > 65535) return fail(NRX_ERR_SHAPE, "batch must be 1..65535");
  if (s->num_tx < 1 || s->num_tx > kMaxUsers) return fail(NRX_ERR_SHAPE, "num_tx must be 1..16");
  if (s->num_subcarriers < 1 || s->num_subcarriers > 12 * 275)
    return fail(NRX_ERR_SHAPE, "num_subcarriers must be 1..3300");
  return NRX_OK;
}

template <class WT, class BT, class S>
static void fill_args(FwdArgs<WT, BT, S>& a, const nrx_handle* h, const nrx_io* io, void* ws, int init_cinp) {
  const nrx_desc* d = &h->desc;
  const nrx_shape* s = &io->shape;
  a.B = s->batch;
  a.llr_B = s->batch;
  a.U = s->num_tx;
  a.F = s->num_subcarriers;
  a.A = d->num_rx_ant;
  a.M = d->num_mcs;
  a.H = num_heads(d);
  a.init_cinp = init_cinp;
  a.num_init = num_init(d);
  a.masking = d->var_mcs_masking;
  a.use_h = d->use_h_hat;
  a.bits_max = bits_max(d);
  for (int i = 0; i < kMaxHeads; ++i)
    a.head_bits[i] = i < a.H ? (d->var_mcs_masking ? bits_max(d) : d->bits[i]) : 0;
  a.y = io->y;
  a.pe = io->pe;
  a.h_hat = io->h_hat;
  a.active = io->active;
  a.mcs_mask = io->mcs_mask;
  a.llr = io->llr;
  a.h_ref = io->h_ref;
  char* p = (char*)ws;
  a.norm = (double*)p;
  p += align256((size_t)s->batch * sizeof(double));
  const size_t sb = state_bytes(s, io->precision);
  a.s_in = (S*)(p + sb);
  a.s_out = (S*)p;
  a.a = (S*)(p + 3 * sb);
  a.a_out = (S*)(p + 2 * sb);
  a.ws_base = (const char*)ws;
  const size_t pb = pe16_bytes(s, io->precision);
  a.pe16 = pb ? (S*)(p + 4 * sb) : nullptr;
  const size_t total = (size_t)(p + 4 * sb + pb - (char*)ws);
  a.ws_bytes = total < 0xFFFFFFFFull ? (unsigned)total : 0xFFFFFFFFu;
}


static int forward_slots(nrx_handle* h, const nrx_io* io, int llr_B, void* workspace, hipStream_t st);

// NRX_ERR_BUSY when a forward that would take the one-launch path arrives on a stream other than
// the previous one-launch forward's while that forward has not finished (the counters are per
// handle).  Called before ANY launch of a forward entry point, so a refused call has launched
// nothing (the y-layout / Aerial preprocessing used to run first).
static int chunk_slots(const nrx_shape* s, int precision);

static int fused_busy(nrx_handle* h, const nrx_io* io, hipStream_t st, bool* takes) {
  *takes = false;
  if (io->precision != NRX_PREC_F16) return NRX_OK;
  // decided on the shapes the forward will run: a forward above the 1 GB workspace runs as slot
  // chunks (nrx_forward), full ones of chunk_slots slots and a remainder, and each chunk may take
  // the one-launch path although the whole batch would not
  const int B = io->shape.batch, bc = chunk_slots(&io->shape, io->precision);
  for (const int n : {bc < B ? bc : B, bc < B && B % bc ? B % bc : 0}) {
    if (n <= 0) continue;
    nrx_io c = *io;
    c.shape.batch = n;
    FwdArgs<_Float16, float, _Float16> a{};
    fill_args(a, h, &c, nullptr, h->m16.init_cinp);   // pointers unused: the decision needs sizes only
    *takes = *takes || fused_would_run(a, io->num_it, h->fused_ctl());
  }
  if (*takes && h->have_last && h->last_stream != st && hipEventQuery(h->last_ev) == hipErrorNotReady)
    return fail(NRX_ERR_BUSY, "a one-launch forward of this handle is still running on another stream");
  return NRX_OK;
}

extern "C" {

const char* nrx_last_error(void) { return g_err.c_str(); }
int32_t nrx_api_version(void) { return NRX_API_VERSION; }

int nrx_weight_layout(const nrx_desc* desc, int32_t* num_weights, int64_t* sizes, int32_t cap) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if (!num_weights) return fail(NRX_ERR_INVALID_ARG, "num_weights is NULL");
  std::vector<int64_t> s = weight_sizes(desc);
  *num_weights = (int32_t)s.size();
  if (sizes)
    for (int i = 0; i < (int)s.size() && i < cap; ++i) sizes[i] = s[i];
  return NRX_OK;
}

int nrx_create(const nrx_desc* desc, const float* const* weights, const int64_t* sizes,
               int32_t num_weights, int32_t device, nrx_handle** out) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if (!weights || !sizes || !out) return fail(NRX_ERR_INVALID_ARG, "null argument");
  std::vector<int64_t> exp = weight_sizes(desc);
  if ((int)exp.size() != num_weights)
    return fail(NRX_ERR_SHAPE, "expected " + std::to_string(exp.size()) + " weight arrays, got " +
                                   std::to_string(num_weights));
  for (int i = 0; i < num_weights; ++i) {
    if (!weights[i]) return fail(NRX_ERR_INVALID_ARG, "weight " + std::to_string(i) + " is NULL");
    if (sizes[i] != exp[i])
      return fail(NRX_ERR_SHAPE, "weight " + std::to_string(i) + " has " + std::to_string(sizes[i]) +
                                     " elements, expected " + std::to_string(exp[i]));
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  e = setup_kernels();
  if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute");
  nrx_handle* h = new nrx_handle();
  h->desc = *desc;
  h->device = device;
  {
    // A/B and bit-identity tests: 0 = three launches, 1 = default, 2 (or "force") = wherever it
    // applies; anything else is rejected rather than silently read as 0
    const char* ev = getenv("NRX_FUSED");
    if (ev && *ev) {
      if (!strcmp(ev, "0") || !strcmp(ev, "off")) h->fused_enabled = 0;
      else if (!strcmp(ev, "1") || !strcmp(ev, "on")) h->fused_enabled = 1;
      else if (!strcmp(ev, "2") || !strcmp(ev, "force")) h->fused_enabled = 2;
      else {
        delete h;
        return fail(NRX_ERR_INVALID_ARG, std::string("NRX_FUSED must be 0/off, 1/on or 2/force, got '") + ev + "'");
      }
    }
  }
  {
    const char* ev = getenv("NRX_UPDATE_RR");   // A/B: 0 = strip update kernels
    if (ev && *ev) {
      char* end = nullptr;
      const long v = strtol(ev, &end, 10);
      if (end && !*end && ev[0] >= '0' && ev[0] <= '9' && v >= 0 && v <= kSchedMax) h->update_rr = (int)v;
      else {
        delete h;
        return fail(NRX_ERR_INVALID_ARG, std::string("NRX_UPDATE_RR must be a stage mask 0..127, got '") + ev + "'");
      }
    }
  }
  e = hipMalloc(&h->fused_sync, fused_sync_bytes());
  if (e == hipSuccess) e = hipMemset(h->fused_sync, 0, fused_sync_bytes());
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->last_ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    nrx_destroy(h);
    return hip_fail(e, "fused forward counters");
  }
  rc = build_model<_Float16, float>(desc, weights, 32, &h->m16);
  if (!rc) rc = build_model<double, double>(desc, weights, 16, &h->m64);
  if (rc) {
    nrx_destroy(h);
    return rc;
  }
  *out = h;
  return NRX_OK;
}

void nrx_destroy(nrx_handle* h) {
  if (!h) return;
  if (h->m16.dev) (void)hipFree(h->m16.dev);
  if (h->m64.dev) (void)hipFree(h->m64.dev);
  if (h->fused_sync) (void)hipFree(h->fused_sync);
  if (h->last_ev) (void)hipEventDestroy(h->last_ev);
  delete h->prof;
  delete h;
}

static size_t ws_bytes_of(const nrx_shape* s, int precision) {
  return align256((size_t)s->batch * sizeof(double)) + 4 * state_bytes(s, precision) + pe16_bytes(s, precision);
}

// Slots per sub-forward.  An f16 forward whose workspace would reach kGzRange runs as
// consecutive forwards of at most this many slots on the caller's stream (slots are independent,
// neural_rx.py:544-595 has no cross-slot term), each in the same workspace: conv1's z-row loader
// then always addresses it with 32-bit buffer offsets, and the workspace shrinks to one chunk's.
static int chunk_slots(const nrx_shape* s, int precision) {
  if (precision != NRX_PREC_F16 || ws_bytes_of(s, precision) < kGzRange) return s->batch;
  int lo = 1, hi = s->batch - 1;   // the largest chunk below the range (one slot always fits: F <= 3300)
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    nrx_shape c = *s;
    c.batch = mid;
    if (ws_bytes_of(&c, precision) < kGzRange) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

int nrx_workspace_size(const nrx_handle* h, const nrx_shape* shape, int32_t precision, size_t* bytes) {
  if (!h || !bytes) return fail(NRX_ERR_INVALID_ARG, "null argument");
  int rc = check_shape(shape);
  if (rc) return rc;
  if (precision != NRX_PREC_F16 && precision != NRX_PREC_F32X)
    return fail(NRX_ERR_INVALID_ARG, "unknown precision");
  nrx_shape c = *shape;
  c.batch = chunk_slots(shape, precision);
  *bytes = ws_bytes_of(&c, precision);
  return NRX_OK;
}

int nrx_forward(nrx_handle* h, const nrx_io* io, void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !io) return fail(NRX_ERR_INVALID_ARG, "null argument");
  int rc = check_shape(&io->shape);
  if (rc) return rc;
  const nrx_desc* d = &h->desc;
  if (io->num_it < 1 || io->num_it > d->num_it) return fail(NRX_ERR_INVALID_ARG, "Invalid number of iterations");
  if (!io->y || !io->pe || !io->active || !io->llr) return fail(NRX_ERR_INVALID_ARG, "null tensor pointer");
  if (d->use_h_hat && !io->h_hat) return fail(NRX_ERR_INVALID_ARG, "h_hat is required by this model");
  size_t need = 0;
  rc = nrx_workspace_size(h, &io->shape, io->precision, &need);
  if (rc) return rc;
  if (!workspace || workspace_bytes < need)
    return fail(NRX_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  hipStream_t st = (hipStream_t)stream;
  const int bc = chunk_slots(&io->shape, io->precision);
  if (bc < io->shape.batch) {
    // slot chunks (chunk_slots): the same forward on [b0, b0 + n) with offset tensors; the LLR
    // tensor keeps its head stride (llr_B)
    const int B = io->shape.batch, U = io->shape.num_tx, F = io->shape.num_subcarriers, A2 = 2 * d->num_rx_ant;
    const size_t re = (size_t)F * kT;
    for (int b0 = 0; b0 < B; b0 += bc) {
      nrx_io c = *io;
      c.shape.batch = b0 + bc < B ? bc : B - b0;
      c.y = io->y + (size_t)b0 * re * A2;
      c.h_hat = io->h_hat ? io->h_hat + (size_t)b0 * U * re * A2 : nullptr;
      c.active = io->active + (size_t)b0 * U;
      c.mcs_mask = io->mcs_mask ? io->mcs_mask + (size_t)b0 * U * d->num_mcs : nullptr;
      c.h_ref = io->h_ref ? io->h_ref + (size_t)b0 * U * re * A2 : nullptr;
      c.llr = io->llr + (size_t)b0 * U * re * bits_max(d);
      rc = forward_slots(h, &c, B, workspace, st);
      if (rc) return rc;
    }
    return NRX_OK;
  }
  return forward_slots(h, io, io->shape.batch, workspace, st);
}

// One forward over io->shape.batch slots of an LLR tensor of llr_B slots (its head stride).
static int forward_slots(nrx_handle* h, const nrx_io* io, int llr_B, void* workspace, hipStream_t st) {
  hipError_t e;
  if (io->precision == NRX_PREC_F16) {
    FwdArgs<_Float16, float, _Float16> a{};
    fill_args(a, h, io, workspace, h->m16.init_cinp);
    a.llr_B = llr_B;
    const FusedCtl fc = h->fused_ctl();
    const bool takes = fused_would_run(a, io->num_it, fc);
    if (takes && h->have_last && h->last_stream != st && hipEventQuery(h->last_ev) == hipErrorNotReady)
      return fail(NRX_ERR_BUSY, "a one-launch forward of this handle is still running on another stream");
    e = launch_forward_f16(a, h->m16.W, io->num_it, st, h->prof, fc);
    if (e == hipSuccess && takes) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
        e = hipEventRecord(h->last_ev, st);
        h->last_stream = st;
        h->have_last = e == hipSuccess;
      }
    }
  } else {
    FwdArgs<double, double, float> a{};
    fill_args(a, h, io, workspace, h->m64.init_cinp);
    a.llr_B = llr_B;
    e = launch_forward_f64(a, h->m64.W, io->num_it, st, h->prof);
  }
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  return NRX_OK;
}

static size_t y_cgnn_bytes(const nrx_handle* h, const nrx_shape* s) {
  return align256((size_t)s->batch * s->num_subcarriers * s->num_symbols * 2 * h->desc.num_rx_ant * sizeof(float));
}

int nrx_workspace_size_ex(const nrx_handle* h, const nrx_shape* shape, int32_t precision, int32_t y_layout,
                          size_t* bytes) {
  int rc = nrx_workspace_size(h, shape, precision, bytes);
  if (rc) return rc;
  if (y_layout < NRX_Y_CGNN || y_layout > NRX_Y_SPLIT) return fail(NRX_ERR_INVALID_ARG, "unknown y layout");
  if (y_layout != NRX_Y_CGNN) *bytes += y_cgnn_bytes(h, shape);
  return NRX_OK;
}

int nrx_forward_ex(nrx_handle* h, const nrx_io* io, int32_t y_layout, const float* y_imag, void* workspace,
                   size_t workspace_bytes, void* stream) {
  if (!h || !io) return fail(NRX_ERR_INVALID_ARG, "null argument");
  if (y_layout == NRX_Y_CGNN) {
    if (y_imag) return fail(NRX_ERR_INVALID_ARG, "y_imag is only used with NRX_Y_SPLIT");
    return nrx_forward(h, io, workspace, workspace_bytes, stream);
  }
  size_t need = 0;
  int rc = nrx_workspace_size_ex(h, &io->shape, io->precision, y_layout, &need);
  if (rc) return rc;
  if (!workspace || workspace_bytes < need)
    return fail(NRX_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  if (!io->y || ((y_layout == NRX_Y_SPLIT) != (y_imag != nullptr)))
    return fail(NRX_ERR_INVALID_ARG, "y / y_imag do not match the y layout");
  bool takes = false;
  if ((rc = fused_busy(h, io, (hipStream_t)stream, &takes))) return rc;
  const size_t yb = y_cgnn_bytes(h, &io->shape);
  float* ycg = (float*)workspace;
  hipError_t e = launch_y_layout(io->y, y_imag, y_layout, io->shape.batch, io->shape.num_subcarriers,
                                 io->shape.num_symbols, h->desc.num_rx_ant, ycg, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "y layout launch");
  nrx_io cio = *io;
  cio.y = ycg;
  return nrx_forward(h, &cio, (char*)workspace + yb, workspace_bytes - yb, stream);
}

// ---------------------------------------------------------------- Aerial contract
namespace {
struct AerialWs {
  float* y;
  float* h;
  float* pe;
  int32_t* nn;
  float* llr;
  void* cgnn;
  size_t cgnn_bytes;
  size_t total;
};

AerialWs aerial_layout(const nrx_handle* h, const nrx_aerial_io* io, void* base, size_t cgnn_bytes) {
  const nrx_shape& s = io->shape;
  const size_t A2 = 2 * (size_t)h->desc.num_rx_ant;
  const size_t re = (size_t)s.num_subcarriers * s.num_symbols;
  AerialWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align256(bytes);
    return (char*)base + o;
  };
  w.y = (float*)take((size_t)s.batch * re * A2 * 4);
  w.h = (float*)take((size_t)s.batch * s.num_tx * re * A2 * 4);
  w.pe = (float*)take((size_t)s.num_tx * re * 2 * 4);
  w.nn = (int32_t*)take((size_t)s.num_tx * s.num_symbols * 12 * 4);
  w.llr = (float*)take((size_t)num_heads(&h->desc) * s.batch * s.num_tx * re * bits_max(&h->desc) * 4);
  w.cgnn = take(cgnn_bytes);
  w.cgnn_bytes = cgnn_bytes;
  w.total = off;
  return w;
}

int check_aerial(const nrx_handle* h, const nrx_aerial_io* io) {
  if (!h || !io) return fail(NRX_ERR_INVALID_ARG, "null argument");
  int rc = check_shape(&io->shape);
  if (rc) return rc;
  if (io->shape.num_subcarriers % 12) return fail(NRX_ERR_SHAPE, "num_subcarriers must be a multiple of 12 (PRBs)");
  if (io->num_dmrs_symbols < 1 || io->num_dmrs_symbols > 14)
    return fail(NRX_ERR_SHAPE, "num_dmrs_symbols must be 1..14");
  if (io->num_dmrs_subcarriers < 2 || io->num_dmrs_subcarriers > 12 || io->num_dmrs_subcarriers % 2)
    return fail(NRX_ERR_SHAPE, "num_dmrs_subcarriers must be even and 2..12 (FOCC pairs)");
  return NRX_OK;
}
}  // namespace

int nrx_aerial_workspace_size(const nrx_handle* h, const nrx_aerial_io* io, size_t* bytes) {
  int rc = check_aerial(h, io);
  if (rc) return rc;
  if (!bytes) return fail(NRX_ERR_INVALID_ARG, "null argument");
  size_t cg = 0;
  rc = nrx_workspace_size(h, &io->shape, io->precision, &cg);
  if (rc) return rc;
  *bytes = aerial_layout(h, io, nullptr, cg).total;
  return NRX_OK;
}

int nrx_forward_aerial(nrx_handle* h, const nrx_aerial_io* io, void* workspace, size_t workspace_bytes,
                       void* stream) {
  int rc = check_aerial(h, io);
  if (rc) return rc;
  if (!io->y_real || !io->y_imag || !io->h_ls_real || !io->h_ls_imag || !io->dmrs_port_mask ||
      !io->dmrs_ofdm_pos || !io->dmrs_subcarrier_pos || !io->llr)
    return fail(NRX_ERR_INVALID_ARG, "null tensor pointer");
  size_t cg = 0;
  rc = nrx_workspace_size(h, &io->shape, io->precision, &cg);
  if (rc) return rc;
  const AerialWs w = aerial_layout(h, io, workspace, cg);
  if (!workspace || workspace_bytes < w.total)
    return fail(NRX_ERR_WORKSPACE, "workspace too small: need " + std::to_string(w.total) + " bytes");
  const nrx_shape& s = io->shape;
  const int A = h->desc.num_rx_ant;
  hipStream_t st = (hipStream_t)stream;
  {
    nrx_io q{};
    q.shape = s;
    q.num_it = io->num_it;
    q.precision = io->precision;
    bool takes = false;
    if ((rc = fused_busy(h, &q, st, &takes))) return rc;
  }
  hipError_t e = launch_aerial_tables(io->dmrs_ofdm_pos, io->dmrs_subcarrier_pos, s.num_tx, io->num_dmrs_symbols,
                                      io->num_dmrs_subcarriers, s.num_symbols, s.num_subcarriers, w.nn, w.pe, st);
  if (e == hipSuccess)
    e = launch_aerial_inputs(io->y_real, io->y_imag, io->h_ls_real, io->h_ls_imag, w.nn, s.batch, s.num_tx,
                             s.num_subcarriers, s.num_symbols, A, io->num_dmrs_symbols, io->num_dmrs_subcarriers,
                             w.y, w.h, st);
  if (e != hipSuccess) return hip_fail(e, "aerial preprocessing launch");
  nrx_io cio{};
  cio.shape = s;
  cio.num_it = io->num_it;
  cio.precision = io->precision;
  cio.y = w.y;
  cio.pe = w.pe;
  cio.h_hat = w.h;
  cio.active = io->dmrs_port_mask;
  cio.mcs_mask = nullptr;
  cio.llr = w.llr;
  cio.h_ref = io->h_hat;
  rc = nrx_forward(h, &cio, w.cgnn, w.cgnn_bytes, stream);
  if (rc) return rc;
  const int bits0 = h->desc.var_mcs_masking ? bits_max(&h->desc) : h->desc.bits[0];
  e = launch_aerial_llr(w.llr, s.batch, s.num_tx, s.num_subcarriers, s.num_symbols, bits_max(&h->desc), bits0,
                        io->llr, st);
  if (e != hipSuccess) return hip_fail(e, "aerial LLR layout launch");
  return NRX_OK;
}

int nrx_llr_demap(const float* llr, int32_t batch, int32_t num_tx, int32_t num_subcarriers, int32_t num_symbols,
                  int32_t bits_stride, int32_t bits, const int32_t* data_re, int32_t n_data, float* out,
                  void* stream) {
  if (!llr || !data_re || !out) return fail(NRX_ERR_INVALID_ARG, "null tensor pointer");
  if (batch < 1 || num_tx < 1 || num_subcarriers < 1 || num_symbols < 1 || bits < 1 || bits > bits_stride ||
      n_data < 1 || n_data > num_subcarriers * num_symbols)
    return fail(NRX_ERR_SHAPE, "inconsistent demap shape");
  hipError_t e = launch_llr_demap(llr, batch, num_tx, num_subcarriers, num_symbols, bits_stride, bits, data_re,
                                  n_data, out, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "llr demap launch");
  return NRX_OK;
}

static int check_gen(const nrx_gen_desc* d) {
  if (!d) return fail(NRX_ERR_INVALID_ARG, "desc is NULL");
  if (d->batch < 1 || d->batch > 65535) return fail(NRX_ERR_SHAPE, "batch must be 1..65535");
  if (d->num_tx < 1 || d->num_tx > kMaxUsers) return fail(NRX_ERR_SHAPE, "num_tx must be 1..16");
  if (d->num_symbols != kT) return fail(NRX_ERR_SHAPE, "num_symbols must be 14");
  if (d->num_subcarriers < 2 || d->num_subcarriers > 3300) return fail(NRX_ERR_SHAPE, "num_subcarriers must be 2..3300");
  if (d->num_rx_ant < 1 || d->num_rx_ant > 16) return fail(NRX_ERR_SHAPE, "num_rx_ant must be 1..16");
  if (d->num_dmrs_symbols < 1 || d->num_dmrs_symbols > 4) return fail(NRX_ERR_SHAPE, "num_dmrs_symbols must be 1..4");
  int mask = 0;
  for (int k = 0; k < d->num_dmrs_symbols; ++k) {
    const int t = d->dmrs_symbols[k];
    if (t < 0 || t >= kT || (k && t <= d->dmrs_symbols[k - 1]))
      return fail(NRX_ERR_INVALID_ARG, "dmrs_symbols must be ascending symbol indices");
    mask |= 1 << t;
  }
  if (mask != d->dmrs_symbol_mask) return fail(NRX_ERR_INVALID_ARG, "dmrs_symbol_mask does not match dmrs_symbols");
  if (d->num_mcs < 1 || d->num_mcs > 8) return fail(NRX_ERR_INVALID_ARG, "num_mcs must be 1..8");
  for (int m = 0; m < d->num_mcs; ++m)
    if (d->mcs_bits[m] != 2 && d->mcs_bits[m] != 4 && d->mcs_bits[m] != 6)
      return fail(NRX_ERR_INVALID_ARG, "mcs_bits must be 2, 4 or 6");
  for (int u = 0; u < d->num_tx; ++u) {
    if (d->cdm_group[u] != 0 && d->cdm_group[u] != 1) return fail(NRX_ERR_INVALID_ARG, "cdm_group must be 0/1");
    if (d->mcs_of_user[u] < -1 || d->mcs_of_user[u] >= d->num_mcs)
      return fail(NRX_ERR_INVALID_ARG, "mcs_of_user must be -1..num_mcs-1");
  }
  if (d->num_active < 1 || d->num_active > d->num_tx) return fail(NRX_ERR_INVALID_ARG, "num_active must be 1..num_tx");
  if (d->num_taps < 1 || d->num_taps > 8) return fail(NRX_ERR_INVALID_ARG, "num_taps must be 1..8");
  if (d->num_sinusoids < 1 || d->num_sinusoids > 16) return fail(NRX_ERR_INVALID_ARG, "num_sinusoids must be 1..16");
  if (!(d->max_delay_s >= 0.0) || !(d->max_doppler_hz >= 0.0) || !(d->subcarrier_spacing > 0.0) || !(d->no >= 0.0))
    return fail(NRX_ERR_INVALID_ARG, "channel parameters must be finite and non-negative (scs > 0)");
  if (d->slot_offset < 0) return fail(NRX_ERR_INVALID_ARG, "slot_offset must be >= 0");
  return NRX_OK;
}

int nrx_gen_workspace_size(const nrx_gen_desc* desc, size_t* bytes) {
  if (int rc = check_gen(desc)) return rc;
  if (!bytes) return fail(NRX_ERR_INVALID_ARG, "bytes is NULL");
  *bytes = gen_workspace_bytes(*desc, nullptr, nullptr);
  return NRX_OK;
}

int nrx_generate_slots(const nrx_gen_desc* desc, const nrx_gen_out* out, void* workspace, size_t workspace_bytes,
                       void* stream) {
  if (int rc = check_gen(desc)) return rc;
  if (!out || !out->y || !workspace) return fail(NRX_ERR_INVALID_ARG, "null tensor pointer");
  int bmax = 0;
  for (int m = 0; m < desc->num_mcs; ++m) bmax = desc->mcs_bits[m] > bmax ? desc->mcs_bits[m] : bmax;
  if (out->bits && out->bits_stride < bmax) return fail(NRX_ERR_SHAPE, "bits_stride < max(mcs_bits)");
  if ((out->y_real == nullptr) != (out->y_imag == nullptr) || (out->h_ls_real == nullptr) != (out->h_ls_imag == nullptr))
    return fail(NRX_ERR_INVALID_ARG, "Aerial outputs come in (real, imag) pairs");
  if (out->h_ls_real && desc->num_subcarriers % 12)
    return fail(NRX_ERR_SHAPE, "Aerial pilot list needs num_subcarriers % 12 == 0");
  const size_t need = gen_workspace_bytes(*desc, nullptr, nullptr);
  if (workspace_bytes < need)
    return fail(NRX_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  hipError_t e = launch_generate(*desc, *out, workspace, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "slot generator launch");
  return NRX_OK;
}

int nrx_count_errors(const nrx_count_io* io, void* stream) {
  if (!io) return fail(NRX_ERR_INVALID_ARG, "null argument");
  if (!io->llr || !io->bits || !io->active || !io->counts) return fail(NRX_ERR_INVALID_ARG, "null tensor pointer");
  if (io->batch < 1 || io->num_tx < 1 || io->num_subcarriers < 1 || io->num_symbols < 1 || io->num_symbols > 31 ||
      io->num_heads < 1 || io->num_mcs < 1 || io->num_mcs > 8 || (io->num_heads > 1 && io->num_heads != io->num_mcs))
    return fail(NRX_ERR_SHAPE, "inconsistent counter shape");
  for (int m = 0; m < io->num_mcs; ++m)
    if (io->mcs_bits[m] < 1 || io->mcs_bits[m] > io->bits_stride)
      return fail(NRX_ERR_SHAPE, "mcs_bits must be 1..bits_stride");
  hipError_t e = launch_count_errors(*io, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "error counter launch");
  return NRX_OK;
}

int nrx_profile_enable(nrx_handle* h, int32_t enable) {
  if (!h) return fail(NRX_ERR_INVALID_ARG, "null handle");
  if (enable) {
    if (!h->prof) h->prof = new EventProf();
    hipError_t e = h->prof->collect();
    h->prof->reset();
    if (e != hipSuccess) return hip_fail(e, "profile reset");
  } else {
    delete h->prof;
    h->prof = nullptr;
  }
  return NRX_OK;
}

int nrx_fused_status(nrx_handle* h, int32_t* status, int32_t reset) {
  if (!h || !status) return fail(NRX_ERR_INVALID_ARG, "null argument");
  int st[3] = {0, 0, 0};
  hipError_t e = fused_sync_status(h->fused_sync, st, reset != 0, h->have_last ? h->last_ev : nullptr);
  if (e != hipSuccess) return hip_fail(e, "fused status");
  for (int i = 0; i < 3; ++i) status[i] = st[i];
  if (st[0])
    return fail(NRX_ERR_FUSED, "one-launch forward error bits " + std::to_string(st[0]) +
                                   " (1: dependency wait timed out, 2: items left undone): outputs invalid");
  return NRX_OK;
}

int nrx_fused_config(nrx_handle* h, int32_t enable, int32_t spin_limit, int32_t inject_err) {
  if (!h) return fail(NRX_ERR_INVALID_ARG, "null argument");
  // every argument < 0 leaves its setting unchanged; spin_limit == 0 restores the
  // default bound
  if (enable > 2) return fail(NRX_ERR_INVALID_ARG, "enable must be 0 (off), 1 (default) or 2 (force)");
  if (enable >= 0) h->fused_enabled = enable;
  if (spin_limit >= 0) h->spin_limit = spin_limit > 0 ? spin_limit : kFusedSpinLimit;
  if (inject_err >= 0) h->dbg_err = inject_err;
  return NRX_OK;
}

int nrx_update_schedule(nrx_handle* h, int32_t update_rr) {
  if (!h) return fail(NRX_ERR_INVALID_ARG, "null argument");
  if (update_rr > kSchedMax) return fail(NRX_ERR_INVALID_ARG, "update_rr is a stage mask 0..127");
  if (update_rr >= 0) h->update_rr = update_rr;
  return NRX_OK;
}

int nrx_profile_read(nrx_handle* h, int32_t kernel, int64_t* launches, double* total_ms) {
  if (!h || !launches || !total_ms) return fail(NRX_ERR_INVALID_ARG, "null argument");
  if (kernel < 0 || kernel >= K_COUNT) return fail(NRX_ERR_INVALID_ARG, "bad kernel id");
  if (!h->prof) return fail(NRX_ERR_INVALID_ARG, "profiling is not enabled");
  hipError_t e = h->prof->collect();
  if (e != hipSuccess) return hip_fail(e, "profile collect");
  *launches = h->prof->launches[kernel];
  *total_ms = h->prof->total_ms[kernel];
  return NRX_OK;
}

// Product-side restatement of the nearest-pilot positional encoding
// (onnx_utils.py:206-260).  Pilots of CDM group g (DMRS config type 1)
// occupy subcarriers f with f % 2 == g on the DMRS symbols.
int nrx_compute_pe(int32_t num_tx, int32_t F, int32_t T, const int32_t* dmrs_symbols, int32_t nsym,
                   const int32_t* cdm_group, float* pe) {
  if (num_tx < 1 || F < 1 || T < 1 || !dmrs_symbols || nsym < 1 || !cdm_group || !pe)
    return fail(NRX_ERR_INVALID_ARG, "bad argument");
  std::vector<double> dt(T), df(F);
  for (int u = 0; u < num_tx; ++u) {
    if (cdm_group[u] != 0 && cdm_group[u] != 1) return fail(NRX_ERR_INVALID_ARG, "cdm_group must be 0/1");
    bool any_f = false;
    for (int t = 0; t < T; ++t) {
      int best = 1 << 30;
      for (int k = 0; k < nsym; ++k) best = std::min(best, std::abs(dmrs_symbols[k] - t));
      dt[t] = best;
    }
    for (int f = 0; f < F; ++f) {
      int best = 1 << 30;
      for (int p = cdm_group[u]; p < F; p += 2) {
        best = std::min(best, std::abs(p - f));
        any_f = true;
      }
      df[f] = best;
    }
    if (!any_f) return fail(NRX_ERR_INVALID_ARG, "user has no pilots");
    // normalise: time over the symbol axis, frequency over the subcarrier axis;
    // population std, left unscaled where std == 0
    auto norm = [](std::vector<double>& v) {
      double m = 0;
      for (double x : v) m += x;
      m /= v.size();
      double s2 = 0;
      for (double& x : v) {
        x -= m;
        s2 += x * x;
      }
      const double sd = std::sqrt(s2 / v.size());
      if (sd > 0)
        for (double& x : v) x /= sd;
    };
    norm(dt);
    norm(df);
    for (int f = 0; f < F; ++f)
      for (int t = 0; t < T; ++t) {
        pe[(((size_t)u * F + f) * T + t) * 2 + 0] = (float)dt[t];
        pe[(((size_t)u * F + f) * T + t) * 2 + 1] = (float)df[f];
      }
  }
  return NRX_OK;
}

double nrx_flops_per_re_user(const nrx_desc* d, int32_t num_it) {
  if (check_desc(d)) return 0.0;
  auto sep = [](double ci, double co) { return 9 * ci + ci * co; };
  const double init = sep(init_cin(d), kHID) + sep(kHID, kHID) + sep(kHID, kDS);
  const double it = kDS * kAGG + kAGG * kDS + sep(2 * kDS + 2, kHID) + sep(kHID, kHID) + sep(kHID, kDS);
  double heads = 0;
  for (int h = 0; h < num_heads(d); ++h)
    heads += kDS * kHID + kHID * (d->var_mcs_masking ? bits_max(d) : d->bits[h]);
  const double ch = kDS * kHID + kHID * 2.0 * d->num_rx_ant;
  return 2.0 * (init * num_init(d) + num_it * it + heads + ch);
}

}  // extern "C"
