/*
 * nrx.h -- C ABI of the MI355X CGNN neural-receiver engine (libnrx.so).
 *
 * Plain C, plain pointers and sizes: no torch, no HIP types in the signatures
 * (streams are passed as `void*` = hipStream_t).  Every entry point returns an int
 * status (NRX_OK = 0, negative on error) and never throws; the last error message of
 * the calling thread is available from nrx_last_error().
 *
 * The reference has no FFI for this path: its hot path is a Python layer call,
 *   CGNN.forward([y, pe, h_hat, active_tx, mcs_ue_mask]) -> (llrs, h_hats)
 *       (utils/neural_rx.py:544-595; faithful TF structure in
 *        utils/neural_rx copy_pytorch.py:474-514),
 * wrapped by CGNNOFDM.forward (neural_rx.py:813-881) and
 * NeuralReceiverONNX.forward (neural_rx.py:1773-1812).  The entry points below are
 * what a binding of that call needs; INTEGRATION.md shows the
 * ctypes binding the Python layer uses.
 *
 * Layouts (all channels-last, as the reference's NHWC tensors):
 *   y        [B][F][T][2A]          f32  channels [Re a0..a(A-1), Im a0..a(A-1)]
 *   pe       [U][F][T][2]           f32  [time, freq] nearest-pilot encoding
 *   h_hat    [B][U][F][T][2A]       f32  initial channel estimate (NULL if unused)
 *   active   [B][U]                 f32  1 = DMRS port active
 *   mcs_mask [B][U][M]              f32  Var-IO state-init mixing weights (NULL: one-hot m=0)
 *   llr      [H][B][U][F][T][bits_max] f32 out, H = number of LLR heads
 *                                   (M for Var-IO, 1 otherwise); head h fills its
 *                                   first bits_h entries, the rest are written 0
 *   h_ref    [B][U][F][T][2A]       f32 out (NULL to skip the ChEst readout)
 * Sign convention: Sionna's LLR = log p(b=1)/p(b=0) (the Aerial layout negates,
 * neural_rx.py:1811; the Python layer does that, not the kernels).
 */
#ifndef NRX_H_
#define NRX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NRX_API_VERSION 7

enum nrx_status {
  NRX_OK = 0,
  NRX_ERR_INVALID_ARG = -1,   /* null pointer / bad enum / bad num_it */
  NRX_ERR_SHAPE = -2,         /* shape inconsistent with the model or limits */
  NRX_ERR_UNSUPPORTED = -3,   /* topology the kernels are not built for */
  NRX_ERR_HIP = -4,           /* HIP runtime error (message has the HIP string) */
  NRX_ERR_NOMEM = -5,
  NRX_ERR_WORKSPACE = -6,     /* workspace too small */
  NRX_ERR_BUSY = -7,          /* a forward of this handle is still running on another stream */
  NRX_ERR_FUSED = -8          /* an earlier one-launch forward reported an error: its outputs
                               * are invalid (see nrx_fused_status) */
};

/* Arithmetic of a forward pass. */
enum nrx_precision {
  NRX_PREC_F16 = 0,    /* perf mode: f16 activations, f16 depthwise, f16 MFMA with f32
                          accumulation (the reference's own TRT export ran --fp16) */
  NRX_PREC_F32X = 1    /* parity mode: f32 activations, f64 arithmetic (f64 MFMA) */
};

/* Model topology.  Mirrors the [neural_receiver] block of the reference cfg
 * (config/nrx_rt.cfg:57-75) plus [system] num_rx_antennas / mcs_index. */
typedef struct nrx_desc {
  int32_t num_rx_ant;        /* A (4 or 16) */
  int32_t d_s;               /* state width; kernels are built for 56 */
  int32_t num_it;            /* trained CGNN iterations (len(iterations)) */
  int32_t num_mcs;           /* M = len(mcs_index), 1..8 */
  int32_t bits[8];           /* bits per symbol of each MCS (2, 4 or 6) */
  int32_t var_mcs_masking;   /* 1: one StateInit + one LLR head of max(bits), sliced */
  int32_t init_units[2];     /* num_units_init, kernels built for {128,128} */
  int32_t agg_units;         /* num_units_agg[i] = [64] */
  int32_t state_units[2];    /* num_units_state[i] = [128,128] */
  int32_t readout_units;     /* num_units_readout = [128] */
  int32_t use_h_hat;         /* 1: StateInit consumes h_hat (initial_chest = "ls") */
} nrx_desc;

typedef struct nrx_shape {
  int32_t batch;             /* B slots */
  int32_t num_tx;            /* U users (DMRS ports) */
  int32_t num_subcarriers;   /* F = 12 * PRBs */
  int32_t num_symbols;       /* T, must be 14 */
} nrx_shape;

typedef struct nrx_io {
  nrx_shape shape;
  int32_t num_it;            /* iterations to run, 1..desc.num_it (CGNN.num_it setter) */
  int32_t precision;         /* enum nrx_precision */
  const float* y;
  const float* pe;
  const float* h_hat;        /* may be NULL only if desc.use_h_hat == 0 */
  const float* active;
  const float* mcs_mask;     /* may be NULL: treated as one-hot on MCS 0 */
  float* llr;
  float* h_ref;              /* may be NULL */
} nrx_io;

typedef struct nrx_handle nrx_handle;

/* Create an engine on `device` from weights in Keras get_weights() order
 * (the reference loads the same list with
 * utils/utils.py:53-70 load_weights).  `weight_sizes[i]` is the element count of
 * weights[i] and is validated against the topology.  Weights are host pointers;
 * they are copied, converted and packed into device buffers. */
int nrx_create(const nrx_desc* desc, const float* const* weights, const int64_t* weight_sizes,
               int32_t num_weights, int32_t device, nrx_handle** out);

/* Number of weight arrays and the element count of array i for a topology. */
int nrx_weight_layout(const nrx_desc* desc, int32_t* num_weights, int64_t* sizes, int32_t cap);

/* Device workspace (bytes) a forward of this shape/precision needs. */
int nrx_workspace_size(const nrx_handle* h, const nrx_shape* shape, int32_t precision,
                       size_t* bytes);

/* Asynchronous forward on `stream` (hipStream_t; NULL = default stream).
 * All pointers in `io` and `workspace` are device pointers.  No allocation, no host
 * synchronisation: the call can be captured into a hipGraph. */
int nrx_forward(nrx_handle* h, const nrx_io* io, void* workspace, size_t workspace_bytes,
                void* stream);

void nrx_destroy(nrx_handle* h);

/* Input layouts of y for nrx_forward_ex (the wrappers' own input tensors, so that a
 * wrapper call launches only libnrx kernels: no host-framework transpose/concat). */
enum nrx_y_layout {
  NRX_Y_CGNN = 0,       /* io->y [B][F][T][2A] f32, as nrx_forward */
  NRX_Y_SIONNA_RG = 1,  /* io->y = the resource grid [B][1][A][T][F] complex64 (re, im
                           interleaved floats), as CGNNOFDM.forward receives it
                           (neural_rx.py:813-833: y[:,0].permute(0,3,2,1), cat(real, imag)) */
  NRX_Y_SPLIT = 2       /* io->y = rx_slot_real [B][F][T][A], y_imag = rx_slot_imag, as
                           NeuralReceiverONNX.forward (neural_rx.py:1787) */
};

/* Workspace of nrx_forward_ex: nrx_workspace_size plus the CGNN-layout copy of y. */
int nrx_workspace_size_ex(const nrx_handle* h, const nrx_shape* shape, int32_t precision, int32_t y_layout,
                          size_t* bytes);

/* nrx_forward with y in one of the layouts above (y_imag: NRX_Y_SPLIT only, else NULL).
 * The other tensors of `io` keep their nrx_forward layouts. */
int nrx_forward_ex(nrx_handle* h, const nrx_io* io, int32_t y_layout, const float* y_imag, void* workspace,
                   size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- Aerial contract
 * The NeuralReceiverONNX / TensorRT engine I/O (neural_rx.py:1773-1812; feed dict of
 * notebooks/real_time_nrx.ipynb:792-844): LS channel estimates at the DMRS pilots in, the
 * FOCC removal + per-PRB nearest-pilot interpolation + positional encoding
 * (NRPreprocessing, neural_rx.py:1614-1711) run on the GPU, LLRs out in the Aerial layout
 * and sign.  Single MCS, as the ONNX export (LLR head 0, mcs mask one-hot on MCS 0).
 *   y_real, y_imag        [B][F][T][A]            f32   rx_slot_{real,imag}
 *   h_ls_real, h_ls_imag  [B][Npil][U][A]         f32   LS estimates at the pilots,
 *                          Npil = nsym * (F/12) * npil, pilot p = (k * F/12 + prb) * npil + j
 *                          (DMRS symbol k, PRB, pilot j of the PRB); FOCC pairs p, p^1
 *   dmrs_port_mask        [B][U]                  f32   active DMRS ports
 *   dmrs_ofdm_pos         [U][nsym]               i32   DMRS symbol indices (device)
 *   dmrs_subcarrier_pos   [U][npil]               i32   pilot subcarriers within a PRB (device)
 *   llr                   [B][bits][U][F][T]      f32   out, LLR = log p(b=0)/p(b=1)
 *   h_hat                 [B][U][F][T][2A]        f32   out, refined estimate (NULL: skip)
 */
typedef struct nrx_aerial_io {
  nrx_shape shape;           /* B, U = num_tx, F (multiple of 12), T = 14 */
  int32_t num_it;
  int32_t precision;
  int32_t num_dmrs_symbols;  /* nsym */
  int32_t num_dmrs_subcarriers; /* npil (even; 6 for DMRS type 1) */
  const float* y_real;
  const float* y_imag;
  const float* h_ls_real;
  const float* h_ls_imag;
  const float* dmrs_port_mask;
  const int32_t* dmrs_ofdm_pos;
  const int32_t* dmrs_subcarrier_pos;
  float* llr;
  float* h_hat;
} nrx_aerial_io;

/* Workspace of nrx_forward_aerial (the CGNN workspace plus the preprocessed y, h_hat, pe,
 * NN table and the Sionna-layout LLRs). */
int nrx_aerial_workspace_size(const nrx_handle* h, const nrx_aerial_io* io, size_t* bytes);

/* Asynchronous Aerial-contract forward on `stream`; device pointers, no allocation, no
 * host synchronisation. */
int nrx_forward_aerial(nrx_handle* h, const nrx_aerial_io* io, void* workspace, size_t workspace_bytes,
                       void* stream);

/* Coded-bit layout of one LLR head (Sionna sign): out[B][U][n_data * bits] with
 * out[b][u][i * bits + k] = llr[b][u][f][t][k] for the i-th data RE, data_re[i] = t * F + f
 * in resource-grid order (symbol-major) -- the ResourceGridDemapper + flatten of
 * CGNNOFDM.forward (neural_rx.py:843-852) and DataEvaluator.post_process_llrs
 * (onnx_utils.py:473-516).  `llr` points at head h of the nrx_forward output
 * ([B][U][F][T][bits_stride]); data_re is a device array.  Asynchronous on `stream`. */
int nrx_llr_demap(const float* llr, int32_t batch, int32_t num_tx, int32_t num_subcarriers,
                  int32_t num_symbols, int32_t bits_stride, int32_t bits, const int32_t* data_re,
                  int32_t n_data, float* out, void* stream);

/* ---------------------------------------------------------------- slot generator
 * Seeded synthetic PUSCH slots generated on the GPU -- replaces the
 * transmitter + channel + LS-estimator chain of E2E_Model.forward (utils/e2e_model.py:
 * 219-344: random active DMRS ports 187-193, x *= active 311-313, Eb/N0 -> no 323-332)
 * for evaluation loops that never leave the device.  The algorithm (Philox4x32-10 draws
 * keyed by seed and counted by the global slot index slot_offset + b, Gray QAM / DMRS type
 * 1 QPSK x sqrt(2), tapped-delay-line channel with exponential PDP and sum-of-sinusoids
 * Doppler, AWGN, LS at the nearest own pilot) is stated in oracle/synth_ref.py. */
typedef struct nrx_gen_desc {
  int32_t batch;               /* B slots in this call */
  int32_t num_tx;              /* U DMRS ports, 1..16 */
  int32_t num_subcarriers;     /* F */
  int32_t num_symbols;         /* T, must be 14 */
  int32_t num_rx_ant;          /* A, 1..16 */
  int32_t num_dmrs_symbols;    /* 1..4 */
  int32_t dmrs_symbols[4];     /* ascending */
  int32_t dmrs_symbol_mask;    /* bit t set <=> t is a DMRS symbol (no data) */
  int32_t cdm_group[16];       /* per port, 0/1 (DMRS type 1: even / odd subcarriers) */
  int32_t num_mcs;             /* M, 1..8 */
  int32_t mcs_bits[8];         /* bits per symbol of each MCS: 2, 4 or 6 */
  int32_t mcs_of_user[16];     /* MCS index per port, -1 = drawn per slot */
  int32_t num_active;          /* active ports per slot (1..U), placed at random */
  int32_t num_taps;            /* TDL taps, 1..8 */
  int32_t num_sinusoids;       /* Doppler sinusoids per tap, 1..16 */
  int32_t pad_;
  double max_delay_s;
  double max_doppler_hz;
  double subcarrier_spacing;   /* Hz */
  double no;                   /* noise variance per RE (complex) */
  uint64_t seed;
  int64_t slot_offset;         /* global index of slot 0 of this call */
} nrx_gen_desc;

/* Device outputs; any pointer except y may be NULL. */
typedef struct nrx_gen_out {
  float* y;                    /* [B][F][T][2A] (nrx_io.y layout) */
  float* h_hat;                /* [B][U][F][T][2A] LS + nearest-neighbour */
  float* h;                    /* [B][U][F][T][2A] true channel */
  float* active;               /* [B][U] */
  float* mcs_mask;             /* [B][U][M] one-hot (nrx_io.mcs_mask) */
  uint8_t* mcs;                /* [B][U] MCS index */
  uint8_t* bits;               /* [B][U][F][T][bits_stride], 0 on DMRS REs and k >= bits */
  int32_t bits_stride;         /* >= max(mcs_bits) */
  int32_t pad_;
  float* y_real;               /* [B][F][T][A] Aerial rx_slot_real */
  float* y_imag;
  float* h_ls_real;            /* [B][Npil][U][A] Aerial LS pilots (nrx_aerial_io), needs F % 12 == 0 */
  float* h_ls_imag;
} nrx_gen_out;

int nrx_gen_workspace_size(const nrx_gen_desc* desc, size_t* bytes);
int nrx_generate_slots(const nrx_gen_desc* desc, const nrx_gen_out* out, void* workspace,
                       size_t workspace_bytes, void* stream);

/* Uncoded error counters of one batch (sim_ber's counting, scripts/evaluate.py:193-202,
 * with the active-port masking of E2E_Model._mask_active_dmrs, e2e_model.py:195-209):
 * counts[u][0..3] += (bit errors, bits, block errors, blocks) over the active (slot, user)
 * pairs, data REs and the first mcs_bits[mcs[b][u]] bits; hard decision LLR > 0 -> 1; a
 * block is one (slot, user) grid.  Asynchronous on `stream`. */
typedef struct nrx_count_io {
  int32_t batch, num_tx, num_subcarriers, num_symbols;
  int32_t num_heads;           /* H heads in llr; head = mcs if H > 1 else 0 */
  int32_t bits_stride;         /* last dim of llr and bits */
  int32_t num_mcs;
  int32_t mcs_bits[8];
  int32_t dmrs_symbol_mask;
  const float* llr;            /* [H][B][U][F][T][bits_stride] (nrx_io.llr) */
  const uint8_t* bits;         /* [B][U][F][T][bits_stride] */
  const uint8_t* mcs;          /* [B][U] or NULL (= 0) */
  const float* active;         /* [B][U] */
  int64_t* counts;             /* [U][4] accumulated (device) */
} nrx_count_io;

int nrx_count_errors(const nrx_count_io* io, void* stream);

/* Host helper: nearest-pilot positional encoding pe[U][F][T][2] for DMRS
 * configuration type 1 (restates onnx_utils.py:172-260 for the product path).
 * dmrs_symbols: the DMRS OFDM symbol indices; cdm_group[u] in {0,1}. */
int nrx_compute_pe(int32_t num_tx, int32_t num_subcarriers, int32_t num_symbols,
                   const int32_t* dmrs_symbols, int32_t num_dmrs_symbols,
                   const int32_t* cdm_group, float* pe_out);

/* Algorithmic FLOPs of one forward per resource element per user
 * (SURVEY.md 8(d) formula). */
double nrx_flops_per_re_user(const nrx_desc* desc, int32_t num_it);

/* Per-kernel timing.  While enabled, nrx_forward records a HIP event pair around
 * every kernel launch on the launch stream (not graph-capture safe).  Kernel ids:
 * 0 norm, 1 state-init (+ fused aggregation tail), 2 state-update (+ fused aggregation
 * or readout tail), 3 the one-launch forward (StateInit + updates + readouts; see
 * nrx_fused_status for when it is taken), 4 the register-resident state-update launch
 * (nrx_update_schedule), 5 the leave-one-out combine pass of U > 2 users (k_combine: after
 * StateInit and after every aggregation update), 6 the whole-column state-update launch, 7 the
 * whole-column StateInit launch (nrx_update_schedule).
 * nrx_profile_enable(h, 1) (re)starts the counters; nrx_profile_read waits for the
 * recorded events and returns the launch count and summed device time of a kernel. */
int nrx_profile_enable(nrx_handle* h, int32_t enable);
int nrx_profile_read(nrx_handle* h, int32_t kernel, int64_t* launches, double* total_ms);

/* The one-launch forward (k_forward, f16 only): StateInit, every update and the readouts as ONE
 * persistent launch whose items wait on per-(stage, slot) counters in a handle-owned buffer.
 * It applies to f16 forwards with 24-row strips and at least two items per CU, U <= 8 users,
 * 2A <= 32 (16 rx antennas), Var-IO (one StateInit stage per MCS), up to 8 iterations
 * (num_init + num_it <= 12) and up to three LLR heads.  Which shapes take it by default is set
 * by nrx_fused_config (default: the shapes where it measured faster -- U <= 2 with at least four
 * stages, i.e. Var-IO and 8-iteration models such as BASELINE cfg4 / cfg4'; the 2-iteration
 * bench forward, U > 2 and the large grids run the three-launch path).  status[3] since the
 * last reset: [0] error bits (1: a bounded dependency wait timed out, 2: items left undone --
 * the results of that forward are invalid), [1] update items whose inputs were not complete
 * when the previous item polled for them, [2] the polls those waits took.  Blocking: waits for
 * an event the handle recorded behind its last one-launch forward (not for the caller's stream,
 * which may have been destroyed since); reset != 0 clears them.  Returns NRX_ERR_FUSED (message
 * with the bits) when the error word is non-zero, so a caller that only checks the status code
 * cannot miss it; status[] is filled either way.
 * Forwards on one handle must not run concurrently on several streams (the counters are per
 * handle): nrx_forward / nrx_forward_ex / nrx_forward_aerial return NRX_ERR_BUSY, before
 * launching anything, when a forward that would take this path arrives on a stream other than
 * the previous one-launch forward's while that forward has not finished.  Forwards captured
 * into a hipGraph record no event: graph replays are outside this guard, so a caller replays
 * one handle's graphs on one stream.  NRX_FUSED in the environment (read by nrx_create): 0/off
 * the three-launch path, 1/on the default, 2/force wherever the path applies; any other value
 * fails nrx_create with NRX_ERR_INVALID_ARG. */
int nrx_fused_status(nrx_handle* h, int32_t* status, int32_t reset);

/* Per-handle control of the one-launch forward: enable = 0 no one-launch forward of any kind
 * (k_forward or k_fwd_col); 1 (default) k_forward only for the shapes it applies to by default
 * (U <= 2 with conv1 reading its rows from memory, at least four stages) that the column launches
 * do not take -- no BASELINE shape since round 6; 2 k_forward for every shape it applies to
 * (also the 2-iteration bench forward, U <= 8 and 2A <= 32 with staged z images; outputs
 * identical to the launch loop); > 2 invalid.  The initial value comes from NRX_FUSED at
 * nrx_create; spin_limit = dependency-wait polls before the timeout error (0: the default,
 * ~0.5 s); inject_err = error bits the next forwards set in the error word (test hook: callers
 * must surface them; 0: none).  Any argument < 0 leaves that setting unchanged. */
int nrx_fused_config(nrx_handle* h, int32_t enable, int32_t spin_limit, int32_t inject_err);

/* Stage schedule of the three-launch f16 forward, a mask (24-row strip tier):
 *   bit 0 (1)  the aggregation update stages (every iteration but the last) and
 *   bit 1 (2)  the readout update stage (the last) as the register-resident 16-row launch
 *              (k_update_rr: layer outputs kept in registers, weights staged once per workgroup);
 *   bit 2 (4)  the aggregation update stages and
 *   bit 3 (8)  the readout update stage as the whole-column launch (k_update_col: 48-position
 *              items, 6 register-resident rows per wave, no halo on grids of <= 48 subcarriers;
 *              taken over bits 0 / 1);
 *   bit 4 (16) StateInit as the whole-column launch (k_init_col: one StateInit, 2A = 8);
 *   bit 5 (32) the one-launch column forward (k_fwd_col: StateInit + every update in one
 *              persistent launch, at most one item per CU and stage; opt-in, measured slower);
 *   bit 6 (64) the column updates on grids wider than one column too (44-output strips;
 *              measured slower than the RR launch there, so off by default).
 * Each applies where it can -- the update launches with conv1 reading its rows from memory (any
 * U: for U > 2 the combine pass's a_u planes), 2A <= 32, for the readout stage one LLR head
 * whose readout fits -- the strip kernels elsewhere.  0: the strip kernels everywhere; < 0
 * unchanged; > 127 invalid.  Outputs are bit-identical either way.  The initial value comes from
 * NRX_UPDATE_RR (0..127) at nrx_create; the default (29: column StateInit and column updates on
 * single-column grids, the RR aggregation update elsewhere) is the mask measured fastest on every
 * BASELINE shape.  Kernel ids 6 / 7 / 8 of nrx_profile_read time the column
 * update / StateInit / one-launch column forward. */
int nrx_update_schedule(nrx_handle* h, int32_t update_rr);

const char* nrx_last_error(void);
int32_t nrx_api_version(void);
/* Content hash of the sources this library was built from (16 hex digits; set at link time by
 * neural_rx_amd/build.py).  Recorded with every committed counter capture so that a bench line
 * can tell whether the counters it quotes were taken from the library that is running. */
const char* nrx_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* NRX_H_ */
