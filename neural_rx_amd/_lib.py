"""ctypes binding of ``libnrx.so`` (the C ABI declared in ``include/nrx.h``).

There is deliberately no fallback: if the HIP library is missing or fails to load,
every engine entry point raises ``NRXLibraryError``.  Build it with
``python -m neural_rx_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# NRX_LIB_PATH: diagnostic override (kernel-variant A/B runs); the default is the in-tree build
LIB_PATH = os.environ.get("NRX_LIB_PATH") or os.path.join(LIB_DIR, "libnrx.so")

NRX_OK = 0
NRX_ERR_INVALID_ARG = -1
NRX_ERR_BUSY = -7
NRX_ERR_FUSED = -8
NRX_PREC_F16 = 0
NRX_PREC_F32X = 1
PRECISIONS = {"f16": NRX_PREC_F16, "fp16": NRX_PREC_F16, "f32x": NRX_PREC_F32X,
              "parity": NRX_PREC_F32X}

# Every exported symbol of include/nrx.h (checked by tests/test_abi.py).
EXPORTS = [
    "nrx_create", "nrx_weight_layout", "nrx_workspace_size", "nrx_forward", "nrx_destroy",
    "nrx_compute_pe", "nrx_flops_per_re_user", "nrx_last_error", "nrx_api_version",
    "nrx_profile_enable", "nrx_profile_read", "nrx_aerial_workspace_size", "nrx_forward_aerial",
    "nrx_llr_demap", "nrx_gen_workspace_size", "nrx_generate_slots", "nrx_count_errors",
    "nrx_workspace_size_ex", "nrx_forward_ex", "nrx_fused_status", "nrx_fused_config",
    "nrx_build_id", "nrx_update_schedule",
]
# enum nrx_y_layout
Y_LAYOUTS = {"cgnn": 0, "sionna": 1, "split": 2}
KERNELS = ["norm", "state_init", "state_update", "forward", "state_update_rr", "combine", "state_update_col",
           "state_init_col", "forward_col"]


class NRXLibraryError(RuntimeError):
    pass


class NRXError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"nrx error {code}: {msg}")
        self.code = code


class nrx_desc(ctypes.Structure):
    _fields_ = [
        ("num_rx_ant", ctypes.c_int32),
        ("d_s", ctypes.c_int32),
        ("num_it", ctypes.c_int32),
        ("num_mcs", ctypes.c_int32),
        ("bits", ctypes.c_int32 * 8),
        ("var_mcs_masking", ctypes.c_int32),
        ("init_units", ctypes.c_int32 * 2),
        ("agg_units", ctypes.c_int32),
        ("state_units", ctypes.c_int32 * 2),
        ("readout_units", ctypes.c_int32),
        ("use_h_hat", ctypes.c_int32),
    ]


class nrx_shape(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int32),
        ("num_tx", ctypes.c_int32),
        ("num_subcarriers", ctypes.c_int32),
        ("num_symbols", ctypes.c_int32),
    ]


class nrx_io(ctypes.Structure):
    _fields_ = [
        ("shape", nrx_shape),
        ("num_it", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("y", ctypes.c_void_p),
        ("pe", ctypes.c_void_p),
        ("h_hat", ctypes.c_void_p),
        ("active", ctypes.c_void_p),
        ("mcs_mask", ctypes.c_void_p),
        ("llr", ctypes.c_void_p),
        ("h_ref", ctypes.c_void_p),
    ]


class nrx_aerial_io(ctypes.Structure):
    _fields_ = [
        ("shape", nrx_shape),
        ("num_it", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("num_dmrs_symbols", ctypes.c_int32),
        ("num_dmrs_subcarriers", ctypes.c_int32),
        ("y_real", ctypes.c_void_p),
        ("y_imag", ctypes.c_void_p),
        ("h_ls_real", ctypes.c_void_p),
        ("h_ls_imag", ctypes.c_void_p),
        ("dmrs_port_mask", ctypes.c_void_p),
        ("dmrs_ofdm_pos", ctypes.c_void_p),
        ("dmrs_subcarrier_pos", ctypes.c_void_p),
        ("llr", ctypes.c_void_p),
        ("h_hat", ctypes.c_void_p),
    ]


class nrx_gen_desc(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int32),
        ("num_tx", ctypes.c_int32),
        ("num_subcarriers", ctypes.c_int32),
        ("num_symbols", ctypes.c_int32),
        ("num_rx_ant", ctypes.c_int32),
        ("num_dmrs_symbols", ctypes.c_int32),
        ("dmrs_symbols", ctypes.c_int32 * 4),
        ("dmrs_symbol_mask", ctypes.c_int32),
        ("cdm_group", ctypes.c_int32 * 16),
        ("num_mcs", ctypes.c_int32),
        ("mcs_bits", ctypes.c_int32 * 8),
        ("mcs_of_user", ctypes.c_int32 * 16),
        ("num_active", ctypes.c_int32),
        ("num_taps", ctypes.c_int32),
        ("num_sinusoids", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("max_delay_s", ctypes.c_double),
        ("max_doppler_hz", ctypes.c_double),
        ("subcarrier_spacing", ctypes.c_double),
        ("no", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("slot_offset", ctypes.c_int64),
    ]


class nrx_gen_out(ctypes.Structure):
    _fields_ = [
        ("y", ctypes.c_void_p),
        ("h_hat", ctypes.c_void_p),
        ("h", ctypes.c_void_p),
        ("active", ctypes.c_void_p),
        ("mcs_mask", ctypes.c_void_p),
        ("mcs", ctypes.c_void_p),
        ("bits", ctypes.c_void_p),
        ("bits_stride", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("y_real", ctypes.c_void_p),
        ("y_imag", ctypes.c_void_p),
        ("h_ls_real", ctypes.c_void_p),
        ("h_ls_imag", ctypes.c_void_p),
    ]


class nrx_count_io(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int32),
        ("num_tx", ctypes.c_int32),
        ("num_subcarriers", ctypes.c_int32),
        ("num_symbols", ctypes.c_int32),
        ("num_heads", ctypes.c_int32),
        ("bits_stride", ctypes.c_int32),
        ("num_mcs", ctypes.c_int32),
        ("mcs_bits", ctypes.c_int32 * 8),
        ("dmrs_symbol_mask", ctypes.c_int32),
        ("llr", ctypes.c_void_p),
        ("bits", ctypes.c_void_p),
        ("mcs", ctypes.c_void_p),
        ("active", ctypes.c_void_p),
        ("counts", ctypes.c_void_p),
    ]


_lib = None


def load(path: str = LIB_PATH):
    """Load libnrx.so once; raise NRXLibraryError if it is missing or broken."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NRXLibraryError(
            f"{path} not found: the MI355X engine is not built "
            "(run `python -m neural_rx_amd.build`); there is no CPU fallback")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.  Load
    # torch first so that libnrx's DT_NEEDED libamdhip64.so.7 binds to that copy
    # (by soname) instead of pulling /opt/rocm's as a second runtime.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - plain C users
        pass
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the box
        raise NRXLibraryError(f"failed to load {path}: {e}") from e
    c = ctypes
    P = c.POINTER
    lib.nrx_create.argtypes = [P(nrx_desc), P(c.c_void_p), P(c.c_int64), c.c_int32, c.c_int32,
                               P(c.c_void_p)]
    lib.nrx_create.restype = c.c_int
    lib.nrx_weight_layout.argtypes = [P(nrx_desc), P(c.c_int32), P(c.c_int64), c.c_int32]
    lib.nrx_weight_layout.restype = c.c_int
    lib.nrx_workspace_size.argtypes = [c.c_void_p, P(nrx_shape), c.c_int32, P(c.c_size_t)]
    lib.nrx_workspace_size.restype = c.c_int
    lib.nrx_forward.argtypes = [c.c_void_p, P(nrx_io), c.c_void_p, c.c_size_t, c.c_void_p]
    lib.nrx_forward.restype = c.c_int
    lib.nrx_workspace_size_ex.argtypes = [c.c_void_p, P(nrx_shape), c.c_int32, c.c_int32, P(c.c_size_t)]
    lib.nrx_workspace_size_ex.restype = c.c_int
    lib.nrx_forward_ex.argtypes = [c.c_void_p, P(nrx_io), c.c_int32, c.c_void_p, c.c_void_p, c.c_size_t,
                                   c.c_void_p]
    lib.nrx_forward_ex.restype = c.c_int
    lib.nrx_destroy.argtypes = [c.c_void_p]
    lib.nrx_destroy.restype = None
    lib.nrx_compute_pe.argtypes = [c.c_int32, c.c_int32, c.c_int32, P(c.c_int32), c.c_int32,
                                   P(c.c_int32), P(c.c_float)]
    lib.nrx_compute_pe.restype = c.c_int
    lib.nrx_flops_per_re_user.argtypes = [P(nrx_desc), c.c_int32]
    lib.nrx_flops_per_re_user.restype = c.c_double
    lib.nrx_last_error.argtypes = []
    lib.nrx_last_error.restype = c.c_char_p
    lib.nrx_profile_enable.argtypes = [c.c_void_p, c.c_int32]
    lib.nrx_profile_enable.restype = c.c_int
    lib.nrx_profile_read.argtypes = [c.c_void_p, c.c_int32, P(c.c_int64), P(c.c_double)]
    lib.nrx_profile_read.restype = c.c_int
    lib.nrx_fused_status.argtypes = [c.c_void_p, c.c_void_p, c.c_int32]
    lib.nrx_fused_status.restype = c.c_int
    lib.nrx_fused_config.argtypes = [c.c_void_p, c.c_int32, c.c_int32, c.c_int32]
    lib.nrx_fused_config.restype = c.c_int
    lib.nrx_aerial_workspace_size.argtypes = [c.c_void_p, P(nrx_aerial_io), P(c.c_size_t)]
    lib.nrx_aerial_workspace_size.restype = c.c_int
    lib.nrx_forward_aerial.argtypes = [c.c_void_p, P(nrx_aerial_io), c.c_void_p, c.c_size_t, c.c_void_p]
    lib.nrx_forward_aerial.restype = c.c_int
    lib.nrx_llr_demap.argtypes = [c.c_void_p, c.c_int32, c.c_int32, c.c_int32, c.c_int32, c.c_int32, c.c_int32,
                                  c.c_void_p, c.c_int32, c.c_void_p, c.c_void_p]
    lib.nrx_llr_demap.restype = c.c_int
    lib.nrx_gen_workspace_size.argtypes = [P(nrx_gen_desc), P(c.c_size_t)]
    lib.nrx_gen_workspace_size.restype = c.c_int
    lib.nrx_generate_slots.argtypes = [P(nrx_gen_desc), P(nrx_gen_out), c.c_void_p, c.c_size_t, c.c_void_p]
    lib.nrx_generate_slots.restype = c.c_int
    lib.nrx_count_errors.argtypes = [P(nrx_count_io), c.c_void_p]
    lib.nrx_count_errors.restype = c.c_int
    lib.nrx_api_version.argtypes = []
    lib.nrx_api_version.restype = c.c_int32
    lib.nrx_update_schedule.argtypes = [c.c_void_p, c.c_int32]
    lib.nrx_update_schedule.restype = c.c_int
    lib.nrx_build_id.argtypes = []
    lib.nrx_build_id.restype = c.c_char_p
    _lib = lib
    return lib


def check(rc: int):
    if rc != NRX_OK:
        msg = _lib.nrx_last_error().decode() if _lib is not None else "?"
        raise NRXError(rc, msg)


def make_desc(spec) -> nrx_desc:
    d = nrx_desc()
    d.num_rx_ant = spec.num_rx_ant
    d.d_s = spec.d_s
    d.num_it = spec.num_it
    d.num_mcs = spec.num_mcs
    for i, b in enumerate(spec.bits):
        d.bits[i] = b
    d.var_mcs_masking = int(spec.masking)
    d.init_units[0], d.init_units[1] = spec.init_units
    d.agg_units = spec.agg_units
    d.state_units[0], d.state_units[1] = spec.state_units
    d.readout_units = spec.readout_units
    d.use_h_hat = int(spec.use_h_hat)
    return d
