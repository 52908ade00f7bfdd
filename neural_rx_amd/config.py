"""Model/system description of the CGNN neural receiver.

The reference keeps its configuration in INI files whose values are Python
``eval``'d into attributes (``utils/parameters.py:91-113``; e.g.
``config/nrx_rt.cfg:57-75`` for the ``[neural_receiver]`` block).  This module
reads the same files with ``configparser`` + ``ast.literal_eval`` (never ``eval``),
keeps only the fields the CGNN forward pass depends on, and ships a built-in table
for the five configurations in scope so that nothing under
``/root/reference`` is needed at run time.
"""
from __future__ import annotations

import ast
import configparser
import dataclasses
from typing import List, Optional, Tuple

import numpy as np

# 5G NR MCS table 1 (TS 38.214 Table 5.1.3.1-1): modulation order per MCS index.
# Only the order matters for the NRX (num_bits_per_symbol per head).
_MCS_TABLE1_QM = [2] * 10 + [4] * 7 + [6] * 12  # MCS 0..28


def mcs_to_bits(mcs_index: int, mcs_table: int = 1) -> int:
    """Bits per symbol for an MCS index (reference: Sionna ``TBConfig`` via
    ``pusch_configs[i][0].tb.num_bits_per_symbol``, neural_rx.py:660-668)."""
    if mcs_table != 1:
        raise ValueError("only MCS table 1 is used by the in-scope configs")
    return _MCS_TABLE1_QM[mcs_index]


@dataclasses.dataclass(frozen=True)
class NRXConfig:
    """The fields of a reference ``.cfg`` that define the CGNN forward pass."""

    label: str
    n_size_bwp: int                     # PRBs used for training/eval grid
    n_size_bwp_eval: int                # PRBs used at evaluation (nrx_rt.cfg:118)
    num_rx_antennas: int                # A
    mcs_index: Tuple[int, ...]          # one entry per supported MCS (Var-IO heads)
    num_nrx_iter: int                   # trained CGNN iterations
    num_nrx_iter_eval: int
    d_s: int
    num_units_init: Tuple[int, ...]
    num_units_agg: Tuple[Tuple[int, ...], ...]
    num_units_state: Tuple[Tuple[int, ...], ...]
    num_units_readout: Tuple[int, ...]
    max_num_tx: int
    var_mcs_masking: bool = False
    initial_chest: Optional[str] = "ls"
    custom_constellation: bool = False
    mask_pilots: bool = False
    # DMRS description (TS 38.211 PUSCH DMRS, mapping type A, config type 1)
    dmrs_type_a_position: int = 2
    dmrs_additional_position: int = 1
    dmrs_length: int = 1
    dmrs_config_type: int = 1
    dmrs_port_sets: Tuple[Tuple[int, ...], ...] = ((0,), (2,))
    num_cdm_groups_without_data: int = 2
    symbol_allocation: Tuple[int, int] = (0, 14)

    @property
    def bits_per_head(self) -> Tuple[int, ...]:
        return tuple(mcs_to_bits(m) for m in self.mcs_index)

    @property
    def num_mcs(self) -> int:
        return len(self.mcs_index)

    @property
    def num_ofdm_symbols(self) -> int:
        return self.symbol_allocation[1]


def _lit(v: str):
    v = v.strip()
    if v in ("tf.float32", "torch.float32"):
        return "float32"
    if v in ("tf.float16", "torch.float16"):
        return "float16"
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def _tup(x):
    if isinstance(x, (list, tuple)):
        return tuple(_tup(i) for i in x)
    return x


def parse_cfg(path: str) -> NRXConfig:
    """Parse a reference-format ``.cfg`` (``utils/parameters.py:91-132``) safely."""
    cp = configparser.ConfigParser(inline_comment_prefixes=("#",))
    cp.optionxform = str
    with open(path) as f:
        cp.read_file(f)
    sec = {}
    for s in cp.sections():
        for k, v in cp.items(s):
            sec[k] = _lit(v)
    n_eval = sec.get("n_size_bwp_eval", sec["n_size_bwp"])
    return NRXConfig(
        label=str(sec["label"]),
        n_size_bwp=int(sec["n_size_bwp"]),
        n_size_bwp_eval=int(n_eval),
        num_rx_antennas=int(sec["num_rx_antennas"]),
        mcs_index=tuple(sec["mcs_index"]),
        num_nrx_iter=int(sec["num_nrx_iter"]),
        num_nrx_iter_eval=int(sec.get("num_nrx_iter_eval", sec["num_nrx_iter"])),
        d_s=int(sec["d_s"]),
        num_units_init=_tup(sec["num_units_init"]),
        num_units_agg=_tup(sec["num_units_agg"]),
        num_units_state=_tup(sec["num_units_state"]),
        num_units_readout=_tup(sec["num_units_readout"]),
        max_num_tx=int(sec["max_num_tx"]),
        var_mcs_masking=bool(sec.get("mcs_var_mcs_masking", False)),
        initial_chest=sec.get("initial_chest", "ls"),
        custom_constellation=bool(sec.get("custom_constellation", False)),
        mask_pilots=bool(sec.get("mask_pilots", False)),
        dmrs_type_a_position=int(sec.get("dmrs_type_a_position", 2)),
        dmrs_additional_position=int(sec.get("dmrs_additional_position", 1)),
        dmrs_length=int(sec.get("dmrs_length", 1)),
        dmrs_config_type=int(sec.get("dmrs_config_type", 1)),
        dmrs_port_sets=_tup(sec.get("dmrs_port_sets", [[0], [2]])),
        num_cdm_groups_without_data=int(sec.get("num_cdm_groups_without_data", 2)),
        symbol_allocation=_tup(sec.get("symbol_allocation", [0, 14])),
    )


def _mk(label, iters, mcs, masking=False, n_eval=132):
    return NRXConfig(
        label=label, n_size_bwp=4, n_size_bwp_eval=n_eval, num_rx_antennas=4,
        mcs_index=tuple(mcs), num_nrx_iter=iters, num_nrx_iter_eval=iters, d_s=56,
        num_units_init=(128, 128), num_units_agg=((64,),) * iters,
        num_units_state=((128, 128),) * iters, num_units_readout=(128,),
        max_num_tx=2, var_mcs_masking=masking)


# Built-in table: values as in the reference cfg files (checked against them by
# tests/test_config.py when /root/reference is present).
BUILTIN = {
    "nrx_rt": _mk("nrx_rt", 2, [14]),                       # nrx_rt.cfg:16-18,57-75
    "nrx_rt_var_mcs": _mk("nrx_rt_var_mcs", 2, [9, 14]),    # nrx_rt_var_mcs.cfg:18
    "nrx_large": _mk("nrx_large", 8, [14]),                 # nrx_large.cfg:57-62
    "nrx_large_64qam": _mk("nrx_large_64qam", 8, [19]),     # nrx_large_64qam.cfg:18
    "nrx_large_var_mcs_64qam_masking": _mk(
        "nrx_large_var_mcs_64qam_masking", 8, [9, 14, 19], masking=True),
}


def get_config(name: str) -> NRXConfig:
    if name.endswith(".cfg"):
        return parse_cfg(name)
    return BUILTIN[name]


def with_overrides(cfg: NRXConfig, **kw) -> NRXConfig:
    return dataclasses.replace(cfg, **kw)


@dataclasses.dataclass(frozen=True)
class ModelSpec:
    """Shapes of one CGNN instance (the topology the weights must match)."""

    num_rx_ant: int
    d_s: int
    num_it: int                  # trained iterations (len(iterations))
    bits: Tuple[int, ...]        # bits per head (len == num_mcs)
    masking: bool                # one head of max(bits) sliced per MCS
    init_units: Tuple[int, ...] = (128, 128)
    agg_units: int = 64
    state_units: Tuple[int, ...] = (128, 128)
    readout_units: int = 128
    use_h_hat: bool = True

    @property
    def num_mcs(self) -> int:
        return len(self.bits)

    @property
    def num_init(self) -> int:
        return 1 if self.masking else self.num_mcs

    @property
    def num_llr_heads(self) -> int:
        return 1 if self.masking else self.num_mcs

    @property
    def head_bits(self) -> List[int]:
        return [max(self.bits)] if self.masking else list(self.bits)

    @property
    def bits_max(self) -> int:
        return max(self.bits)

    @property
    def init_in_ch(self) -> int:
        return 4 * self.num_rx_ant + 2 if self.use_h_hat else 2 * self.num_rx_ant + 2

    @property
    def update_in_ch(self) -> int:
        return 2 * self.d_s + 2


def spec_from_config(cfg: NRXConfig, num_rx_ant: Optional[int] = None) -> ModelSpec:
    for u in cfg.num_units_agg:
        if len(u) != 1:
            raise ValueError("only one hidden aggregation layer is supported")
    if len(set(cfg.num_units_agg)) != 1 or len(set(cfg.num_units_state)) != 1:
        raise ValueError("per-iteration widths must be identical")
    return ModelSpec(
        num_rx_ant=num_rx_ant or cfg.num_rx_antennas,
        d_s=cfg.d_s,
        num_it=cfg.num_nrx_iter,
        bits=cfg.bits_per_head,
        masking=cfg.var_mcs_masking,
        init_units=tuple(cfg.num_units_init),
        agg_units=cfg.num_units_agg[0][0],
        state_units=tuple(cfg.num_units_state[0]),
        readout_units=cfg.num_units_readout[0],
        use_h_hat=cfg.initial_chest not in (None, "None"),
    )


def dmrs_symbols(cfg: NRXConfig) -> Tuple[int, ...]:
    """DMRS OFDM symbol positions for PUSCH mapping type A, single-symbol DMRS,
    slot of 14 symbols (TS 38.211 Table 6.4.1.1.3-3).  The reference takes them from
    Sionna's ``PUSCHDMRSConfig`` (printed as [2, 11] for nrx_rt,
    notebooks/jumpstart_tutorial.ipynb:298)."""
    if cfg.dmrs_length != 1 or cfg.symbol_allocation != (0, 14):
        raise ValueError("only single-symbol DMRS over a 14-symbol allocation")
    l0 = cfg.dmrs_type_a_position
    extra = {0: (), 1: (11,), 2: (7, 11), 3: (5, 8, 11)}[cfg.dmrs_additional_position]
    return (l0,) + extra


def dmrs_cdm_group(port: int, config_type: int = 1) -> int:
    """CDM group lambda of a DMRS port (TS 38.211 Table 6.4.1.1.3-1)."""
    if config_type != 1:
        raise ValueError("only DMRS configuration type 1")
    return (port // 2) % 2


def user_cdm_groups(cfg: NRXConfig, num_users: int) -> Tuple[int, ...]:
    """CDM group per user.  Users beyond the cfg's port sets (BASELINE configs with
    4 or 8 users) are synthesised as CDM group ``u mod 2``."""
    groups = []
    for u in range(num_users):
        if u < len(cfg.dmrs_port_sets):
            groups.append(dmrs_cdm_group(cfg.dmrs_port_sets[u][0], cfg.dmrs_config_type))
        else:
            groups.append(u % 2)
    return tuple(groups)


def data_re_indices(cfg: NRXConfig, num_subcarriers: int, num_symbols: int = 14) -> np.ndarray:
    """Data-carrying REs of the PUSCH resource grid as ``t * F + f`` in grid order
    (symbol-major), int32.  DMRS type 1 with two CDM groups without data: the DMRS symbols
    carry no data (jumpstart_tutorial.ipynb:339); no guard / DC subcarriers in a PUSCH
    allocation.  The reference's RG type grid (siona_tf.py:2153-2195) marks the same REs
    0 = data; ``argsort`` of it (onnx_utils.py:465) lists them in this order."""
    dm = set(dmrs_symbols(cfg))
    ts = [t for t in range(num_symbols) if t not in dm]
    return np.array([t * num_subcarriers + f for t in ts for f in range(num_subcarriers)], np.int32)
