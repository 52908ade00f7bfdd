"""Shared test fixtures: seeded cases run through the oracle and the engine."""
from __future__ import annotations

import dataclasses
from typing import Optional, Sequence

import numpy as np

from neural_rx_amd import synth
from neural_rx_amd import weights as W
from neural_rx_amd.config import dmrs_symbols, get_config, spec_from_config, user_cdm_groups
from oracle import cgnn_ref, pe_ref


@dataclasses.dataclass
class Case:
    name: str
    cfg: object
    spec: object
    weights: list
    y: np.ndarray
    pe: np.ndarray
    h_hat: Optional[np.ndarray]
    active: np.ndarray
    mcs_mask: Optional[np.ndarray]
    slots: Optional[synth.Slots] = None
    num_it: Optional[int] = None


def make_case(config="nrx_rt", batch=2, users=2, prbs=4, snr_db=15.0, seed=1,
              active=None, mcs_choice: Optional[Sequence[int]] = None, num_rx_ant=None,
              random_inputs=False, num_it=None, seeded_weights=False) -> Case:
    cfg = get_config(config)
    spec = spec_from_config(cfg, num_rx_ant)
    weights = W.seeded(spec, seed=seed) if seeded_weights else W.load(cfg.label)
    groups = user_cdm_groups(cfg, users)
    f = 12 * prbs
    pe = pe_ref.pe_for_groups(f, 14, dmrs_symbols(cfg), groups)
    rng = np.random.default_rng(seed + 100)
    if mcs_choice is None:
        mcs_choice = rng.integers(0, spec.num_mcs, size=(batch, users))
    mcs_choice = np.asarray(mcs_choice).reshape(batch, users)
    mask = np.eye(spec.num_mcs, dtype=np.float32)[mcs_choice]
    if active is None:
        active = np.ones((batch, users), np.float32)
    active = np.asarray(active, np.float32)
    slots = None
    if random_inputs:
        a2 = 2 * spec.num_rx_ant
        y = rng.standard_normal((batch, f, 14, a2)).astype(np.float32)
        h = rng.standard_normal((batch, users, f, 14, a2)).astype(np.float32)
    else:
        bits = [spec.bits[mcs_choice[0, u]] for u in range(users)]
        slots = synth.generate(batch, users, prbs, spec.num_rx_ant, bits, groups,
                               dmrs_symbols(cfg), snr_db=snr_db, seed=seed, active=active)
        y, h = slots.y, slots.h_hat
    return Case(config, cfg, spec, weights, y, pe, h, active, mask, slots, num_it)


def run_oracle(case: Case, dtype=np.float64):
    w = cgnn_ref.split_keras_weights(case.weights, case.spec)
    return cgnn_ref.cgnn_forward(case.y, case.pe, case.h_hat, case.active, case.mcs_mask, w,
                                 case.spec, num_it=case.num_it, dtype=dtype)


def run_engine(case: Case, precision="f16", engine=None):
    import torch
    from neural_rx_amd.receiver import CGNNEngine
    eng = engine or CGNNEngine(case.spec, case.weights)
    dev = "cuda:0"
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
    llr, h = eng.forward(t(case.y), t(case.pe), t(case.h_hat), t(case.active), t(case.mcs_mask),
                         num_it=case.num_it, precision=precision)
    torch.cuda.synchronize()
    llr = llr.cpu().numpy()
    sp = case.spec
    per_mcs = [llr[0 if sp.masking else m, ..., :nb] for m, nb in enumerate(sp.bits)]
    return {"llr": per_mcs, "llr_raw": llr, "h_hat": h.cpu().numpy()}


def compare(ref, got):
    """max-abs LLR / h errors, relative-to-max error and hard-decision disagreement."""
    out = {}
    lmax = max(float(np.abs(r).max()) for r in ref["llr"])
    errs = [float(np.abs(r - g).max()) for r, g in zip(ref["llr"], got["llr"])]
    flips = [float((np.sign(r) != np.sign(g)).mean()) for r, g in zip(ref["llr"], got["llr"])]
    out["llr_maxabs"] = max(errs)
    out["llr_rel"] = max(errs) / max(lmax, 1e-12)
    out["flip_rate"] = max(flips)
    out["h_maxabs"] = float(np.abs(ref["h_hat"] - got["h_hat"]).max())
    out["llr_max"] = lmax
    # hard-decision disagreement restricted to confident reference bits
    conf = [float((np.sign(r) != np.sign(g))[np.abs(r) > 0.5].mean()) if (np.abs(r) > 0.5).any() else 0.0
            for r, g in zip(ref["llr"], got["llr"])]
    out["flip_rate_confident"] = max(conf)
    rms = [float(np.sqrt(np.mean((r - g) ** 2)) / max(np.sqrt(np.mean(r ** 2)), 1e-12))
           for r, g in zip(ref["llr"], got["llr"])]
    out["llr_rms_rel"] = max(rms)
    return out


@dataclasses.dataclass
class AerialCase:
    """NeuralReceiverONNX inputs (Aerial pilot order) + the oracle's preprocessed CGNN case."""
    inputs: dict
    case: Case


def make_aerial_case(config="nrx_rt", batch=2, users=2, prbs=4, snr_db=15.0, seed=1, active=None):
    base = make_case(config, batch=batch, users=users, prbs=prbs, snr_db=snr_db, seed=seed, active=active)
    cfg = base.cfg
    groups = user_cdm_groups(cfg, users)
    syms = list(dmrs_symbols(cfg))
    sl = base.slots
    yc = np.transpose(sl.y_complex[:, 0], (0, 3, 2, 1))                 # [B, F, T, A]
    h_re, h_im = synth.aerial_ls_pilots(yc, sl.x, groups, syms, prbs)
    ofdm = np.array([syms for _ in range(users)], np.int32)
    scp = np.array([[g + 2 * j for j in range(6)] for g in groups], np.int32)
    inputs = dict(y_real=np.ascontiguousarray(yc.real, np.float32), y_imag=np.ascontiguousarray(yc.imag, np.float32),
                  h_ls_real=h_re, h_ls_imag=h_im, dmrs_port_mask=base.active.copy(),
                  dmrs_ofdm_pos=ofdm, dmrs_subcarrier_pos=scp)
    y, h, pe = pe_ref.aerial_preprocess(inputs["y_real"], inputs["y_imag"], h_re, h_im, ofdm, scp, users)
    mask = np.zeros((batch, users, base.spec.num_mcs), np.float32)
    mask[..., 0] = 1.0                    # single MCS (the ONNX export's dummy mask)
    case = dataclasses.replace(base, y=y, h_hat=h, pe=pe, mcs_mask=mask)
    return AerialCase(inputs, case)


def run_engine_aerial(ac: AerialCase, precision="f16", engine=None):
    import torch
    from neural_rx_amd.receiver import CGNNEngine
    eng = engine or CGNNEngine(ac.case.spec, ac.case.weights)
    dev = "cuda:0"
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in ac.inputs.items()}
    llr, h = eng.forward_aerial(t["y_real"], t["y_imag"], t["h_ls_real"], t["h_ls_imag"], t["dmrs_port_mask"],
                                t["dmrs_ofdm_pos"], t["dmrs_subcarrier_pos"], num_it=ac.case.num_it,
                                precision=precision)
    torch.cuda.synchronize()
    return llr.cpu().numpy(), h.cpu().numpy()
