"""SURVEY.md 8(d)'s third f16 criterion: the uncoded BER of the f16 engine on generated slots is
within statistical noise of the fp64 oracle's BER on the same slots (needs an MI355X).

Slots come from the GPU generator (nrx_generate_slots: 16-QAM / var-MCS QPSK..64-QAM, DMRS
type 1, TDL channel, AWGN, LS + NN h_hat), the same y / h_hat / active feed the f16 engine and
the fp64 numpy oracle (oracle/cgnn_ref.py, neural_rx.py:544-595), and the hard decisions
(LLR > 0 -> bit 1) of both are compared with the transmitted bits on the data REs of the active
users (DMRS symbols carry no data, jumpstart_tutorial.ipynb:339).

Gate: |BER_f16 - BER_oracle| <= 3 sigma + 1/n with sigma = sqrt(p (1 - p) / n), p = the
oracle's BER and n the counted bits: the binomial standard error of the oracle's own BER
estimate, i.e. the f16 engine may not move the BER by more than the Monte-Carlo noise of the
measurement.  The decisions are paired (same slots), so the difference is bounded by the
decision flips, reported beside it.  Two Eb/N0 points per model: nrx_rt (16-QAM, 2 UE) and
nrx_large_var_mcs_64qam_masking (8 iterations, QPSK / 16 / 64-QAM drawn per (slot, user), one
sliced head).
"""
import numpy as np
import pytest

from tests.helpers import Case, run_engine, run_oracle

pytestmark = pytest.mark.gpu


def _generated_case(config, users, prbs, batch, ebno_db, var_mcs, seed):
    import torch
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import get_config, spec_from_config
    from neural_rx_amd.generator import GenParams, SlotGenerator, ebno_to_no
    from oracle import pe_ref
    cfg = get_config(config)
    spec = spec_from_config(cfg)
    p = GenParams.from_config(cfg, num_tx=users, num_prbs=prbs, var_mcs=var_mcs, seed=seed)
    sb = SlotGenerator(p)(batch, ebno_to_no(ebno_db, len(p.dmrs_symbols)))
    torch.cuda.synchronize()
    h = lambda t: t.cpu().numpy()  # noqa: E731
    pe = pe_ref.pe_for_groups(p.num_subcarriers, 14, p.dmrs_symbols, p.cdm_group)
    mask = h(sb.mcs_mask)   # the oracle takes the one-hot mask for every non-masking model
    case = Case(config, cfg, spec, W.load(cfg.label), h(sb.y), pe, h(sb.h_hat), h(sb.active), mask)
    return case, h(sb.bits), h(sb.mcs), p


def _decisions(get, bits, mcs, active, spec, p):
    """hard decisions and transmitted bits on the data REs of active users; ``get(m)`` =
    LLRs ``[B,U,F,T,>= bits_m]`` of MCS m."""
    data_t = np.array([t not in p.dmrs_symbols for t in range(14)])
    dec, tx = [], []
    B, U = active.shape
    for b in range(B):
        for u in range(U):
            if active[b, u] == 0:
                continue
            m = int(mcs[b, u])
            nb = spec.bits[m]
            dec.append((get(m)[b, u][:, data_t, :nb] > 0).ravel())
            tx.append((bits[b, u][:, data_t, :nb] != 0).ravel())
    return np.concatenate(dec), np.concatenate(tx)


@pytest.mark.parametrize("config,users,batch,var_mcs,points", [
    ("nrx_rt", 2, 32, False, (2.0, 8.0)),
    ("nrx_large_var_mcs_64qam_masking", 2, 16, True, (8.0, 16.0)),
])
def test_f16_ber_within_oracle_noise(config, users, batch, var_mcs, points):
    from tests.test_gpu_parity import engine_for
    for k, ebno in enumerate(points):
        case, bits, mcs, p = _generated_case(config, users, 4, batch, ebno, var_mcs, seed=4321 + k)
        ref = run_oracle(case)
        raw = run_engine(case, "f16", engine_for(case))["llr_raw"]
        sp = case.spec
        d_o, tx = _decisions(lambda m: np.asarray(ref["llr"][m]), bits, mcs, case.active, sp, p)
        d_g, tx2 = _decisions(lambda m: raw[0 if sp.masking else m], bits, mcs, case.active, sp, p)
        assert np.array_equal(tx, tx2) and tx.size > 0
        n = tx.size
        ber_o, ber_g = float(np.mean(d_o != tx)), float(np.mean(d_g != tx))
        sigma = np.sqrt(max(ber_o * (1 - ber_o), 1.0 / n) / n)
        flips = int(np.count_nonzero(d_o != d_g))
        print(f"{config} Eb/N0 {ebno} dB: BER oracle {ber_o:.4e}  f16 {ber_g:.4e}  n {n}  "
              f"sigma {sigma:.2e}  decision flips {flips}")
        assert abs(ber_g - ber_o) <= 3 * sigma + 1.0 / n, (config, ebno, ber_o, ber_g, sigma)
