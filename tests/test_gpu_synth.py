"""GPU slot generator + error counters against the oracle (needs an MI355X).

Tolerances: integer outputs (bits, MCS, active ports, error counters) bit-exact; float
outputs (y, h, h_hat, Aerial LS pilots) within 2 f32 ulps of the oracle's relative scale
(1e-6 relative to max |.|, plus 1e-7 absolute): both sides compute in f64 and round once,
so only libm ulp differences of exp/log/sin/cos remain.
"""
import numpy as np
import pytest

from oracle import synth_ref as S

pytestmark = pytest.mark.gpu


def _gpu(params, batch, no, off=0, want_h=True, aerial=False):
    import torch
    from neural_rx_amd.generator import SlotGenerator
    g = SlotGenerator(params, want_h=want_h, aerial=aerial)
    sb = g(batch, no, slot_offset=off)
    torch.cuda.synchronize()
    return {k: (v.cpu().numpy() if v is not None else None) for k, v in vars(sb).items()}


def _oracle(params, batch, no, off=0):
    return S.generate(S.GenSpec(batch=batch, num_tx=params.num_tx, num_subcarriers=params.num_subcarriers,
                                num_rx_ant=params.num_rx_ant, dmrs_symbols=params.dmrs_symbols,
                                cdm_group=params.cdm_group, mcs_bits=params.mcs_bits,
                                mcs_of_user=params.mcs_of_user, num_active=params.num_active,
                                num_taps=params.num_taps, num_sinusoids=params.num_sinusoids,
                                max_delay_s=params.max_delay_s, max_doppler_hz=params.max_doppler_hz,
                                subcarrier_spacing=params.subcarrier_spacing, no=no, seed=params.seed,
                                slot_offset=off))


def _close(a, b, name):
    scale = float(np.abs(b).max()) if b.size else 1.0
    err = float(np.abs(a - b).max()) if b.size else 0.0
    assert err <= 1e-6 * scale + 1e-7, (name, err, scale)


def _check(params, batch, no, off=0):
    g = _gpu(params, batch, no, off)
    o = _oracle(params, batch, no, off)
    np.testing.assert_array_equal(g["active"], o.active)
    np.testing.assert_array_equal(g["mcs"], o.mcs)
    np.testing.assert_array_equal(g["bits"], o.bits)
    M = len(params.mcs_bits)
    np.testing.assert_array_equal(g["mcs_mask"], np.eye(M, dtype=np.float32)[o.mcs])
    _close(g["h"], o.h, "h")
    _close(g["y"], o.y, "y")
    _close(g["h_hat"], o.h_hat, "h_hat")
    return g, o


@pytest.mark.parametrize("config,users,prbs,ant", [("nrx_rt", 2, 4, 4), ("nrx_rt", 1, 1, 4),
                                                   ("nrx_large_64qam", 8, 2, 4), ("nrx_large", 4, 1, 16)])
def test_generator_matches_oracle(config, users, prbs, ant):
    from neural_rx_amd.generator import GenParams, ebno_to_no
    p = GenParams.from_config(config, num_tx=users, num_prbs=prbs, num_rx_ant=ant, seed=11)
    _check(p, 3, ebno_to_no(6.0), off=5)


def test_generator_var_mcs_and_random_ports():
    from neural_rx_amd.generator import GenParams, ebno_to_no
    p = GenParams.from_config("nrx_large_var_mcs_64qam_masking", num_tx=4, num_prbs=2, var_mcs=True, seed=3)
    p.num_active = 2
    g, o = _check(p, 6, ebno_to_no(10.0))
    assert (g["active"].sum(1) == 2).all()
    assert len(np.unique(g["mcs"])) > 1


def test_generator_odd_width_and_extremes():
    from neural_rx_amd.generator import GenParams
    p = GenParams(num_tx=2, num_subcarriers=13, num_rx_ant=2, dmrs_symbols=(2,), cdm_group=(1, 0), mcs_bits=(2,),
                  num_taps=1, num_sinusoids=1, max_delay_s=0.0, max_doppler_hz=0.0, seed=2**40 + 3)
    _check(p, 2, 0.0, off=2**33)


def test_shards_generate_the_same_slots():
    from neural_rx_amd.generator import GenParams
    p = GenParams.from_config("nrx_rt", seed=5)
    full = _gpu(p, 6, 0.05)
    part = _gpu(p, 2, 0.05, off=4)
    for k in ("y", "h_hat", "bits", "active"):
        np.testing.assert_array_equal(part[k], full[k][4:])


def test_aerial_outputs_consistent():
    from neural_rx_amd.generator import GenParams
    p = GenParams.from_config("nrx_rt", seed=9)
    g = _gpu(p, 2, 0.05, aerial=True)
    A = p.num_rx_ant
    np.testing.assert_array_equal(g["y_real"], g["y"][..., :A])
    np.testing.assert_array_equal(g["y_imag"], g["y"][..., A:])
    # pilot p = (k * nprb + prb) * 6 + j of user u sits at subcarrier prb*12 + cdm + 2j of DMRS symbol k,
    # where h_hat equals the LS value itself
    nprb = p.num_subcarriers // 12
    for u, c in enumerate(p.cdm_group):
        for k, t in enumerate(p.dmrs_symbols):
            for prb in range(nprb):
                for j in range(6):
                    pi = (k * nprb + prb) * 6 + j
                    f = prb * 12 + c + 2 * j
                    np.testing.assert_array_equal(g["h_ls_real"][:, pi, u], g["h_hat"][:, u, f, t, :A])
                    np.testing.assert_array_equal(g["h_ls_imag"][:, pi, u], g["h_hat"][:, u, f, t, A:])


@pytest.mark.parametrize("config,var_mcs", [("nrx_rt", False), ("nrx_rt_var_mcs", True),
                                            ("nrx_large_var_mcs_64qam_masking", True)])
def test_error_counters_match_oracle(config, var_mcs):
    import torch
    from neural_rx_amd import weights as W
    from neural_rx_amd.generator import GenParams, SlotGenerator, count_errors, ebno_to_no
    from neural_rx_amd.receiver import CGNNEngine, compute_pe, spec_for
    spec = spec_for(config)
    p = GenParams.from_config(config, num_prbs=2, var_mcs=var_mcs, seed=21)
    p.num_active = 1
    gen = SlotGenerator(p)
    sb = gen(8, ebno_to_no(4.0))
    eng = CGNNEngine(spec, W.load(config))
    pe = torch.from_numpy(compute_pe(p.num_tx, p.num_subcarriers, p.dmrs_symbols, p.cdm_group)).cuda()
    llr, _ = eng.forward(sb.y, pe, sb.h_hat, sb.active, mcs_mask=sb.mcs_mask if spec.num_mcs > 1 else None,
                         want_h=False)
    counts = count_errors(llr, sb.bits, sb.active, sb.mcs, p.mcs_bits, p.dmrs_symbols)
    counts = count_errors(llr, sb.bits, sb.active, sb.mcs, p.mcs_bits, p.dmrs_symbols, counts=counts)  # accumulates
    torch.cuda.synchronize()
    ref = S.count_errors(llr.cpu().numpy(), sb.bits.cpu().numpy(), sb.mcs.cpu().numpy(), p.mcs_bits,
                         sb.active.cpu().numpy(), p.dmrs_symbols)
    np.testing.assert_array_equal(counts.cpu().numpy(), 2 * ref)
    assert ref[:, 3].sum() == 8                     # one active port per slot
    assert ref[:, 0].sum() > 0                      # 4 dB: errors present


@pytest.mark.parametrize("batch,heads,bs", [(100, 1, 4), (2085, 3, 6), (33, 2, 8), (50, 1, 2), (40, 1, 5)])
def test_error_counters_many_slots(batch, heads, bs):
    """Workgroups that own several slots (G = 32 slot groups per user) and more than one
    64-slot pass (batch 2085), per-slot MCS heads, random activity; synthetic LLRs (some
    exactly 0, which decide 0) against the oracle's counters."""
    import torch
    from neural_rx_amd.generator import count_errors
    rng = np.random.default_rng(batch)
    U, F, T = 2, 12, 14
    mcs_bits = [2, 4, 6][:heads] if heads > 1 else [bs if bs <= 6 else 4]
    llr = rng.standard_normal((heads, batch, U, F, T, bs)).astype(np.float32)
    llr[rng.random(llr.shape) < 0.05] = 0.0
    bits = (rng.random((batch, U, F, T, bs)) < 0.5).astype(np.uint8)
    active = (rng.random((batch, U)) < 0.7).astype(np.float32)
    mcs = rng.integers(0, len(mcs_bits), (batch, U)).astype(np.uint8)
    dmrs = [2, 11]
    t = lambda a: torch.from_numpy(a).cuda()
    counts = count_errors(t(llr), t(bits), t(active), t(mcs), mcs_bits, dmrs)
    torch.cuda.synchronize()
    ref = S.count_errors(llr, bits, mcs, mcs_bits, active, dmrs)
    np.testing.assert_array_equal(counts.cpu().numpy(), ref)


def test_sim_ber_loop():
    from neural_rx_amd import weights as W
    from neural_rx_amd.evaluate import sim_ber
    from neural_rx_amd.generator import GenParams, SlotGenerator
    from neural_rx_amd.receiver import CGNNEngine, spec_for
    eng = CGNNEngine(spec_for("nrx_rt"), W.load("nrx_rt"))
    gen = SlotGenerator(GenParams.from_config("nrx_rt", seed=4))
    r = sim_ber(eng, gen, [0.0, 8.0, 16.0], batch_size=32, max_mc_iter=4, num_target_block_errors=10**9,
                early_stop=False, num_it=2)
    assert r.mc_iters == [4, 4, 4]
    assert r.counts[0][3] == 4 * 32 * 2
    assert r.ber[0] > r.ber[1] > r.ber[2]
    assert r.ber[2] < 1e-2 and r.ber[0] > 5e-2
    # target block errors stop a point early -- tested at each counter reduction, i.e. every
    # sync_every batches (one host sync / all-reduce per window)
    r2 = sim_ber(eng, gen, [0.0], batch_size=32, max_mc_iter=50, num_target_block_errors=1, sync_every=1)
    assert r2.mc_iters == [1]
    r3 = sim_ber(eng, gen, [0.0], batch_size=32, max_mc_iter=50, num_target_block_errors=1, sync_every=8)
    assert r3.mc_iters == [8]
