"""Slot generator: the oracle restatement pinned by known answers, the
C-ABI structs, argument validation and the closed forms the GPU kernels use.  CPU only."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from neural_rx_amd import _lib
from neural_rx_amd.config import dmrs_symbols, get_config, user_cdm_groups
from neural_rx_amd.generator import GenParams, ebno_to_no
from oracle import cgnn_ref, pe_ref
from oracle import synth_ref as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Random123 kat_vectors, philox4x32 R=10: (counter, key) -> output
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(ctr, key, want):
    got = tuple(int(w) for w in S.philox4x32(*ctr, *key))
    assert got == want


def test_philox_words_are_uniform():
    w = np.stack(S.draw(99, 5, S.STREAM_NOISE, np.arange(20000)), -1).ravel()
    u = S.uniform(w)
    assert 0 < u.min() and u.max() < 1
    assert abs(u.mean() - 0.5) < 0.005 and abs(u.var() - 1 / 12) < 0.002
    z = np.concatenate(S.box_muller(*S.draw(99, 5, S.STREAM_NOISE, np.arange(20000))[:2]))
    assert abs(z.mean()) < 0.02 and abs(z.var() - 1) < 0.03


def _spec(**kw):
    base = dict(batch=6, num_tx=2, num_subcarriers=24, num_rx_ant=4, no=ebno_to_no(10.0))
    base.update(kw)
    return S.GenSpec(**base)


def test_grid_structure():
    o = S.generate(_spec(mcs_bits=(2, 4, 6), mcs_of_user=[-1, -1]))
    dm = np.zeros(14, bool)
    dm[[2, 11]] = True
    assert not o.bits[:, :, :, dm].any()                       # DMRS symbols carry no data
    nb = np.array((2, 4, 6))[o.mcs]
    for b in range(6):
        for u in range(2):
            assert not o.bits[b, u, ..., nb[b, u]:].any()
            e = np.abs(o.x[b, u][:, ~dm]) ** 2
            if nb[b, u] == 2:
                np.testing.assert_allclose(e, 1.0)            # QPSK: constant modulus
            assert abs(e.mean() - 1.0) < 0.35                  # unit average energy
    # pilots: QPSK x sqrt(2) on the own CDM group, zeros on the other
    for u, g in enumerate((0, 1)):
        p = o.x[:, u][:, :, dm]
        np.testing.assert_allclose(np.abs(p[:, g::2]) ** 2, 2.0)
        assert not p[:, 1 - g::2].any()


def test_slot_offset_invariance():
    """Slot b of a call at offset k is slot k + b of any other split (shards agree)."""
    full = S.generate(_spec(batch=5))
    part = S.generate(_spec(batch=2, slot_offset=3))
    for name in ("y", "h_hat", "h", "active", "bits", "mcs"):
        np.testing.assert_array_equal(getattr(part, name), getattr(full, name)[3:])


def test_active_ports_are_random_and_counted():
    """E2E_Model._active_dmrs_mask (e2e_model.py:187-193): num_active ones, random places;
    inactive ports transmit nothing and get a zero channel estimate."""
    o = S.generate(_spec(batch=400, num_tx=4, num_subcarriers=12, num_rx_ant=1, cdm_group=(0, 1, 0, 1),
                         num_active=2))
    assert (o.active.sum(1) == 2).all()
    frac = o.active.mean(0)
    assert np.all(np.abs(frac - 0.5) < 0.1)
    off = o.active == 0
    assert not o.x[off].any()
    hh = o.h_hat.reshape(400, 4, -1)
    assert not hh[off].any()


def test_ls_at_pilots_is_exact():
    o = S.generate(_spec(no=0.0, max_doppler_hz=0.0))
    A = 4
    yr = o.y[..., :A] + 1j * o.y[..., A:]
    hh = o.h_hat[..., :A] + 1j * o.h_hat[..., A:]
    for u, g in enumerate((0, 1)):
        for t in (2, 11):
            for f in range(g, 24, 2):
                np.testing.assert_allclose(hh[:, u, f, t], yr[:, f, t] / o.x[:, u, f, t][:, None], rtol=1e-6)
    # noiseless, no Doppler: single-user grids see the true channel at the pilots
    o1 = S.generate(_spec(num_tx=1, cdm_group=(0,), no=0.0, max_doppler_hz=0.0))
    np.testing.assert_allclose(o1.h_hat[:, 0, 0::2, 2], o1.h[:, 0, 0::2, 2], atol=2e-6)


def _nearest_closed_form(F, syms, g):
    """The kernel's closed form (nrx_synth.hip nearest_pilot), restated."""
    fp = np.empty((F, 14), int)
    tp = np.empty((F, 14), int)
    for f in range(F):
        for t in range(14):
            fp[f, t] = f if f % 2 == g else (f - 1 if f - 1 >= 0 else f + 1)
            d = [abs(t - s) for s in syms]
            tp[f, t] = syms[int(np.argmin(d))]
    return fp, tp


@pytest.mark.parametrize("F,syms", [(24, (2, 11)), (13, (2,)), (48, (2, 7, 11)), (36, (2, 5, 8, 11))])
@pytest.mark.parametrize("g", [0, 1])
def test_nearest_pilot_closed_form_equals_argmin(F, syms, g):
    a = S.nearest_pilot(F, syms, g)
    b = _nearest_closed_form(F, syms, g)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_ebno_to_no_follows_e2e_model():
    # e2e_model.py:323-332 with 2 of 14 symbols pilots
    assert ebno_to_no(4.0) == pytest.approx(10 ** (-(4.0 - 10 * np.log10(12 / 14)) / 10))
    assert ebno_to_no(4.0) == S.ebno_to_no(4.0)


def test_count_errors_oracle():
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2, size=(3, 2, 12, 14, 4)).astype(np.uint8)
    bits[:, :, :, [2, 11]] = 0
    llr = np.where(bits > 0, 3.0, -3.0)[None].astype(np.float32)
    llr[0, 0, 0, 5, 0, 1] *= -1           # one error, slot 0 user 0
    llr[0, 1, 1, 2, 2, 0] *= -1           # on a DMRS symbol: not counted
    act = np.array([[1, 1], [1, 0], [1, 1]], np.float32)
    c = S.count_errors(llr, bits, np.zeros((3, 2), np.uint8), (4,), act, (2, 11))
    assert c.tolist() == [[1, 3 * 12 * 12 * 4, 1, 3], [0, 2 * 12 * 12 * 4, 0, 2]]


def test_generated_slots_decode_with_trained_weights():
    """The oracle CGNN (trained nrx_rt weights) decodes generator slots: the generator
    produces what the network was trained on (DMRS layout, PE, LS h_hat, normalisation)."""
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import spec_from_config
    cfg = get_config("nrx_rt")
    spec = spec_from_config(cfg)
    s = S.GenSpec(batch=2, num_tx=2, num_subcarriers=48, num_rx_ant=4, no=ebno_to_no(14.0), seed=7)
    o = S.generate(s)
    pe = pe_ref.pe_for_groups(48, 14, dmrs_symbols(cfg), user_cdm_groups(cfg, 2))
    w = cgnn_ref.split_keras_weights(W.load("nrx_rt"), spec)
    ref = cgnn_ref.cgnn_forward(o.y, pe, o.h_hat, o.active, np.ones((2, 2, 1), np.float32), w, spec,
                                dtype=np.float32)
    llr = np.asarray(ref["llr"][0])[None]
    c = S.count_errors(llr, o.bits, o.mcs, (4,), o.active, (2, 11))
    ber = c[:, 0].sum() / c[:, 1].sum()
    assert ber < 0.02, ber


# ------------------------------------------------------------------ C ABI (no GPU needed)
@pytest.fixture(scope="module")
def lib():
    from neural_rx_amd import build
    build.build(verbose=False)
    return _lib.load()


_C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "nrx.h"
#define F(T, m) printf(#T " " #m " %zu\n", offsetof(T, m));
int main(void) {
  printf("nrx_gen_desc size %zu\n", sizeof(nrx_gen_desc));
  printf("nrx_gen_out size %zu\n", sizeof(nrx_gen_out));
  printf("nrx_count_io size %zu\n", sizeof(nrx_count_io));
  %FIELDS%
  return 0;
}
"""


def test_ctypes_structs_match_header(tmp_path):
    structs = {"nrx_gen_desc": _lib.nrx_gen_desc, "nrx_gen_out": _lib.nrx_gen_out,
               "nrx_count_io": _lib.nrx_count_io}
    fields = "\n".join(f"F({n}, {f})" for n, cls in structs.items() for f, _ in cls._fields_)
    src = tmp_path / "layout.c"
    src.write_text(_C_LAYOUT.replace("%FIELDS%", fields))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for n, cls in structs.items():
        assert got[(n, "size")] == ctypes.sizeof(cls), n
        for f, _ in cls._fields_:
            assert got[(n, f)] == getattr(cls, f).offset, (n, f)


def test_generator_validates_arguments(lib):
    p = GenParams.from_config("nrx_rt")
    d = p.desc(4, 0.1)
    n = ctypes.c_size_t()
    assert lib.nrx_gen_workspace_size(ctypes.byref(d), ctypes.byref(n)) == 0
    assert n.value >= 4 * 2 * 48 * 14 * 16
    bad = [("num_active", 3), ("num_taps", 9), ("dmrs_symbol_mask", 1), ("num_symbols", 12),
           ("num_tx", 17), ("slot_offset", -1)]
    for field, val in bad:
        d2 = p.desc(4, 0.1)
        setattr(d2, field, val)
        assert lib.nrx_gen_workspace_size(ctypes.byref(d2), ctypes.byref(n)) < 0, field
    d2 = p.desc(4, 0.1)
    d2.mcs_bits[0] = 3
    assert lib.nrx_gen_workspace_size(ctypes.byref(d2), ctypes.byref(n)) == -1
    assert b"mcs_bits" in lib.nrx_last_error()
    o = _lib.nrx_gen_out()
    assert lib.nrx_generate_slots(ctypes.byref(d), ctypes.byref(o), None, 0, None) == -1
    c = _lib.nrx_count_io()
    assert lib.nrx_count_errors(ctypes.byref(c), None) == -1


def test_params_from_config():
    p = GenParams.from_config("nrx_large_64qam", num_tx=8, num_prbs=2)
    assert p.cdm_group == user_cdm_groups(get_config("nrx_large_64qam"), 8)
    assert p.mcs_bits == (6,) and p.num_subcarriers == 24
    v = GenParams.from_config("nrx_rt_var_mcs", var_mcs=True)
    assert v.mcs_bits == (2, 4) and list(v.mcs_of_user) == [-1, -1]
