"""The C-ABI library loads and exports every symbol include/nrx.h declares; host-side
entry points (no GPU compute) behave as documented."""
import ctypes
import os
import re

import numpy as np
import pytest

from neural_rx_amd import _lib
from neural_rx_amd import metrics
from neural_rx_amd.config import BUILTIN, get_config, spec_from_config
from oracle import cgnn_ref, pe_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "nrx.h")).read()
    return sorted(set(re.findall(r"\b(nrx_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from neural_rx_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTS)
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.nrx_api_version() == 7


@pytest.mark.parametrize("name", sorted(BUILTIN))
def test_weight_layout_matches_keras_order(lib, name):
    spec = spec_from_config(get_config(name))
    d = _lib.make_desc(spec)
    n = ctypes.c_int32()
    assert lib.nrx_weight_layout(ctypes.byref(d), ctypes.byref(n), None, 0) == 0
    sizes = (ctypes.c_int64 * n.value)()
    assert lib.nrx_weight_layout(ctypes.byref(d), ctypes.byref(n), sizes, n.value) == 0
    from neural_rx_amd import weights as W
    assert list(sizes) == [a.size for a in W.load(name)]


def test_flops_formula(lib):
    spec = spec_from_config(get_config("nrx_rt"))
    d = _lib.make_desc(spec)
    # 282 956 FLOP per RE-user for nrx_rt
    assert lib.nrx_flops_per_re_user(ctypes.byref(d), 2) == 282956
    assert metrics.forward_flops_per_re_user(spec, 2) == 282956


@pytest.mark.parametrize("groups,F", [((0, 1), 48), ((0, 1, 0, 1), 1584), ((1,), 36), ((0, 1, 0, 1, 0, 1, 0, 1), 12)])
def test_product_pe_matches_oracle(lib, groups, F):
    from neural_rx_amd.receiver import compute_pe
    pe = compute_pe(len(groups), F, (2, 11), groups)
    np.testing.assert_allclose(pe, pe_ref.pe_for_groups(F, 14, (2, 11), groups), atol=1e-6)


def test_invalid_topology_is_rejected(lib):
    spec = spec_from_config(get_config("nrx_rt"))
    d = _lib.make_desc(spec)
    d.d_s = 32
    n = ctypes.c_int32()
    rc = lib.nrx_weight_layout(ctypes.byref(d), ctypes.byref(n), None, 0)
    assert rc == -3
    assert b"d_s" in lib.nrx_last_error()
    assert lib.nrx_forward(None, None, None, 0, None) == -1


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.NRXLibraryError):
        _lib.load(str(tmp_path / "nope.so"))
