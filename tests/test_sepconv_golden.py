"""The oracle's separable convolution (oracle/cgnn_ref.py sepconv: Keras SeparableConv2D 3x3 SAME,
NHWC) against the reference's own torch SeparableConv2d (utils/neural_rx copy_pytorch.py:34-51,
depthwise Conv2d(groups=C, padding=k//2) then a 1x1 conv) run on every trained StateInit and
UpdateState layer of nrx_rt (tests/golden/ref_sepconv_nrx_rt.npz, made by
tests/golden/make_golden.py from the reference file; data only).  Pins the tap orientation (i along
subcarriers, j along symbols), the SAME padding and the Keras -> torch weight transposes with
reference-authored code."""
import os

import numpy as np
import pytest

from neural_rx_amd import weights as W
from neural_rx_amd.config import get_config, spec_from_config
from oracle import cgnn_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_sepconv_nrx_rt.npz")


@pytest.mark.parametrize("name,k", [("init", 0), ("init", 1), ("init", 2), ("upd", 0), ("upd", 1), ("upd", 2)])
def test_oracle_sepconv_matches_reference_module(name, k):
    g = np.load(GOLD)
    spec = spec_from_config(get_config("nrx_rt"))
    cw = cgnn_ref.split_keras_weights(W.load("nrx_rt"), spec)
    w = (cw.init[0] if name == "init" else cw.update[0])[k]
    x = np.transpose(g[f"{name}{k}_x"], (0, 2, 3, 1)).astype(np.float64)      # NCHW -> NHWC
    ref = np.transpose(g[f"{name}{k}_y"], (0, 2, 3, 1)).astype(np.float64)
    got = cgnn_ref.sepconv(x, w, relu=False)
    scale = np.abs(ref).max()
    # the reference ran in f32 (torch CPU), the oracle in f64
    assert np.abs(got - ref).max() <= 1e-5 * max(scale, 1.0), (np.abs(got - ref).max(), scale)


def test_a_transposed_tap_grid_would_fail():
    # the check has teeth: the same layer with the depthwise taps transposed (i <-> j) disagrees
    g = np.load(GOLD)
    spec = spec_from_config(get_config("nrx_rt"))
    w = cgnn_ref.split_keras_weights(W.load("nrx_rt"), spec).update[0][1]
    wt = cgnn_ref.SepConvW(np.transpose(w.dw, (1, 0, 2, 3)).copy(), w.pw, w.b)
    x = np.transpose(g["upd1_x"], (0, 2, 3, 1)).astype(np.float64)
    ref = np.transpose(g["upd1_y"], (0, 2, 3, 1)).astype(np.float64)
    assert np.abs(cgnn_ref.sepconv(x, wt, relu=False) - ref).max() > 1e-2
