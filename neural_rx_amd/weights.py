"""Trained CGNN weights shipped with the repository (``weights/*.npz``).

The arrays are the reference's Keras ``get_weights()`` lists (``weights/<label>_weights``
in the reference, loaded there by ``utils/utils.py:53-70``), converted once by
``tools/convert_weights.py`` without unpickling.  They are distributed under the
NVIDIA License (``weights/NVIDIA_LICENSE.txt``): research/evaluation use only.
"""
from __future__ import annotations

import os
from typing import List

import numpy as np

WEIGHTS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "weights")


def available() -> List[str]:
    if not os.path.isdir(WEIGHTS_DIR):
        return []
    return sorted(f[:-4] for f in os.listdir(WEIGHTS_DIR) if f.endswith(".npz"))


def load(label: str) -> List[np.ndarray]:
    path = os.path.join(WEIGHTS_DIR, f"{label}.npz")
    with np.load(path, allow_pickle=False) as d:
        return [np.ascontiguousarray(d[f"w{i:03d}"], dtype=np.float32)
                for i in range(int(d["count"]))]


def seeded(spec, seed: int = 0) -> List[np.ndarray]:
    """Random Keras-ordered weights of a topology (Glorot uniform kernels).  Used
    for BASELINE config 3 (16 rx antennas), for which no trained weights exist."""
    rng = np.random.default_rng(seed)
    out: List[np.ndarray] = []

    def glorot(shape, fan_in, fan_out):
        lim = np.sqrt(6.0 / (fan_in + fan_out))
        return rng.uniform(-lim, lim, size=shape).astype(np.float32)

    def bias(n):
        return rng.uniform(-0.05, 0.05, size=(n,)).astype(np.float32)

    def sep(cin, cout):
        out.extend([glorot((3, 3, cin, 1), 9, 9), glorot((1, 1, cin, cout), cin, cout), bias(cout)])

    def dense(cin, cout):
        out.extend([glorot((cin, cout), cin, cout), bias(cout)])

    u1, u2 = spec.init_units
    for _ in range(spec.num_init):
        sep(spec.init_in_ch, u1)
        sep(u1, u2)
        sep(u2, spec.d_s)
    v1, v2 = spec.state_units
    for _ in range(spec.num_it):
        dense(spec.d_s, spec.agg_units)
        dense(spec.agg_units, spec.d_s)
        sep(spec.update_in_ch, v1)
        sep(v1, v2)
        sep(v2, spec.d_s)
    for nb in spec.head_bits:
        dense(spec.d_s, spec.readout_units)
        dense(spec.readout_units, nb)
    dense(spec.d_s, spec.readout_units)
    dense(spec.readout_units, 2 * spec.num_rx_ant)
    return out
