"""The static pickle reader reproduces the committed weights and refuses code."""
import os
import pickle

import numpy as np
import pytest

from tests.conftest import have_reference

import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import convert_weights  # noqa: E402


@pytest.mark.skipif(not have_reference(), reason="reference weights not present")
def test_static_reader_matches_committed_npz():
    from neural_rx_amd import weights as W
    arrs = convert_weights.read_weight_list("/root/reference/weights/nrx_rt_weights")
    ref = W.load("nrx_rt")
    assert len(arrs) == len(ref) == 43
    for a, b in zip(arrs, ref):
        np.testing.assert_array_equal(a.astype(np.float32), b)


def test_reader_roundtrip_and_refuses_globals(tmp_path):
    arrs = [np.arange(6, dtype=np.float32).reshape(2, 3), np.ones(4, np.float32)]
    p = tmp_path / "w"
    p.write_bytes(pickle.dumps(arrs, protocol=4))       # written by this test, not the reference
    got = convert_weights.read_weight_list(str(p))
    for a, b in zip(arrs, got):
        np.testing.assert_array_equal(a, b)
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    q = tmp_path / "evil"
    q.write_bytes(pickle.dumps([Evil()], protocol=4))
    with pytest.raises(ValueError):
        convert_weights.read_weight_list(str(q))
