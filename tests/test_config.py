"""Config parsing: built-in table vs the reference cfg files; no eval."""
import dataclasses
import os

import pytest

from neural_rx_amd.config import BUILTIN, parse_cfg, spec_from_config, mcs_to_bits
from tests.conftest import have_reference


@pytest.mark.skipif(not have_reference(), reason="reference cfg files not present")
@pytest.mark.parametrize("name", sorted(BUILTIN))
def test_builtin_matches_reference_cfg(name):
    got = parse_cfg(f"/root/reference/config/{name}.cfg")
    want = BUILTIN[name]
    diff = {f.name: (getattr(got, f.name), getattr(want, f.name))
            for f in dataclasses.fields(want) if getattr(got, f.name) != getattr(want, f.name)}
    assert not diff


def test_parse_never_evaluates(tmp_path):
    p = tmp_path / "evil.cfg"
    p.write_text("[global]\nlabel = __import__('os').system('false')\n[system]\nn_size_bwp = 4\n"
                 "num_rx_antennas = 4\nmcs_index = [14]\n[neural_receiver]\nnum_nrx_iter = 2\n"
                 "d_s = 56\nnum_units_init = [128, 128]\nnum_units_agg = [[64],[64]]\n"
                 "num_units_state = [[128,128],[128,128]]\nnum_units_readout = [128]\nmax_num_tx = 2\n"
                 "nrx_dtype = torch.float32\n")
    cfg = parse_cfg(str(p))
    assert cfg.label.startswith("__import__")          # kept as a string, never run


def test_mcs_bits_and_specs():
    assert [mcs_to_bits(m) for m in (9, 14, 19)] == [2, 4, 6]
    sp = spec_from_config(BUILTIN["nrx_large_var_mcs_64qam_masking"])
    assert sp.masking and sp.head_bits == [6] and sp.num_init == 1
    sp = spec_from_config(BUILTIN["nrx_rt_var_mcs"])
    assert sp.num_init == 2 and sp.head_bits == [2, 4]


def test_mask_pilots_rejected():
    # CGNNOFDM.forward zeroes the pilot REs of y when mask_pilots is set (neural_rx.py:828-830);
    # only the e2e configs set it and they are out of scope: the wrapper refuses them before
    # creating an engine (no GPU needed for this check)
    import dataclasses
    import pytest
    from neural_rx_amd.config import get_config
    from neural_rx_amd.receiver import NeuralReceiver
    cfg = dataclasses.replace(get_config("nrx_rt"), mask_pilots=True)
    with pytest.raises(NotImplementedError, match="mask_pilots"):
        NeuralReceiver(cfg)
