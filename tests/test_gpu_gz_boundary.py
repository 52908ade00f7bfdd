"""The GZ z-row loader at its edges.

conv1 of a GZ update item reads its z rows [a | s | pe] with raw buffer loads through one
descriptor spanning the workspace (nrx_device.inc, struct GZ): lanes with nothing to read (pad
symbols, chunk 15, the missing other user of U = 1) carry an out-of-range voffset, and grid
rows outside [0, F) an out-of-range soffset.  Both rely on the descriptor's range check
returning zeros.  The first test probes that check on the device for both operands with every
address kept inside one allocation (no outcome can fault); the second runs the boundary the
check protects: the last strip of the last slot, F not a multiple of 24, U = 1, the workspace
exactly sized (a fresh engine), against the fp64 oracle."""
import ctypes

import numpy as np
import pytest

from tests.helpers import compare, make_case, run_engine, run_oracle

pytestmark = pytest.mark.gpu


def test_buffer_range_check_covers_voffset_and_soffset():
    import torch
    from neural_rx_amd import _lib
    lib = _lib.load()
    lib.nrx_probe_buffer_oob.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_void_p]
    buf = torch.full(((8 << 20) // 4,), 0x11223344, dtype=torch.int32, device="cuda:0")   # 8 MB, marker words
    out = torch.zeros(64, dtype=torch.int32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    marker = 0x11223344

    def probe(records, voff, soff):
        out.zero_()
        assert lib.nrx_probe_buffer_oob(buf.data_ptr(), records, voff, soff, out.data_ptr(), stream) == 0
        torch.cuda.synchronize()
        return out.cpu().numpy()

    mb = 1 << 20
    assert (probe(mb, 64, 4096) == marker).all()          # in range: the data
    assert (probe(mb, 2 * mb, 0) == 0).all()              # voffset beyond records: zeros
    assert (probe(mb, 0, 2 * mb) == 0).all()              # soffset beyond records: zeros (GZ's kGzOob rows)
    edge = probe(mb, mb - 128, 0)                        # a wave straddling the end: lanes 0-31 in range
    assert (edge[:32] == marker).all() and (edge[32:] == 0).all()


def test_gz_last_strip_last_slot_f_not_multiple_of_24_u1():
    # F = 36 (3 PRB): two 24-row strips, the second with rows 36..47 and its halo outside the grid;
    # U = 1 (the a chunks are out of range); B = 160 gives 320 items > 256 CUs, so the 24-row tier
    # (GZ) runs, not the small-strip tiers
    from neural_rx_amd.receiver import CGNNEngine
    case = make_case("nrx_rt", batch=160, users=1, prbs=3, snr_db=15, seed=41)
    eng = CGNNEngine(case.spec, case.weights)          # fresh: workspace allocated at the exact size
    try:
        got = run_engine(case, "f16", eng)
        assert eng._ws["buf"].numel() == eng.workspace_bytes(160, 1, 36)
    finally:
        eng.close()
    ref = run_oracle(case)
    c = compare(ref, got)
    assert np.isfinite(got["llr_raw"]).all() and np.isfinite(got["h_hat"]).all()
    assert c["llr_rms_rel"] < 0.02 and c["flip_rate_confident"] <= 1e-3, c
    # the last slot's last strip on its own: the rows where the halo leaves the grid
    last = compare({"llr": [r[-1:, :, 24:] for r in ref["llr"]], "h_hat": ref["h_hat"][-1:, :, 24:]},
                   {"llr": [g[-1:, :, 24:] for g in got["llr"]], "h_hat": got["h_hat"][-1:, :, 24:]})
    assert last["llr_rms_rel"] < 0.02 and last["flip_rate_confident"] <= 1e-3, last
