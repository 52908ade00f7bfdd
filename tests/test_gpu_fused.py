"""The one-launch forward (k_forward) against the three-launch forward (needs an MI355X).

k_forward runs the same per-item code as k_init / k_update, only scheduled through per-XCD
work queues with cross-workgroup dependency counters, so its outputs
must equal the three-launch path bit for bit (``fused_config(enable=False)`` selects that
path per handle).  The oracle comparison of the same launch shape is tests/test_gpu_baseline_shapes.py
(cfg2, B = 128, which takes k_forward by default).  Covered here: the bench shape, inactive
users, U = 1, U = 3 / 4 (z images with the inline combine), U = 8 (combine stages), 16
antennas, Var-IO, 8 iterations, num_it = 1 (StateInit straight into the readout stage),
repeated forwards (the
counters are reset by the last workgroup of each launch), a hipGraph replay, the sticky
timeout word staying 0, that an error word reaches the caller (CGNNEngine.check, sim_ber) and
that a second stream is refused while the first still runs.
"""
import numpy as np
import pytest

from neural_rx_amd._lib import NRX_ERR_FUSED, NRXError
from tests.helpers import make_case, run_engine
from tests.test_gpu_parity import engine_for

pytestmark = pytest.mark.gpu


def _run(case, fused: bool):
    # fused: every shape the one-launch forward applies to ("force"; the default takes it only
    # for the bench-type schedule, where it is the faster one)
    eng = engine_for(case)
    eng.fused_config(enable="force" if fused else False)
    try:
        return run_engine(case, "f16", eng)
    finally:
        eng.fused_config(enable=True)


def _took_fused(case) -> bool:
    """True when the profiler saw the one-launch kernel for this case."""
    eng = engine_for(case)
    eng.profile(True)
    _run(case, True)
    prof = eng.profile_read()
    eng.profile(False)
    return prof["forward"][0] == 1 and prof["state_update"][0] == 0


def _check_identical(case):
    assert _took_fused(case), "the case was expected to take k_forward"
    ref = _run(case, False)
    for rep in range(3):          # repeated launches: the counters reset themselves
        got = _run(case, True)
        assert np.array_equal(ref["llr_raw"], got["llr_raw"]), f"LLRs differ (repeat {rep})"
        assert np.array_equal(ref["h_hat"], got["h_hat"]), f"h_hat differs (repeat {rep})"
    assert engine_for(case).fused_status(reset=True) == 0


def test_fused_bench_shape_identical():
    _check_identical(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=31))


def test_fused_random_activity_identical():
    rng = np.random.default_rng(32)
    active = (rng.random((128, 2)) < 0.6).astype(np.float32)
    _check_identical(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=32, active=active))


def test_fused_one_user_identical():
    _check_identical(make_case("nrx_rt", batch=256, users=1, prbs=4, snr_db=12, seed=33))


def test_fused_num_it_1_identical():
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=34)
    case.num_it = 1
    _check_identical(case)


def test_fused_var_io_identical():
    # BASELINE cfg4 per-GPU shard: Var-IO (two accumulating StateInit stages, two LLR heads
    # staged in the strip image at the readout), random MCS per (slot, user)
    rng = np.random.default_rng(39)
    mcs = rng.integers(0, 2, size=(128, 2))
    _check_identical(make_case("nrx_rt_var_mcs", batch=128, users=2, prbs=4, snr_db=12, seed=39, mcs_choice=mcs))


def test_fused_four_users_16_antennas_identical():
    # cfg3's topology at a small width: U = 4 (z images with the inline leave-one-out combine
    # of three planes), 16 antennas (StateInit K = 66, ChEst head of 32 outputs in the strip
    # image), 8 iterations, seeded weights, some users inactive
    rng = np.random.default_rng(40)
    active = (rng.random((64, 4)) < 0.8).astype(np.float32)
    _check_identical(make_case("nrx_large", batch=64, users=4, prbs=4, num_rx_ant=16, seeded_weights=True,
                               random_inputs=True, seed=40, active=active))


def test_fused_eight_users_combine_identical():
    # cfg5's user count: U = 8 > 4, so a combine stage (k_combine's pass, one item per (slot,
    # strip)) runs before every update and conv1 reads the combined a_u planes; 64-QAM,
    # 8 iterations, some users inactive
    rng = np.random.default_rng(42)
    active = (rng.random((32, 8)) < 0.8).astype(np.float32)
    _check_identical(make_case("nrx_large_64qam", batch=32, users=8, prbs=4, snr_db=20, seed=42, active=active))


def test_fused_three_users_identical():
    _check_identical(make_case("nrx_rt", batch=96, users=3, prbs=4, snr_db=12, seed=41))


def test_fused_8_iterations_identical():
    # BASELINE cfg4' per-GPU shard: the masking model, 8 iterations (nine stages), 6-bit head
    rng = np.random.default_rng(40)
    mcs = rng.integers(0, 3, size=(128, 2))
    _check_identical(make_case("nrx_large_var_mcs_64qam_masking", batch=128, users=2, prbs=4, snr_db=22, seed=40,
                               mcs_choice=mcs))


def test_fused_odd_batch_identical():
    # B not a multiple of the 8 queues: queues hold 17 or 16 slots
    _check_identical(make_case("nrx_rt", batch=131, users=2, prbs=4, snr_db=12, seed=35))


def test_fused_graph_replay():
    import torch
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=36)
    ref = _run(case, False)
    eng = engine_for(case)
    dev = "cuda:0"
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    args = (t(case.y), t(case.pe), t(case.h_hat), t(case.active), t(case.mcs_mask))
    eng.fused_config(enable="force")
    try:
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            eng.forward(*args, num_it=None, precision="f16")    # warm-up (workspace allocation)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            llr, h = eng.forward(*args, num_it=None, precision="f16")
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    finally:
        eng.fused_config(enable=True)
    assert np.array_equal(ref["llr_raw"], llr.cpu().numpy())
    assert eng.fused_status(reset=True) == 0


def _device_args(case):
    import torch
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to("cuda:0")  # noqa: E731
    return (t(case.y), t(case.pe), t(case.h_hat), t(case.active), t(case.mcs_mask))


def test_fused_error_reaches_caller():
    """An error word set in the one-launch forward (injected through the test hook) is raised
    by CGNNEngine.check / NeuralReceiver.check as NRX_ERR_FUSED, not returned as NRX_OK LLRs."""
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=37)
    eng = engine_for(case)
    eng.check()                                   # clean before
    args = _device_args(case)
    eng.fused_config(enable="force", inject_err=4)
    try:
        eng.forward(*args, num_it=None, precision="f16")
        with pytest.raises(NRXError) as ei:
            eng.check()
        assert ei.value.code == NRX_ERR_FUSED
        eng.fused_config(enable="force", inject_err=0)
        eng.forward(*args, num_it=None, precision="f16")
        eng.check()                               # cleared by the failed check, clean again
    finally:
        eng.fused_config(enable=True, inject_err=0)


def test_fused_error_raised_by_sim_ber():
    """sim_ber checks the error word at every reduction window."""
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import get_config, spec_from_config
    from neural_rx_amd.evaluate import sim_ber
    from neural_rx_amd.generator import GenParams, SlotGenerator
    from neural_rx_amd.receiver import CGNNEngine
    cfg = get_config("nrx_rt")
    eng = CGNNEngine(spec_from_config(cfg), W.load(cfg.label), 0)
    eng.fused_config(enable="force")
    gen = SlotGenerator(GenParams.from_config(cfg, num_tx=2, num_prbs=4), device=0)
    ok = sim_ber(eng, gen, [8.0], batch_size=128, max_mc_iter=2, num_target_block_errors=10 ** 9, sync_every=2)
    assert ok.slots == 256
    eng.fused_config(enable="force", inject_err=2)
    with pytest.raises(NRXError):
        sim_ber(eng, gen, [8.0], batch_size=128, max_mc_iter=2, num_target_block_errors=10 ** 9, sync_every=2)
    eng.close()


def test_fused_second_stream_refused_while_busy():
    """One stream per handle on the one-launch path: a forward on another stream is refused
    (NRX_ERR_BUSY) while the previous forward's stream still has work; accepted once idle."""
    import torch
    from neural_rx_amd._lib import NRX_ERR_BUSY
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=38)
    eng = engine_for(case)
    eng.fused_config(enable="force")
    args = _device_args(case)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        # the forward queued behind a spin kernel (~0.1 s: the second call's host work -- output
        # and workspace allocations on a stream new to the caching allocator -- must fit inside it)
        torch.cuda._sleep(200_000_000)
        eng.forward(*args, num_it=None, precision="f16")
    with torch.cuda.stream(s2):
        with pytest.raises(NRXError) as ei:
            eng.forward(*args, num_it=None, precision="f16")
    assert ei.value.code == NRX_ERR_BUSY
    s1.synchronize()
    with torch.cuda.stream(s2):
        eng.forward(*args, num_it=None, precision="f16")
    torch.cuda.synchronize()
    eng.check()
    eng.fused_config(enable=True)



def test_fused_guard_survives_destroyed_stream():
    """The one-stream guard keeps an event of its own, not the caller's stream: after
    the first forward's stream is destroyed, a forward on a second stream runs and check()
    waits on that event, not on the dead stream handle."""
    import ctypes
    import torch
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=39)
    eng = engine_for(case)
    eng.fused_config(enable="force")
    args = _device_args(case)
    # the HIP runtime torch loaded (by its path: a second runtime in the process sees no GPUs)
    path = next(l.split()[-1] for l in open("/proc/self/maps").read().splitlines() if "libamdhip64" in l)
    hip = ctypes.CDLL(path)
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
    try:
        s1 = torch.cuda.ExternalStream(raw.value)
        with torch.cuda.stream(s1):
            eng.forward(*args, num_it=None, precision="f16")
        s1.synchronize()
        del s1
        assert hip.hipStreamDestroy(raw) == 0    # the handle's last forward stream is gone
        s2 = torch.cuda.Stream()
        with torch.cuda.stream(s2):
            eng.forward(*args, num_it=None, precision="f16")
        eng.check()
        s2.synchronize()
    finally:
        eng.fused_config(enable=True)
