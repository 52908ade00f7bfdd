"""tools/bench_configs.py's per-kernel figures (CPU): a launch of a chunked forward is charged the
FLOPs of its slot chunk, so no kernel row can report more than the f16 MFMA peak (VERDICT r05
item 2: cfg5's update launch read 2 470 TF when the whole batch's FLOPs were divided by one
chunk's launch time)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import bench_configs as bc  # noqa: E402
from neural_rx_amd import metrics  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402


def test_slot_chunks_match_the_library_rule():
    assert bc.slot_chunks(128, 2, 48) == 1              # cfg2: one forward
    assert bc.slot_chunks(64, 4, 1584) == 3             # cfg3 shard
    assert bc.slot_chunks(32, 8, 3276) == 6             # cfg5 shard


def test_chunked_kernel_tflops_below_peak():
    spec = spec_from_config(get_config("nrx_large_64qam"))
    kfl = metrics.launch_flops_per_re_user(spec, 8)
    B, U, F, steps = 32, 8, 3276, 20
    re_users = B * U * F * 14
    chunks = bc.slot_chunks(B, U, F)
    # the r05 cfg5 profile: 6 chunks x 7 RR update launches of ~470 us per forward
    prof = {"state_update_rr": (steps * 7 * chunks, steps * 7 * chunks * 0.470),
            "state_init": (steps * chunks, steps * chunks * 0.40), "combine": (steps * 8 * chunks, steps * 8 * chunks * 0.07)}
    rows = bc.kernel_rows(prof, kfl, re_users, chunks, steps)
    peak = metrics.PEAK_TFLOPS["f16"]
    for k, r in rows.items():
        assert r["tflops"] is None or r["tflops"] <= 0.5 * peak, (k, r)
    assert 300 < rows["state_update_rr"]["tflops"] < 500, rows
    assert rows["combine"]["tflops"] is None
