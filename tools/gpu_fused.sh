#!/bin/bash
# Fused-forward check on one MI355X: k_forward vs the three-launch path (bit-identity tests),
# the cfg2 oracle test, then the bench line both ways.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py \
  "tests/test_gpu_baseline_shapes.py::test_cfg2_nrx_rt_2ue_b128" > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -3 gpurun_out/fused_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-e2e > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || exit 1
NRX_FUSED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-e2e > gpurun_out/bench_3l.json 2> gpurun_out/bench_3l.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-e2e > gpurun_out/bench_fused2.json 2>> gpurun_out/bench_fused.err || exit 1
python - <<'PY'
import json
for f in ("bench_fused", "bench_3l", "bench_fused2"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["kernel"][:10], r["avg_launch_us"], r["frac"], r["whole_forward_frac"], d["kernels"])
PY
