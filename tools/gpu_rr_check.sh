#!/bin/bash
# RR kernel bring-up: the oracle tests at the bench shapes + the batch-composition
# invariance tests (RR at B >= 128 vs the small-strip tiers at B = 4, bit for bit).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-rr}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
