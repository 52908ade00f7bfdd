#!/bin/bash
# bit-identity tests of the one-launch forward + the paired path, then interleaved A/B rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_baseline_shapes.py tests/test_gpu_parity.py > gpurun_out/fused_tests.log 2>&1 || { tail -40 gpurun_out/fused_tests.log; exit 1; }
tail -3 gpurun_out/fused_tests.log
bash tools/gpu_ab_fused.sh "$@"
