#!/bin/bash
# Round-3 GPU check: the full -m gpu suite, then the bench line and a kernel trace of the
# Sionna-layout wrapper call.  Every GPU step has its own time limit; steps chained by &&.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/pytest_gpu_${tag}.log 2>&1
