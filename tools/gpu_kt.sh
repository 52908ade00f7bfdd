#!/bin/bash
# Kernel-trace stats of the bench workload (short): per-kernel average durations.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-kt}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${tag} -o kt -- \
  python3 bench.py --profile-only --steps 100 --warmup 20 > gpurun_out/kt_${tag}.log 2>&1 && \
cut -d, -f1-4 gpurun_out/kt_${tag}/kt_kernel_stats.csv | head -6
