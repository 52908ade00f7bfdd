#!/bin/bash
# Round-3 bench line + kernel traces (bench workload, Sionna-layout wrapper call).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${tag} -o kt -- \
  python3 bench.py --profile-only --steps 200 --warmup 20 > gpurun_out/kt_${tag}.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sionna_${tag} -o kt -- \
  python3 tools/trace_sionna_call.py > gpurun_out/sionna_${tag}.log 2>&1
