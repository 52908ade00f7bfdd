#!/bin/bash
# Same-box A/B of kernel durations: tools/gpu_ab.sh TAG LIB [TAG LIB ...] (env applies to all);
# each arm is one rocprofv3 kernel-trace of the bench workload, arms interleaved twice.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args=("$@")
for rep in 1 2; do
  for ((i = 0; i < ${#args[@]}; i += 2)); do
    tag=${args[i]}; lib=${args[i+1]}
    NRX_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/ab_${tag}_${rep} -o kt -- python3 bench.py --profile-only --steps 100 --warmup 20 \
      > gpurun_out/ab_${tag}_${rep}.log 2>&1 || exit 1
  done
done
python3 - "$@" <<'PY'
import csv, sys
a = sys.argv[1:]
for i in range(0, len(a), 2):
    tag = a[i]
    for rep in (1, 2):
        rows = list(csv.DictReader(open(f"gpurun_out/ab_{tag}_{rep}/kt_kernel_stats.csv")))
        print(tag, rep, " | ".join(f"{r['Name'][:40]} {float(r['AverageNs']) / 1e3:.2f}" for r in rows if 'rocclr' not in r['Name']))
PY
