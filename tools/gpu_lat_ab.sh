#!/bin/bash
# Small-grid k_forward check on one MI355X: fused bit-identity tests (throughput and small
# tiers), the oracle parity tests, then interleaved batch-1 latency rounds with the one-launch
# forward (default) and the three-launch forward (NRX_FUSED=0).
# usage: bash tools/gpu_lat_ab.sh <tag> <rounds>
set -o pipefail
O=gpurun_out/$1; R=${2:-2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name fused
  NRX_FUSED=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 100 \
    > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));l=d['p50_latency_ms'];print('$1',d['value'],{k:(v['device_p50'],v['e2e_p50']) for k,v in l.items()})" | tee -a $O/summary.txt
}
for r in $(seq $R); do
  run fused_$r 1
  run three_$r 0
done
