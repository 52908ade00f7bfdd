#!/bin/bash
# Variant check on one MI355X: the fused bit-identity tests against each variant library, then
# interleaved bench rounds of the default library and the variants (one-launch forward only).
# usage: bash tools/gpu_ab_var.sh <tag> <rounds> <variant> ...
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
for v in "$@"; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$v/libnrx.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_fused.py > $O/test_$v.log 2>&1 || { tail -30 $O/test_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/test_$v.log)"
done
run() {  # name lib
  NRX_LIB_PATH=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-latency --no-e2e \
    > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()},r.get('fused_queue',{}).get('update_items_waited'))" | tee -a $O/summary.txt
}
for r in $(seq $R); do
  run def_$r $PWD/neural_rx_amd/lib/libnrx.so
  for v in "$@"; do run ${v}_$r $PWD/neural_rx_amd/lib/var/$v/libnrx.so; done
done
