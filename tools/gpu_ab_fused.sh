#!/bin/bash
# Interleaved same-box bench rounds: one-launch forward vs three-launch forward, default
# library vs variants.  usage: bash tools/gpu_ab_fused.sh <tag> <rounds> [variant ...]
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
run() {  # name lib fused
  NRX_LIB_PATH=$2 NRX_FUSED=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-latency --no-e2e \
    > $O/$1.json 2> $O/$1.err || { cat $O/$1.err | tail -5; exit 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()},r.get('fused_queue',{}).get('update_items_waited'))" | tee -a $O/summary.txt
}
DEF=$PWD/neural_rx_amd/lib/libnrx.so
for r in $(seq $R); do
  run fused_$r $DEF 1
  run three_$r $DEF 0
  for v in "$@"; do
    run ${v}_fused_$r $PWD/neural_rx_amd/lib/var/$v/libnrx.so 1
    run ${v}_three_$r $PWD/neural_rx_amd/lib/var/$v/libnrx.so 0
  done
done
