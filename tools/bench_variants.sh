# Time every variant library under neural_rx_amd/lib/var/ (diagnostic only).
# usage (on the GPU box): bash tools/bench_variants.sh <tag> [steps]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for d in neural_rx_amd/lib/var/*/; do
  n=$(basename $d)
  NRX_LIB_PATH=$PWD/$d/libnrx.so timeout -k 10 200 python bench.py --steps ${2:-200} --warmup 20 --no-cpu-baseline --no-latency > $O/bench_$n.json 2> $O/bench_$n.err
  python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', round(d['value']), {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
