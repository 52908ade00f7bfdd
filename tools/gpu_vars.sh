# Interleaved bench rounds of named variant libraries (diagnostic).
# usage: bash tools/gpu_vars.sh <tag> <rounds> <var>...   (var 'default': the in-tree library)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for n in "$@"; do
    if [ $n = default ]; then L=""; else L=$PWD/neural_rx_amd/lib/var/$n/libnrx.so; fi
    NRX_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); print('$n', $r, round(d['value']), {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
