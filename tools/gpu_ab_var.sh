# Same-box A/B of the default library against one variant library (tools/build_variants.py):
# interleaved bench.py rounds (per-kernel times) and, optionally, bench_configs over a config.
# usage (GPU box): bash tools/gpu_ab_var.sh <tag> <variant> [rounds] [config substring]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; V=$2; R=${3:-2}; mkdir -p $O
for r in $(seq 1 $R); do
  for v in default $V; do
    if [ $v = default ]; then L=""; else L="neural_rx_amd/lib/var/$v/libnrx.so"; fi
    NRX_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); k=d['kernels']; print('$v', round(d['value']), {n: v['avg_us'] for n, v in k.items()})"
    if [ -n "$4" ]; then
      NRX_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_configs.py --steps 10 --only "$4" --out $O/cfg_${v}_$r.json > $O/cfg_${v}_$r.log 2>&1 || exit 1
      python -c "
import json
for x in json.load(open('$O/cfg_${v}_$r.json')): print('  $v', x['path'], x['slots_per_s_per_gpu'], {n: v['avg_us'] for n, v in x['kernels'].items()})"
    fi
  done
done
