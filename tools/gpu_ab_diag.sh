# Same-box interleaved A/B: the in-tree library against variant libraries (tools/build_diag.py),
# short bench runs; optional NRX_UPDATE_RR mask per run (MASK).
# usage (GPU box): [MASK=29] bash tools/gpu_ab_diag.sh <tag> <rounds> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  for v in default "$@"; do
    L=$PWD/neural_rx_amd/lib/libnrx.so
    [ $v != default ] && L=$PWD/neural_rx_amd/lib/diag/$v/libnrx.so
    NRX_LIB_PATH=$L NRX_UPDATE_RR=${MASK:-29} timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', round(d['value']), d['ms_per_step'], {n: v['avg_us'] for n, v in d['kernels'].items()})"
  done
done
