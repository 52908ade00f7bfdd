# Same-box A/B of update-schedule masks (NRX_UPDATE_RR) at the bench shape: interleaved bench.py
# rounds.  usage (GPU box): bash tools/gpu_mask_ab.sh <tag> <rounds> <mask>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  for m in "$@"; do
    NRX_UPDATE_RR=$m timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_m${m}_$r.json 2> $O/bench_m${m}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_m${m}_$r.json')); print('mask $m', $r, round(d['value']), {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
