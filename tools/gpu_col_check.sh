# Column launches on the GPU: their bit-identity / oracle tests, then interleaved short bench
# rounds over schedule masks (NRX_UPDATE_RR), then kernel traces of the masks in KT.
# usage (GPU box): [MASKS="1 28"] [KT="1 28"] bash tools/gpu_col_check.sh <tag> [rounds] [full]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=${2:-2}; mkdir -p $O
export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_col.py -x -v --timeout 150 --timeout-method thread > $O/pytest_col.log 2>&1
rc=$?; [ -n "$NOTEST" ] || { tail -4 $O/pytest_col.log; [ $rc -eq 0 ] || exit $rc; }
if [ "$3" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $R); do
  for m in ${MASKS:-1 28}; do
    NRX_UPDATE_RR=$m timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_m${m}_$r.json 2> $O/bench_m${m}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_m${m}_$r.json')); r=d['roofline']; k=d['kernels']; print('mask $m', round(d['value']), r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in k.items()})"
  done
done
for m in ${KT:-1 28}; do
  NRX_UPDATE_RR=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$m -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --profile-only > $O/kt$m.log 2>&1 || exit 1
  echo "mask $m"; find $O/kt$m -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | cut -c1-150 | head -8
done
