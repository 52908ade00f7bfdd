# GPU tests + smoke on the default library, then interleaved short bench rounds of the default
# library and named variant libraries (neural_rx_amd/lib/var/<name>/libnrx.so).
# variant "three" = the default library with NRX_FUSED=0 (three-launch forward).
# usage (GPU box): bash tools/gpu_r04_ab.sh <tag> <rounds> [notests] <var>...
set -o pipefail
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
export TMPDIR=/tmp
if [ "$1" = "notests" ]; then shift; else
  timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
for r in $(seq 1 $R); do
  for n in default "$@"; do
    # variant "three": the default library with the one-launch forward disabled
    F=1
    if [ $n = default ] || [ $n = three ]; then L=$PWD/neural_rx_amd/lib/libnrx.so; else L=$PWD/neural_rx_amd/lib/var/$n/libnrx.so; fi
    if [ $n = three ]; then F=0; fi
    NRX_FUSED=$F NRX_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); r=d['roofline']; print('$n', $r, round(d['value']), r['avg_launch_us'], r['frac'], r.get('fused_queue', {}).get('update_items_waited'))"
  done
done
