# RR update launch on the GPU: its tests (bit-identity vs the strip kernels, oracle), the GZ
# boundary and slot-chunk tests, optionally the whole GPU suite, then interleaved short bench
# rounds over the stage masks NRX_UPDATE_RR=0..3 and kernel traces of masks 0 (strip) and 3 (RR).
# usage (GPU box): [VARS="variant ..."] bash tools/gpu_rr_check.sh <tag> [rounds] [full]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=${2:-2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_update_rr.py tests/test_gpu_gz_boundary.py tests/test_gpu_chunks.py -x -v --timeout 150 --timeout-method thread > $O/pytest_rr.log 2>&1
rc=$?; tail -4 $O/pytest_rr.log; [ $rc -eq 0 ] || exit $rc
if [ "$3" = "full" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $R); do
  for m in ${MASKS:-0 1 2 3}; do
    NRX_UPDATE_RR=$m timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_m${m}_$r.json 2> $O/bench_m${m}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_m${m}_$r.json')); r=d['roofline']; print('mask $m', round(d['value']), r['avg_launch_us'], r['frac'], r['kernel'][:12])"
  done
  for v in $VARS; do   # variant libraries (tools/build_variants.py), mask $VMASK (default 1)
    NRX_LIB_PATH=neural_rx_amd/lib/var/$v/libnrx.so NRX_UPDATE_RR=${VMASK:-1} timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); r=d['roofline']; print('var $v', round(d['value']), r['avg_launch_us'], r['frac'], r['kernel'][:12])"
  done
done
# per-kernel durations of the strip (mask 0) and RR (mask 3) schedules
for m in 0 3; do
  NRX_UPDATE_RR=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$m -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --profile-only > $O/kt$m.log 2>&1 || exit 1
  echo "mask $m"; find $O/kt$m -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | cut -c1-150 | head -8
done
