#  check of the tree: GPU tests, smoke, default bench line (+ optional kernel trace).
# usage (GPU box): bash tools/gpu_check.sh <tag> [kt|-] [notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
if [ "$3" != "notests" ]; then
  timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], r['frac'], r['avg_launch_us'], r.get('fused_queue'))"
if [ "$2" = "kt" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --profile-only > $O/kt.log 2>&1 || exit 1
fi
