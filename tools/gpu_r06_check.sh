# Round-6 check of the tree on the GPU: the whole GPU suite, smoke, the default bench line and a
# kernel trace of the same command (profiles/r06).
# usage (GPU box): bash tools/gpu_r06_check.sh <tag> [nobench]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ "$2" = "nobench" ] && exit 0
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(round(d['value']), d['ms_per_step'], r['kernel'][:60], r['avg_launch_us'], r['frac'], {n: v['avg_us'] for n, v in d['kernels'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --profile-only > $O/kt.log 2>&1 || exit 1
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | cut -c1-150 | head -8
