# Quick GPU iteration: parity tests, bench line, per-phase stamps of both k_update launches.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-e2e > $O/bench_drv.json 2> $O/bench_drv.err
python -c "import json; d=json.load(open('$O/bench_drv.json')); print('drv', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, d['roofline']['frac'])"
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-latency --no-e2e > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print('long', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, d['roofline']['frac'])"
timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v amdgpu.ids > $O/stamps.log
NRX_STAMP_LAUNCH=1 timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v amdgpu.ids >> $O/stamps.log
NRX_STAMP_LAUNCH=-1 timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v amdgpu.ids >> $O/stamps.log
cat $O/stamps.log
