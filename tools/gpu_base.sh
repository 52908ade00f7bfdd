# Baseline of the current tree on a fresh box: the driver's bench command, a long bench and
# per-phase stamps of both k_update launches.  usage: bash tools/gpu_base.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_drv.json 2> $O/bench_drv.err
python -c "import json; d=json.load(open('$O/bench_drv.json')); print('drv', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --steps 400 --warmup 50 --no-cpu-baseline --no-latency --no-e2e > $O/bench_long.json 2> $O/bench_long.err
python -c "import json; d=json.load(open('$O/bench_long.json')); print('long', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-e2e > $O/bench_drv2.json 2> $O/bench_drv2.err
python -c "import json; d=json.load(open('$O/bench_drv2.json')); print('drv2', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v amdgpu.ids > $O/stamps.log
NRX_STAMP_LAUNCH=1 timeout -k 10 300 python tools/stamps.py 2>&1 | grep -v amdgpu.ids >> $O/stamps.log
cat $O/stamps.log
