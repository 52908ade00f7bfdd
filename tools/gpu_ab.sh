# GPU parity tests with the default library, bit-exactness of two variants and interleaved
# A/B bench rounds.  usage: bash tools/gpu_ab.sh <tag> <varA> <varB>
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
A=${2:-nodma}
B=${3:-dma}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for n in $A $B; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 200 python tools/ab_exact.py $O/out_$n.npz > $O/exact_$n.log 2>&1
done
python tools/ab_exact.py --cmp $O/out_$A.npz $O/out_$B.npz
for r in 1 2 3; do
  for n in $A $B; do
    NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err
    python -c "import json; d=json.load(open('$O/bench_${n}_$r.json')); print('$n', $r, round(d['value']), {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
