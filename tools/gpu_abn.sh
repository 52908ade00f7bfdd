# GPU parity tests (default library), bit-exactness of every variant against the first, and
# interleaved bench rounds.  usage: bash tools/gpu_abn.sh <tag> <rounds> <var0> <var1> ...
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for n in "$@"; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 200 python tools/ab_exact.py $O/out_$n.npz > $O/exact_$n.log 2>&1
done
for n in "${@:2}"; do echo "== $1 vs $n"; python tools/ab_exact.py --cmp $O/out_$1.npz $O/out_$n.npz; done
bash tools/gpu_vars.sh $(basename $O)_b $R "$@"
