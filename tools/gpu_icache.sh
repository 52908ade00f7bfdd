# Instruction-cache counters of the bench forward: one --pmc pass each for the default library,
# the three-launch forward (NRX_FUSED=0) and any variant libraries (lib/var/<name>).
# usage (GPU box): bash tools/gpu_icache.sh <tag> [var...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
IC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY"
for n in default three "$@"; do
  F=1; L=$PWD/neural_rx_amd/lib/libnrx.so
  [ $n = three ] && F=0
  [ $n != default ] && [ $n != three ] && L=$PWD/neural_rx_amd/lib/var/$n/libnrx.so
  NRX_FUSED=$F NRX_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $IC -d $O/ic_$n -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/ic_$n.log 2>&1 || exit 1
  python tools/pmc_summary.py $O/ic_$n > $O/ic_$n.txt 2>&1
done
