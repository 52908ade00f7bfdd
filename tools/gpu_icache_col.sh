# Instruction-cache counters of the column schedule (mask 28) vs the RR default (mask 1).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
IC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY"
for m in 28 1; do
  NRX_UPDATE_RR=$m timeout -s KILL 120 rocprofv3 --pmc $IC -d $O/ic_$m -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/ic_$m.log 2>&1 || exit 1
  python tools/pmc_summary.py $O/ic_$m > $O/ic_$m.txt 2>&1
  echo "mask $m"; cat $O/ic_$m.txt
done
