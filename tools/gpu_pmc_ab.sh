# PMC counters of k_update for two variant libraries (diagnostic).  usage: bash tools/gpu_pmc_ab.sh <tag> <varA> <varB>
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for n in "$@"; do
  i=0
  for P in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL"; do
    i=$((i+1))
    NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_update" -d $O/pmc_${n}_$i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/pmc_${n}_$i.log 2>&1
  done
  echo "== $n"; python tools/pmc_summary.py $O/pmc_${n}_*
done
