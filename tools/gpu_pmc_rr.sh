# SQ issue/stall breakdown of the update kernels (both stages register-resident, NRX_UPDATE_RR=3,
# and the strip kernels, =0) at the bench shape: two --pmc passes each, separate runs.
# usage (GPU box): bash tools/gpu_pmc_rr.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for m in 3 0; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    NRX_UPDATE_RR=$m timeout -s KILL 90 rocprofv3 --pmc $P -d $O/m${m}_p$i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/m${m}_p$i.log 2>&1 || exit 1
  done
  python tools/pmc_summary.py $O/m${m}_p1 $O/m${m}_p2 > $O/m${m}_summary.txt
  grep -E "k_update" $O/m${m}_summary.txt
done
