# PMC passes for one kernel of the bench workload (usage: bash tools/prof_pmc.sh <regex> <tag> [bench args])
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RE=${1:-k_update}
TAG=${2:-upd}
shift 2 || true
ARGS="--steps 20 --warmup 3 --profile-only $*"
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAVES" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt
cat gpurun_out/pmc_${TAG}_summary.txt
