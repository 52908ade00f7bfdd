#!/bin/bash
# Round-3 capture of the one-launch forward (k_forward, the default throughput path) on one
# MI355X: FETCH/WRITE per launch (-> profiles/pmc_traffic.json via tools/pmc_traffic.py), the
# SQ/GRBM passes over k_forward, kernel-trace stats of the bench workload, the per-item
# stamps of the fused kernel (diagnostic build), then the bench line.
# usage: bash tools/gpu_r03_fwd_final.sh <tag> [skip-stamps]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03fwd}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex "nrx::k_" -d $O/pmc_$C -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --profile-only > $O/pmc_$C.log 2>&1 || exit 1
done
python tools/pmc_traffic.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE nrx_rt_b128_u2_p4_f16 profiles/$TAG/pmc_traffic.txt > $O/pmc_traffic.txt || exit 1
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAVES SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "nrx::k_forward" -d $O/pmc_fwd_$i -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --profile-only > $O/pmc_fwd_$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py $O/pmc_fwd_* > $O/pmc_fwd_summary.txt || exit 1
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 bench.py --profile-only --steps 200 --warmup 20 > $O/kt.log 2>&1 || exit 1
if [ "$2" != "skip-stamps" ]; then
  step stamps
  timeout -k 10 200 python tools/stamps_fused.py > $O/stamps_fused.txt 2>&1 || { tail -20 $O/stamps_fused.txt; exit 1; }
  cat $O/stamps_fused.txt
fi
step bench
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
