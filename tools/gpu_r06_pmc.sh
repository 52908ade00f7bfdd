# Round-6 PMC passes (separate runs: SQ, FETCH_SIZE, WRITE_SIZE, SQ LDS/issue) of the bench forward and of cfg5's
# per-GPU shard; records profiles/pmc_traffic.json + pmc_sq.json via tools/pmc_record.py.
# usage (GPU box): bash tools/gpu_pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
i=0
for P in "$SQ" FETCH_SIZE WRITE_SIZE "$SQ2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/cfg2_p$i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/cfg2_p$i.log 2>&1 || exit 1
done
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d $O/cfg5_p$i -o run --output-format csv -- python bench.py --config nrx_large_64qam --users 8 --prbs 273 --batch 32 --steps 2 --warmup 1 --prewarm-s 0 --profile-only > $O/cfg5_p$i.log 2>&1 || exit 1
done
python tools/pmc_record.py nrx_rt_b128_u2_p4_f16 "profiles/r06/$1" $O/cfg2_p1 $O/cfg2_p2 $O/cfg2_p3 $O/cfg2_p4 > $O/record_cfg2.txt 2>&1
python tools/pmc_record.py nrx_large_64qam_b32_u8_p273_f16 "profiles/r06/$1" $O/cfg5_p1 $O/cfg5_p2 > $O/record_cfg5.txt 2>&1
cp profiles/pmc_traffic.json profiles/pmc_sq.json $O/ 2>/dev/null
python tools/pmc_summary.py $O/cfg2_p1 $O/cfg2_p2 $O/cfg2_p3 $O/cfg2_p4 > $O/cfg2_summary.txt
python tools/pmc_summary.py $O/cfg5_p1 $O/cfg5_p2 > $O/cfg5_summary.txt
cat $O/record_cfg2.txt | head -30
