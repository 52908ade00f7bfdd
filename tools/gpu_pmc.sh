# PMC passes + kernel trace of the bench workload.  usage: bash tools/gpu_pmc.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
bash tools/prof_pmc.sh "k_update|k_init" $T > /dev/null 2>&1 || { echo pmc failed; ls gpurun_out; exit 1; }
cat gpurun_out/pmc_${T}_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$T -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --profile-only > gpurun_out/kt_$T.log 2>&1
find gpurun_out/kt_$T -name "*stats*" | head; cat $(find gpurun_out/kt_$T -name "*kernel_stats.csv" | head -1)
