# Round-end GPU pass: the full round check (tests, smoke, PMC, kernel trace, bench) and the
# per-config table.  usage: bash tools/gpu_final.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh $1
timeout -k 10 600 python tools/bench_configs.py --out gpurun_out/$1/configs.json > gpurun_out/$1/configs.log 2>&1
tail -6 gpurun_out/$1/configs.log
