# Full round check on one MI355X: GPU parity tests, smoke, bench line, kernel-trace
# stats and FETCH/WRITE PMC passes.  usage: bash tools/gpu_round.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "nrx::k_" -d $O/pmc_$C -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/pmc_$C.log 2>&1
done
python tools/pmc_traffic.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE nrx_rt_b128_u2_p4_f16 > $O/pmc_traffic.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-latency > $O/kt_bench.json 2> $O/kt.err
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
