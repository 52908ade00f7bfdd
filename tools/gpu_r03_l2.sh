#!/bin/bash
# L2 hit rate of the one-launch forward and of the three-launch kernels (one TCC pass each),
# then the bench line of the current tree.  usage: bash tools/gpu_r03_l2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r03l2}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum \
  --kernel-include-regex "nrx::k_" -d $O/tcc_fused -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --profile-only > $O/tcc_fused.log 2>&1 || exit 1
NRX_FUSED=0 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum \
  --kernel-include-regex "nrx::k_" -d $O/tcc_three -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --profile-only > $O/tcc_three.log 2>&1 || exit 1
python tools/pmc_summary.py $O/tcc_fused $O/tcc_three > $O/tcc_summary.txt || exit 1
cat $O/tcc_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 bench.py --profile-only --steps 200 --warmup 20 > $O/kt.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
