#!/bin/bash
# Round-end check of the committed tree on one MI355X: GPU tests, smoke, kernel-trace stats of
# the bench workload, the default bench line.  usage: bash tools/gpu_r03_end.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r03end}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 bench.py --profile-only --steps 200 --warmup 20 > $O/kt.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
