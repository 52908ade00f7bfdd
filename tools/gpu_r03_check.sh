#!/bin/bash
# Re-entry check on one MI355X: full GPU test suite, smoke, then interleaved bench rounds of the
# one-launch forward (default) against the three-launch path (NRX_FUSED=0).
set -o pipefail
O=gpurun_out/${1:-r03chk}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/gpu_ab_fused.sh ${1:-r03chk}/ab 2
