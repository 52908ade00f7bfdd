set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python tools/diag_rr.py > $O/diag.txt 2>&1; rc=$?; cat $O/diag.txt | grep -v amdgpu.ids; exit $rc
