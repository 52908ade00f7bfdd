# A/B (tests, exactness, interleaved bench) followed by per-item stamps of the default build.
# usage: bash tools/gpu_ab_st.sh <tag> <varA> <varB>
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab.sh "$@"
O=gpurun_out/$1
for L in 0 1 -1; do NRX_STAMP_LAUNCH=$L timeout -k 10 200 python tools/stamps2.py 2>&1 | grep -v amdgpu.ids >> $O/st.log; done
cat $O/st.log
