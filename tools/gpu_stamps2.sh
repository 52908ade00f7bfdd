set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/st1; mkdir -p $O
for L in 0 1 -1; do NRX_STAMP_LAUNCH=$L timeout -k 10 200 python tools/stamps2.py 2>&1 | grep -v amdgpu.ids >> $O/st.log; done
cat $O/st.log
