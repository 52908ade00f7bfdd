# Per-phase stamps (tools/stamps2.py) of named NRX_STAMPS variant builds for one launch.
# usage: bash tools/gpu_stamps_vars.sh <tag> <launch> <var>...
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; L=$2; shift 2
mkdir -p $O
for n in "$@"; do
  echo "== $n" >> $O/st.log
  NRX_STAMPS_LIB=$PWD/neural_rx_amd/lib/var/$n/libnrx.so NRX_STAMP_LAUNCH=$L timeout -k 10 200 python tools/stamps2.py 2>&1 | grep -v amdgpu.ids >> $O/st.log
done
cat $O/st.log
