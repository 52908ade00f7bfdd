# Per-phase stamps of the RR update launches (NRX_STAMPS variant library), aggregation and readout.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for L in 300 301; do
  NRX_STAMP_RR=$L timeout -k 10 200 python tools/stamps_rr.py > $O/stamps_rr_$L.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/stamps_rr_$L.txt
done
