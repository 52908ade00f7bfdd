# Per-phase stamps of the column launches (NRX_STAMPS library at neural_rx_amd/lib/diag).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for L in ${LAUNCHES:-300 301 302}; do
  NRX_STAMP_COL=$L timeout -k 10 200 python tools/stamps_col.py > $O/stamps_col_$L.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/stamps_col_$L.txt
done
