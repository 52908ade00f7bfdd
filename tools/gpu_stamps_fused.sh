#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps_fused.py > gpurun_out/stamps_fused.txt 2>&1 || { tail -20 gpurun_out/stamps_fused.txt; exit 1; }
cat gpurun_out/stamps_fused.txt
NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/stamps/libnrx.so NRX_FUSED=0 NRX_STAMPS_LIB=$PWD/neural_rx_amd/lib/var/stamps/libnrx.so NRX_STAMP_LAUNCH=0 timeout -k 10 200 python tools/stamps2.py > gpurun_out/stamps_three_l0.txt 2>&1 && head -20 gpurun_out/stamps_three_l0.txt
bash tools/gpu_ab_fused.sh ab_def 2
