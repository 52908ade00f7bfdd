set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ab4; mkdir -p $O
NRX_LIB_PATH=$PWD/neural_rx_amd/lib/libnrx.so timeout -k 10 120 python tools/ab_exact.py $O/out_pairs.npz > $O/exact_pairs.log 2>&1
NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/nopairs/libnrx.so timeout -k 10 120 python tools/ab_exact.py $O/out_nopairs.npz > $O/exact_nopairs.log 2>&1
python tools/ab_exact.py --cmp $O/out_pairs.npz $O/out_nopairs.npz
bash tools/gpu_r04_ab.sh r04ab4 3 notests nopairs
