set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/det1
mkdir -p $O
for n in v13 v14; do for r in 1 2 3; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 120 python tools/ab_exact.py $O/out_${n}_$r.npz > $O/exact_${n}_$r.log 2>&1
done; done
for n in v13 v14; do python tools/ab_exact.py --cmp $O/out_${n}_1.npz $O/out_${n}_2.npz | head -2; python tools/ab_exact.py --cmp $O/out_${n}_1.npz $O/out_${n}_3.npz | head -2; done
python tools/ab_exact.py --cmp $O/out_v13_1.npz $O/out_v14_1.npz | head -2
