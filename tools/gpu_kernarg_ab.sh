set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ka1; mkdir -p $O
for r in 1 2; do
for ev in 0 1; do
  HIP_FORCE_DEV_KERNARG=$ev NRX_UPDATE_RR=28 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e > $O/b_$ev_$r.json 2> $O/b_$ev.err || exit 1
  python -c "import json; d=json.load(open('$O/b_$ev_$r.json')); k=d['kernels']; print('devkernarg $ev', round(d['value']), {n: v['avg_us'] for n, v in k.items()})"
done
done
HIP_FORCE_DEV_KERNARG=1 NRX_STAMP_COL=301 timeout -k 10 200 python tools/stamps_col.py > $O/stamps_dk1.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_dk1.txt
HIP_FORCE_DEV_KERNARG=0 NRX_STAMP_COL=301 timeout -k 10 200 python tools/stamps_col.py > $O/stamps_dk0.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_dk0.txt
