# Build ablation variants of libnrx.so and time each kernel (diagnostic only).
set -e
cd $GRAFT_REPO_ROOT
for A in 0 1 2 4 8 16 31; do
  mkdir -p /tmp/abl$A
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DNRX_ABLATE=$A neural_rx_amd/csrc/nrx_kernels.hip neural_rx_amd/csrc/nrx_api.cpp -o /tmp/abl$A/libnrx.so
done
for A in 0 1 2 4 8 16 31; do
  cp /tmp/abl$A/libnrx.so neural_rx_amd/lib/libnrx.so
  echo "ABLATE=$A $(timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-latency 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k:v["avg_us"] for k,v in d["kernels"].items()})')"
done
cp /tmp/abl0/libnrx.so neural_rx_amd/lib/libnrx.so
