# Per-kernel trace averages (rocprofv3 --kernel-trace --stats) of named variant libraries,
# interleaved rounds (diagnostic).  usage: bash tools/gpu_kt_vars.sh <tag> <rounds> <var>...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for n in "$@"; do
    NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${n}_$r -o run --output-format csv -- python bench.py --steps 300 --warmup 30 --profile-only > $O/kt_${n}_$r.log 2>&1
    python - $O/kt_${n}_$r/run_kernel_stats.csv $n $r <<'PY'
import csv, sys
rows = {r["Name"]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(sys.argv[1])) if "nrx::k_" in r["Name"]}
short = {k.split("(")[0].replace("void nrx::", "").replace("nrx::", ""): round(v, 2) for k, v in rows.items()}
print(sys.argv[2], sys.argv[3], short)
PY
  done
done
