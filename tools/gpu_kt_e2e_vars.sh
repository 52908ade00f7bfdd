# Kernel-trace averages of the e2e generator / counter kernels for named variant libraries
# (diagnostic).  usage: bash tools/gpu_kt_e2e_vars.sh <tag> <var>...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for n in "$@"; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-latency > $O/kt_$n.log 2>&1
  python - $O/kt_$n/run_kernel_stats.csv $n <<'PY'
import csv, sys
rows = {r["Name"].replace("nrx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]: round(float(r["AverageNs"]) / 1000, 2)
        for r in csv.DictReader(open(sys.argv[1])) if "gen_" in r["Name"] or "count" in r["Name"]}
print(sys.argv[2], rows)
PY
done
