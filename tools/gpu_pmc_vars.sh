# One PMC pass (instruction mix + cycles) of k_update / k_init for each named variant (diagnostic).
# usage: [PMC="counters"] bash tools/gpu_pmc_vars.sh <tag> <var>...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for n in "$@"; do
  NRX_LIB_PATH=$PWD/neural_rx_amd/lib/var/$n/libnrx.so timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE} --kernel-include-regex "k_update|k_init" -d $O/pmc_${n}${SFX:-} -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --profile-only > $O/pmc_${n}${SFX:-}.log 2>&1
  echo "== $n"; python tools/pmc_summary.py $O/pmc_${n}${SFX:-} | sed 's/void nrx::k_//'
done
