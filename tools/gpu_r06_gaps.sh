set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s2; mkdir -p $O
LAUNCHES="300 301 302" bash tools/gpu_stamps_col.sh s2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python bench.py --steps 50 --warmup 5 --profile-only > $O/kt.log 2>&1 || exit 1
python tools/kt_gaps.py $O/kt/run_kernel_trace.csv | tee $O/gaps.txt
