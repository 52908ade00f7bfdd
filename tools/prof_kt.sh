set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --profile-only > gpurun_out/prof_kt.log 2>&1
ls -R gpurun_out/prof_kt | head -20
