set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r04_base_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r04_base_bench.json 2> gpurun_out/r04_base_bench.err
