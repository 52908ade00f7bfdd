set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_r04_ab.sh r04ab9 3 notests nogz
