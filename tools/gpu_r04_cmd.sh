set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_r04_ab.sh r04ab6 3 notests base
timeout -k 10 600 python tools/bench_configs.py --steps 20 --out $O/configs.json > $O/configs.log 2>&1
python -c "
import json
for r in json.load(open('$O/configs.json')): print(r['config'][:24], r['path'], r['default'], r['ms_per_batch'], r['frac_f16_mfma_peak'])"
