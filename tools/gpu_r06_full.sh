# Round-6 full check: GPU suite, smoke, default bench line + kernel trace, per-config table.
# usage (GPU box): bash tools/gpu_r06_full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r06_check.sh $1 || exit 1
O=gpurun_out/$1
timeout -k 10 800 python tools/bench_configs.py --out $O/configs.json > $O/configs.log 2>&1 || { tail -3 $O/configs.log; exit 1; }
python - <<PY
import json
for r in json.load(open("$O/configs.json")):
    print(f"{r['config'][:34]:34s} {r['path']:17s} def={r['default']!s:5s} ms={r['ms_per_batch']:8.4f} slots/s={r['slots_per_s_per_gpu']:10.1f} frac={r['frac_f16_mfma_peak']}")
PY
