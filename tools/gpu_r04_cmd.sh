set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r; mkdir -p $O
for r in 1 2 3; do
  for g in direct graph; do
    F=""; [ $g = graph ] && F="--graph"
    timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-latency --no-e2e $F > $O/b_${g}_$r.json 2> $O/b_${g}_$r.err
    python -c "import json; d=json.load(open('$O/b_${g}_$r.json')); print('$g', $r, round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
  done
done
