# per-stage W-MSA rates (bench line "stages") for several forward routings, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stages
for rep in 1 2; do for v in $VARIANTS; do
  env ${v//,/ } timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/stages/b.json 2> gpurun_out/stages/b.err || { tail -20 gpurun_out/stages/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/stages/b.json')); r=d['roofline']
print('$v', d['value'], d['ms_per_step'], r['frac'], ' '.join('%.1f/%.3f' % (s['avg_launch_us'], s['frac']) for s in r['stages']))"
done; done 2>&1 | tee gpurun_out/stages/stages.txt
