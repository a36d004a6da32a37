# per-stage W-MSA forward rates on the SwinV2-B 224 + multitask bench (config 4) for env variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stages
for rep in 1 2; do for v in $VARIANTS; do
  env ${v//,/ } timeout -k 10 300 python bench.py --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/stages/b.json 2> gpurun_out/stages/b.err || { tail -20 gpurun_out/stages/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/stages/b.json')); r=d['roofline']
print('$v', d['value'], d['ms_per_step'], r['frac'], ' '.join('%.1f/%.3f' % (s['avg_launch_us'], s['frac']) for s in r['stages']))"
done; done 2>&1 | tee gpurun_out/stages/stages_b224.txt
