# A/B of two bench argument sets (AB_A / AB_B, REPS interleaved pairs, default 2) with the W-MSA
# per-stage rates of each run (the bench line's roofline.stages / roofline_bwd.stages):
#   AB_A="--opt wmsa_fwd_hg=1" AB_B="" bash tools/gpu_ab_stages.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_stages
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    if [ $arm = A ]; then args="$AB_A"; else args="$AB_B"; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 $args > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json'))
f=[(s['avg_launch_us'], s['frac']) for s in d['roofline']['stages']]; b=[(s['avg_launch_us'], s['frac']) for s in d['roofline_bwd']['stages']]
print('$arm [$args]', d['value'], d['ms_per_step'], 'fwd', d['roofline']['frac'], f, 'bwd', d['roofline_bwd']['frac'], b)" | tee -a $O/ab.txt
  done
done
