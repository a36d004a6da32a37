# Fused-LN-epilogue diagnostic, then an interleaved A/B of AB_A / AB_B bench argument sets (no test run).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-diagab}
mkdir -p $O
timeout -k 10 120 python -u tools/diag_lnepi.py > $O/diag.log 2>&1 || { tail -30 $O/diag.log; exit 1; }
cat $O/diag.log
for rep in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    if [ $arm = A ]; then args="$AB_A"; else args="$AB_B"; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 $args > $O/b$arm$rep.json 2> $O/b$arm$rep.err || { tail -20 $O/b$arm$rep.err; exit 1; }
    echo "$arm [$args] $(python3 -c "
import json; d=json.load(open('$O/b$arm$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'], d['mfma']['binding']['all'])")"
  done
done
