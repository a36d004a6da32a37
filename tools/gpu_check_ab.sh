# All -m gpu tests + smoke, then an interleaved A/B of two bench argument sets on the default bench
# line (AB_A / AB_B, e.g. "--host-opt ln_epilogue=0" vs ""), REPS pairs; each GPU step under its own
# limit, stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-checkab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    if [ $arm = A ]; then args="$AB_A"; else args="$AB_B"; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 $args > $O/b$arm$rep.json 2> $O/b$arm$rep.err || { tail -20 $O/b$arm$rep.err; exit 1; }
    echo "$arm [$args] $(python3 -c "
import json; d=json.load(open('$O/b$arm$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'], d['mfma']['binding']['all'])")"
  done
done
