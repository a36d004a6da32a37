# Three-arm interleaved A/B/C of bench argument sets on the default bench line (ARM_A / ARM_B /
# ARM_C), REPS rounds, after an optional test file list (TESTS); each GPU step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-ab3}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-3}); do
  for arm in A B C; do
    eval args=\"\$ARM_$arm\"
    [ "$args" = "-" ] && continue
    timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline $args > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    echo "$arm [$args] $(python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'])")"
  done
done
