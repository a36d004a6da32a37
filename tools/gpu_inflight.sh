# Bounded host run-ahead (Trainer.max_steps_in_flight) against unbounded: the config-5 and the
# default bench lines, each arm once, interleaved.  Each GPU step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${IF_OUT:-inflight}
mkdir -p $O
for r in $(seq 1 ${REPS:-1}); do
for arm in 2 0; do
  timeout -k 10 300 python bench.py --model swinv2_base_window24_384 --loss hxe --steps ${B384_STEPS:-8} --warmup 2 --cpu-baseline 0 --steps-in-flight $arm > $O/b384_$arm.json 2> $O/b384_$arm.err || { tail -20 $O/b384_$arm.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b384_$arm.json')); print('B384 inflight=$arm', d['value'], d['ms_per_step'], d['memory'], d['roofline']['ms_per_step'], d['roofline_bwd']['ms_per_step'])"
done
for arm in 2 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --steps-in-flight $arm > $O/t_$arm.json 2> $O/t_$arm.err || { tail -20 $O/t_$arm.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/t_$arm.json')); print('T inflight=$arm', d['value'], d['ms_per_step'], d['memory'])"
done
done
