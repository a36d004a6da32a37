# Side-stream buffers held until the join (ops.wgrad_hold) instead of record_stream: the side-stream
# / DDP / routing GPU tests, then the config-5 and default bench lines with their allocator stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${HOLD_OUT:-hold}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad_stream.py tests/test_gpu_ddp.py tests/test_gpu_bench_routing.py tests/test_gpu_steps.py -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in $(seq 1 ${REPS:-1}); do
timeout -k 10 300 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 8 --warmup 2 --cpu-baseline 0 > $O/b384_$r.json 2> $O/b384_$r.err || { tail -20 $O/b384_$r.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b384_$r.json')); print('B384', d['value'], d['ms_per_step'], d['memory'], d['roofline']['ms_per_step'], d['roofline_bwd']['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/t_$r.json 2> $O/t_$r.err || { tail -20 $O/t_$r.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/t_$r.json')); print('T', d['value'], d['ms_per_step'], d['memory'])"
done
