# Round-6 session-2 baseline: the default bench line, the config-5 bench line (SwinV2-B 384 w24 +
# HXE) and the large-window W-MSA per-stage timings.  Each GPU step under its own limit; stops at
# the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${BASE_OUT:-base6}
mkdir -p $O
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('T', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'])"
if [ -z "$NO_B384" ]; then
timeout -k 10 500 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 --cpu-baseline 0 > $O/b384.json 2> $O/b384.err || { tail -20 $O/b384.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b384.json')); print('B384', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'], d['roofline_bwd']['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'])"
timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 > $O/wmsa_b384.txt 2>&1 || { cat $O/wmsa_b384.txt; exit 1; }
cat $O/wmsa_b384.txt
fi
