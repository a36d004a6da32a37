# Config-5 (SwinV2-B 384 w24 + HXE) step diagnosis: the bench line as shipped, then with the qkv
# weight gradient / every parameter gradient off the side stream (allocator stats in `memory`).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${DIAG_OUT:-b384diag}
mkdir -p $O
run() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 --cpu-baseline 0 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('memory'), d['library_fallbacks'])"
}
run tree ${TREE_ARGS:-}
run noqkv --no-roofline --host-opt wgrad_stream_qkv=0
run noside --no-roofline --host-opt wgrad_stream=0
