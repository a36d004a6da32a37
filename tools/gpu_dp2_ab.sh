# DDP checks for the parameter-gradient side stream: the DDP / side-stream GPU tests, then the dp2
# gloo rehearsal (two ranks sharing GPU 0) with the side stream off / on, REPS interleaved pairs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-dp2ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_wgrad_stream.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in $(seq 1 ${REPS:-2}); do
  for o in 0 1; do
    timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --cpu-baseline 0 --no-roofline --host-opt wgrad_stream=$o > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    echo "wgrad_stream=$o $(grep '^{' $O/b.json | python3 -c 'import json, sys; d = json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"])')"
  done
done
