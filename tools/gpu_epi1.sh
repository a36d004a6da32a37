# EPI 1 two-image staging: the tile GEMM tests, then hvk_gemm_gelu_fwd per shape for the tree and
# abl/epi1old.so (-DHVK_EPI1_TWO=0), interleaved REPS rounds, then the default bench A/B (lib swap).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${E_OUT:-epi1}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_merge.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq 1 ${REPS:-2}); do
  echo "== tree $r"; timeout -k 10 200 python tools/bench_epi1.py || exit 1
  echo "== old $r"; timeout -k 10 200 python tools/bench_epi1.py --lib abl/epi1old.so || exit 1
done
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "tree bench $(python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'])")"
  HVK_LIB_PATH=$PWD/abl/epi1old.so timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "old bench $(python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'])")"
done
