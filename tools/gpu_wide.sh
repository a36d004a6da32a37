# The 208 x 384 whole-row GEMM tile: its GPU tests, the per-shape interleaved A/B against the
# 128-row tiles (tools/bench_wide.py), then the default bench line with / without it (interleaved).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${W_OUT:-wide}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_wide.py > $O/bench_wide.txt 2>&1 || { tail -20 $O/bench_wide.txt; exit 1; }
cat $O/bench_wide.txt
if [ -z "$NO_E2E" ]; then
for rep in 1 2; do
  for arm in 0 1; do
    timeout -k 10 300 python bench.py --cpu-baseline 0 --opt gemm_wide=$arm > $O/b$arm.json 2> $O/b$arm.err || { tail -20 $O/b$arm.err; exit 1; }
    echo "gemm_wide=$arm $(python3 -c "import json; d=json.load(open('$O/b$arm.json')); print(d['value'], d['ms_per_step'], d['mfma']['binding'])")"
  done
done
fi
