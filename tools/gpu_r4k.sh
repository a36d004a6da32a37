# Round 4: LayerNorm at 12 channels per lane for C = 96 ... 768 (abl/lnnew.so) vs the 8 / 16
# layouts (abl/lnold.so): LN parity tests, per-stage LN microbench, end-to-end A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "layernorm" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in lnold lnnew; do
    timeout -k 10 200 python3 tools/bench_ln.py --lib abl/$v.so > $O/ln_$v.txt 2>&1 || { tail $O/ln_$v.txt; exit 1; }
    echo "== $v"; grep -v amdgpu $O/ln_$v.txt
  done
done
AB_LIBS="lnold lnnew" bash tools/gpu_ab_lib.sh
