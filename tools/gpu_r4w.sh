# Round 4: LayerNorm forward at C = 96 with the bf16 rows (192 B, not whole lines) moved through a
# per-wave LDS block by whole-line accesses (lnbfl) against direct 8-B-per-lane accesses (lnbase).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4w
HVK_LIB_PATH=$PWD/abl/lnbfl.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_steps.py > gpurun_out/r4w/tests.txt 2>&1 || { tail -30 gpurun_out/r4w/tests.txt; exit 1; }
tail -1 gpurun_out/r4w/tests.txt
for v in lnbase lnbfl lnbase lnbfl; do
  echo "== $v"; timeout -k 10 300 python3 tools/bench_ln.py --iters 20 --lib abl/$v.so 2>&1 | grep stage || exit 1
done
AB_LIBS="lnbase lnbfl" timeout -k 10 900 bash tools/gpu_ab_lib.sh
