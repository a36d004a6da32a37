# weight-gradient kernel: parity tests (every tile variant), then the per-shape timing table
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dw
rm -f gpurun_out/dw/bench.txt
for v in ${DW_VARIANTS:-4 5 6 7}; do
  HVK_DW_TILE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_weight_grad.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dw/tests$v.log 2>&1 || { tail -40 gpurun_out/dw/tests$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/dw/tests$v.log)"
done
for v in ${DW_VARIANTS:-4 5 6 7}; do
  echo "== HVK_DW_TILE=$v" >> gpurun_out/dw/bench.txt
  HVK_DW_TILE=$v timeout -k 10 300 python tools/bench_dw.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/dw/bench.txt || { cat gpurun_out/dw/bench.txt; exit 1; }
done
cat gpurun_out/dw/bench.txt
