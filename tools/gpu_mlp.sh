# fused-MLP tests, then the default bench line with the fused stage-0 MLP forward off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mlp
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp/tests.log 2>&1 || { tail -30 gpurun_out/mlp/tests.log; exit 1; }
tail -1 gpurun_out/mlp/tests.log
AB_VAR=HVK_MLP_FUSED AB_A=0 AB_B=1 bash tools/gpu_ab.sh
