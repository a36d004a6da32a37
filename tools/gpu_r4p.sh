# Round 4: stage-1 fc1 + GELU on the tiled EPI 1 kernel (now with the LDS-staged epilogue) instead
# of the skinny kernel, end-to-end A/B on one box; then the staged build's GELU-epilogue tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py -k "gelu" > gpurun_out/r4p_tests.txt 2>&1 || { tail -30 gpurun_out/r4p_tests.txt; exit 1; }
tail -1 gpurun_out/r4p_tests.txt
AB_VAR=HVK_S1_GELU_TILE AB_A=0 AB_B=1 timeout -k 10 900 bash tools/gpu_ab.sh
AB_VAR=HVK_S1_GELU_TILE AB_A=0 AB_B=1 timeout -k 10 900 bash tools/gpu_ab.sh
