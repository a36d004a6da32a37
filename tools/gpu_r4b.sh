# Round 4: LayerNorm lane-contiguous layout (tests + interleaved in-step A/B against abl/base.so =
# the previous commit's kernels), the persistent row-range GEMM v2 (parity tests + per-shape A/B
# microbench against the tile kernel), then the DDP overlap trace (one-rank RCCL, buckets forced).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "layernorm or norm_pool or swinv2t or block" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -1 gpurun_out/r4b/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -k "xr" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/xr_test.log 2>&1 || { tail -30 gpurun_out/r4b/xr_test.log; exit 1; }
tail -1 gpurun_out/r4b/xr_test.log
timeout -k 10 300 python -u tools/bench_xr.py > gpurun_out/r4b/bench_xr.txt 2>&1 || { tail -30 gpurun_out/r4b/bench_xr.txt; exit 1; }
cat gpurun_out/r4b/bench_xr.txt
AB_LIBS="base ln" bash tools/gpu_ab_lib.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4b/ddp -o ddp -- python3 $R/tools/ddp_trace.py > $R/gpurun_out/r4b/ddp.log 2>&1 || { tail -20 $R/gpurun_out/r4b/ddp.log; exit 1; }
cd $R && python3 tools/ddp_overlap.py gpurun_out/r4b/ddp > gpurun_out/r4b/ddp_overlap.txt 2>&1; head -60 gpurun_out/r4b/ddp_overlap.txt
