# Round 4: LayerNorm lane-contiguous layout -- its GPU tests, then interleaved in-step A/B against
# the previous build (abl/base.so = HEAD, abl/ln.so = working tree); then the DDP overlap trace
# (one-rank RCCL, buckets forced, rocprofv3 kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "layernorm or norm_pool or swinv2t or block" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -1 gpurun_out/r4b/tests.log
AB_LIBS="base ln" bash tools/gpu_ab_lib.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4b/ddp -o ddp -- python3 $R/tools/ddp_trace.py > $R/gpurun_out/r4b/ddp.log 2>&1 || { tail -20 $R/gpurun_out/r4b/ddp.log; exit 1; }
cd $R && python3 tools/ddp_overlap.py gpurun_out/r4b/ddp > gpurun_out/r4b/ddp_overlap.txt 2>&1; head -60 gpurun_out/r4b/ddp_overlap.txt
