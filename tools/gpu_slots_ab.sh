# w7 backward chunk-count A/B: per-stage backward timings of abl/<lib>.so for each lib in LIBS
# (2 interleaved rounds), then the bench line A/B (tools/gpu_ab_lib.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slots
for r in 1 2; do
  for v in $LIBS; do
    echo "== $v (rep $r)"
    timeout -k 10 300 python tools/bench_wmsa.py --normed --only bwd --lib abl/$v.so > gpurun_out/slots/${v}_$r.txt 2>&1 || { cat gpurun_out/slots/${v}_$r.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/slots/${v}_$r.txt
  done
done
AB_LIBS="$LIBS" bash tools/gpu_ab_lib.sh
