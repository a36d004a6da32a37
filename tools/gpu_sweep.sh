set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/copy_calib.py > gpurun_out/copy.log 2>&1 || exit 1
for w in 512 768 2048 4096; do
  HVK_WMSA_FWD_WGS=$w timeout -k 10 120 python tools/bench_wmsa.py --iters 10 > gpurun_out/bw_wgs$w.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 15 --warmup 3 --cpu-baseline 0 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1
