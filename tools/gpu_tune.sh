set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
timeout -k 10 300 python tools/bench_gemm.py --iters 10 --only "s2|s3" > gpurun_out/tune/base.txt 2>&1 || exit 1
timeout -k 10 600 python tools/bench_gemm.py --iters 10 --only "s2|s3" --tunable gpurun_out/tune/tunable.csv > gpurun_out/tune/tuned.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/tune/base.txt; grep -v amdgpu gpurun_out/tune/tuned.txt
