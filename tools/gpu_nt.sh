set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/stream > gpurun_out/stream.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_wmsa.py -q -x > gpurun_out/t.log 2>&1 || exit 1
for w in 1024 3072 6144; do
  HVK_WMSA_FWD_WGS=$w timeout -k 10 120 python tools/bench_wmsa.py --iters 10 > gpurun_out/bw_nt_$w.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/bench_wmsa.py --iters 10 --lib tools/probe/libhvk_nont.so > gpurun_out/bw_nont.log 2>&1 || exit 1
