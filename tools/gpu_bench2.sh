# default bench line (full JSON), then A/B of library variants, then the Swin-B configs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b2
timeout -k 10 300 python bench.py > gpurun_out/b2/default.json 2> gpurun_out/b2/default.err || { tail -20 gpurun_out/b2/default.err; exit 1; }
cat gpurun_out/b2/default.json
if [ -n "$AB_LIBS" ]; then AB_LIBS="$AB_LIBS" bash tools/gpu_ab_lib.sh || exit 1; fi
if [ -n "$SWINB" ]; then
  timeout -k 10 400 python bench.py --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 > gpurun_out/b2/b224.json 2> gpurun_out/b2/b224.err || { tail -20 gpurun_out/b2/b224.err; exit 1; }
  cat gpurun_out/b2/b224.json
  timeout -k 10 600 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 > gpurun_out/b2/b384.json 2> gpurun_out/b2/b384.err || { tail -20 gpurun_out/b2/b384.err; exit 1; }
  cat gpurun_out/b2/b384.json
fi
