# All -m gpu tests, the default bench line and the two SwinV2-B bench lines (configs 4 and 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/all
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/all/tests.log 2>&1 || { tail -40 gpurun_out/all/tests.log; exit 1; }
tail -2 gpurun_out/all/tests.log
timeout -k 10 400 python bench.py > gpurun_out/all/default.json 2> gpurun_out/all/default.err || { tail -20 gpurun_out/all/default.err; exit 1; }
cat gpurun_out/all/default.json
timeout -k 10 400 python bench.py --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 > gpurun_out/all/b224.json 2> gpurun_out/all/b224.err || { tail -20 gpurun_out/all/b224.err; exit 1; }
cat gpurun_out/all/b224.json
timeout -k 10 600 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 > gpurun_out/all/b384.json 2> gpurun_out/all/b384.err || { tail -20 gpurun_out/all/b384.err; exit 1; }
cat gpurun_out/all/b384.json
