# SwinV2-B skinny GEMMs: linear tests, then configs 4/5 bench A/B (HVK_SKINNY_B=0 / 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_swinb.py > gpurun_out/skb_tests.log 2>&1; rc=$?
tail -2 gpurun_out/skb_tests.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/skb_tests.log | head -30; exit $rc; }
for sk in 0 1; do
  HVK_SKINNY_B=$sk timeout -k 10 400 python bench.py --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/skb_b224_$sk.json 2> gpurun_out/skb.err || { tail -20 gpurun_out/skb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/skb_b224_$sk.json')); print('b224 skinny=$sk', d['value'], d['ms_per_step'], d['mfma']['gemm'])"
done
for sk in 0 1; do
  HVK_SKINNY_B=$sk timeout -k 10 600 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/skb_b384_$sk.json 2> gpurun_out/skb.err || { tail -20 gpurun_out/skb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/skb_b384_$sk.json')); print('b384 skinny=$sk', d['value'], d['ms_per_step'], d['mfma']['gemm'])"
done
