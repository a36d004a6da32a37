# Round 4: q / k normalisation in the qkv GEMM epilogue.  Its parity tests and the W-MSA /
# GEMM / model suites, then an interleaved end-to-end A/B (HVK_QK_EPILOGUE 0 / 1, 3 pairs), then the
# LayerNorm row-prefetch A/B (abl/lnold.so vs abl/lnnew.so, tools/build_variant.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qknorm.py tests/test_gpu_head.py tests/test_gpu_wmsa.py tests/test_gpu_linear.py tests/test_gpu_model.py tests/test_gpu_steps.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for e in 0 1; do
    HVK_QK_EPILOGUE=$e timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 20 > $O/ab_${e}_$r.json 2> $O/ab_${e}_$r.err || { tail -20 $O/ab_${e}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/ab_${e}_$r.json')); r=d['roofline']; print('epi=$e run=$r', d['value'], d['ms_per_step'], r['frac'], r.get('avg_launch_us'), [round(s.get('frac',0),3) for s in r.get('stages',[])], 'bwd', (d.get('roofline_bwd') or {}).get('frac'), [s.get('avg_launch_us') for s in (d.get('roofline_bwd') or {}).get('stages') or []])"
  done
done
AB_LIBS="lnold lnnew" bash tools/gpu_ab_lib.sh
