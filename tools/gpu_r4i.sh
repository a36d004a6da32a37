# Round 4: after the rn-gradient fill fix and the consolidated rn stores: the affected parity
# suites, then interleaved end-to-end A/B of HVK_QK_EPILOGUE 0/1 and HVK_HEAD_GEMM 0/1.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qknorm.py tests/test_gpu_head.py tests/test_gpu_wmsa.py tests/test_gpu_linear.py tests/test_gpu_model.py tests/test_gpu_steps.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; rb=d.get('roofline_bwd') or {}; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('avg_launch_us'), [round(s.get('frac',0),3) for s in r.get('stages',[])], 'bwd', rb.get('frac'), (d.get('mfma') or {}).get('gemm',{}).get('frac') if isinstance((d.get('mfma') or {}).get('gemm'),dict) else None)"; }
for r in 1 2 3; do
  for e in 0 1; do
    HVK_QK_EPILOGUE=$e timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 20 > $O/epi_${e}_$r.json 2> $O/epi_${e}_$r.err || { tail -20 $O/epi_${e}_$r.err; exit 1; }
    row $O/epi_${e}_$r.json "epi=$e run=$r"
  done
done
for r in 1 2; do
  for e in 0 1; do
    HVK_HEAD_GEMM=$e timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 20 > $O/head_${e}_$r.json 2> $O/head_${e}_$r.err || { tail -20 $O/head_${e}_$r.err; exit 1; }
    row $O/head_${e}_$r.json "head=$e run=$r"
  done
done
