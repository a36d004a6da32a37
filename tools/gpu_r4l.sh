# Round 4: q pre-scaled by the logit scale in the qkv epilogue (the W-MSA forward then takes q, k as
# they are), patch-embedding weight gradient on the dW kernel.  Parity suites, interleaved
# end-to-end A/B of HVK_QK_EPILOGUE 0/1, W-MSA microbench raw vs normed.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_qknorm.py tests/test_gpu_ddp.py tests/test_gpu_wmsa.py tests/test_gpu_weight_grad.py tests/test_gpu_model.py tests/test_gpu_steps.py tests/test_gpu_graph.py tests/test_gpu_head.py tests/test_gpu_linear.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; rb=d.get('roofline_bwd') or {}; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('avg_launch_us'), [round(s.get('frac',0),3) for s in r.get('stages',[])], 'bwd', rb.get('frac'), [s.get('avg_launch_us') for s in rb.get('stages') or []])"; }
for r in 1 2 3; do
  for e in 0 1; do
    HVK_QK_EPILOGUE=$e timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 20 > $O/epi_${e}_$r.json 2> $O/epi_${e}_$r.err || { tail -20 $O/epi_${e}_$r.err; exit 1; }
    row $O/epi_${e}_$r.json "epi=$e run=$r"
  done
done
timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 > $O/wmsa_raw.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --normed > $O/wmsa_normed.txt 2>&1 || exit 1
grep -v amdgpu $O/wmsa_raw.txt $O/wmsa_normed.txt
