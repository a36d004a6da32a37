# One-window-per-workgroup W-MSA forward (wmsa_win.hip): parity tests, per-stage microbench,
# interleaved in-step bench A/B against the persistent ring form (HVK_WMSA_FWD_FORM=ring), and
# an SQ PMC pass of the win kernel at stage 0.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/winfwd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py -k "forward or scale100" > gpurun_out/winfwd/tests.log 2>&1; rc=$?
tail -3 gpurun_out/winfwd/tests.log; [ $rc -eq 0 ] || exit $rc
for f in ring win; do
  echo "== form=$f"
  HVK_WMSA_FWD_FORM=$f timeout -k 10 120 python tools/bench_wmsa.py --only fwd || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/winfwd/micro.txt
for rep in 1 2; do for f in ring win; do
  HVK_WMSA_FWD_FORM=$f timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/winfwd/b.json 2> gpurun_out/winfwd/b.err || { tail -20 gpurun_out/winfwd/b.err; exit 1; }
  echo "$f $(python3 -c "
import json; d=json.load(open('gpurun_out/winfwd/b.json')); r=d.get('roofline') or {}; rb=d.get('roofline_bwd') or {}
print(d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), rb.get('frac'))")"
done; done 2>&1 | tee gpurun_out/winfwd/ab.txt
if [ -n "$WIN_PMC" ]; then
  STAGE=0 bash tools/pmc_wmsa.sh fwd winfwd2 sq,lds || exit 1
  python3 tools/pmc_report.py gpurun_out/pmc_winfwd2 wmsa 2>&1 | tee gpurun_out/winfwd/pmc.txt
fi
