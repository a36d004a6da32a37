# win forward: W-MSA tests, then interleaved in-step A/B of library variants (abl/*.so) and the
# ring form, per-stage microbench of each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/winfwd
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py > gpurun_out/winfwd/tests.log 2>&1; rc=$?
tail -3 gpurun_out/winfwd/tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARS:-noprio prio}; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 120 python tools/bench_wmsa.py --only fwd || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/winfwd/micro.txt
for rep in 1 2; do for v in ${VARS:-noprio prio} ring; do
  if [ $v = ring ]; then E="HVK_WMSA_FWD_FORM=ring"; L=$PWD/abl/prio.so; else E="X=1"; L=$PWD/abl/$v.so; fi
  env $E HVK_LIB_PATH=$L timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/winfwd/b.json 2> gpurun_out/winfwd/b.err || { tail -20 gpurun_out/winfwd/b.err; exit 1; }
  echo "$v $(python3 -c "
import json; d=json.load(open('gpurun_out/winfwd/b.json')); r=d.get('roofline') or {}; rb=d.get('roofline_bwd') or {}
print(d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), rb.get('frac'))")"
done; done 2>&1 | tee gpurun_out/winfwd/ab.txt
