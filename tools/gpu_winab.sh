# win forward A/B: library variants (abl/*.so) and env switches, interleaved in-step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/winab
for rep in 1 2; do for v in $VARIANTS; do
  lib=${v%%:*}; env=${v#*:}; [ "$env" = "$v" ] && env="X=1"
  env $env HVK_LIB_PATH=$PWD/abl/$lib.so timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/winab/b.json 2> gpurun_out/winab/b.err || { tail -20 gpurun_out/winab/b.err; exit 1; }
  echo "$v $(python3 -c "
import json; d=json.load(open('gpurun_out/winab/b.json')); r=d.get('roofline') or {}; rb=d.get('roofline_bwd') or {}
print(d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), rb.get('frac'))")"
done; done 2>&1 | tee gpurun_out/winab/ab.txt
