# A/B of library builds (abl/<name>.so, tools/build_variant.sh) on the default bench line,
# interleaved on one box:  AB_LIBS="base new" [BENCH_ARGS=...] bash tools/gpu_ab_lib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for v in $AB_LIBS; do
    HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 300 python bench.py --cpu-baseline 0 $BENCH_ARGS > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
    echo "$v $(python3 -c "
import json; d=json.load(open('gpurun_out/ab/b.json')); r=d.get('roofline') or {}; rb=d.get('roofline_bwd') or {}
print(d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), rb.get('frac'), rb.get('avg_launch_us'))")"
  done
done
