# Round 4 against the round-3 end tree (commit c5db82f, extracted to r3tree/ with its own libhvk),
# interleaved on one box: config 3 (default bench line) x3, config 4 x2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4z
line() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; rb=d.get('roofline_bwd') or {}
print(d['value'], d['ms_per_step'], r.get('frac'), rb.get('frac'))" $1; }
for rep in 1 2 3; do
  (cd r3tree && timeout -k 10 300 python bench.py --cpu-baseline 0 > ../gpurun_out/r4z/r3.json 2> ../gpurun_out/r4z/r3.err) || { tail -20 gpurun_out/r4z/r3.err; exit 1; }
  echo "round3 $(line gpurun_out/r4z/r3.json)"
  timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/r4z/r4.json 2> gpurun_out/r4z/r4.err || { tail -20 gpurun_out/r4z/r4.err; exit 1; }
  echo "round4 $(line gpurun_out/r4z/r4.json)"
done
for rep in 1 2; do
  (cd r3tree && timeout -k 10 400 python bench.py --cpu-baseline 0 --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 > ../gpurun_out/r4z/r3b.json 2> ../gpurun_out/r4z/r3b.err) || { tail -20 gpurun_out/r4z/r3b.err; exit 1; }
  echo "round3 b224 $(line gpurun_out/r4z/r3b.json)"
  timeout -k 10 400 python bench.py --cpu-baseline 0 --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 > gpurun_out/r4z/r4b.json 2> gpurun_out/r4z/r4b.err || { tail -20 gpurun_out/r4z/r4b.err; exit 1; }
  echo "round4 b224 $(line gpurun_out/r4z/r4b.json)"
done
