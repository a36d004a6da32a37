# A/B of one environment switch on the default bench line, interleaved on one box:
#   AB_VAR=HVK_PREPARE_WEIGHTS AB_A=0 AB_B=1 bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in $AB_A $AB_B; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
    echo "$AB_VAR=$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print(d['value'], d['ms_per_step'])")"
  done
done
