# A/B of two bench argument sets on the default bench line, interleaved on one box (options are
# explicit bench flags: --host-opt NAME=VALUE for hvamd.options, --opt NAME=VALUE for libhvk):
#   AB_A="--host-opt mlp_fused=0" AB_B="" bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then args="$AB_A"; else args="$AB_B"; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline $args > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
    echo "$arm [$args] $(python3 -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print(d['value'], d['ms_per_step'])")"
  done
done
