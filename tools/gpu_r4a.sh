# Round-4 first call: the quick checkpoint (tests, smoke, bench) on the cleaned-up library, then
# the W-MSA forward memory-shape probe (tools/probe/wmsa_mem) at stage 0 and the LayerNorm
# access-shape probe (tools/probe/ln_probe), both built here.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
timeout -k 10 120 ./tools/probe/ln_probe > gpurun_out/probe/ln_probe.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/probe/wmsa_mem 3 > gpurun_out/probe/wmsa_mem_stage0.txt 2>&1 || exit 1
bash tools/gpu_check.sh || exit 1
