# win-form W-MSA forward: full vs memory-only vs math-only builds (abl/*.so), per stage, then
# SQ / LDS PMC passes of the full kernel at stage 0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/winprobe
for rep in 1 2; do for v in base winmem winmath; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 120 python tools/bench_wmsa.py --only fwd || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/winprobe/micro.txt
STAGE=0 bash tools/pmc_wmsa.sh fwd winfwd sq,lds || exit 1
python3 tools/pmc_report.py gpurun_out/pmc_winfwd 2>&1 | tee gpurun_out/winprobe/pmc.txt
