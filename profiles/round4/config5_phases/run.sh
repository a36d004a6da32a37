# Round 4: where the config-5 large-window backward spends its time: the w24 / w12 backward per
# stage with phase 1 skipped (lprobe3), phase 2 skipped (lprobe4), no CPB bins (lprobe1) and the
# full kernel (lbase); timing-only builds (results wrong), tools/bench_wmsa.py --b384.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in lbase lprobe3 lprobe4 lprobe1 lbase; do
  timeout -k 10 300 python3 tools/bench_wmsa.py --b384 --iters 3 --lib abl/$v.so > gpurun_out/r4m_$v.txt 2>&1 || { tail gpurun_out/r4m_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu gpurun_out/r4m_$v.txt
done
