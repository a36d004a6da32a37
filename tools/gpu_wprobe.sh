# W-MSA forward: full kernel vs its memory-only (probe1) and math-only (probe2) builds, per stage
set -o pipefail
cd $GRAFT_REPO_ROOT
for l in new probe1 probe2 ${EXTRA_LIBS}; do
  echo "== $l"
  HVK_LIB_PATH=$PWD/abl/$l.so timeout -k 10 120 python tools/bench_wmsa.py --only fwd --iters 20 || exit 1
done
