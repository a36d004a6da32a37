# stage microbench of W-MSA kernels for library variants: KLV="a b" (abl/<v>.so), BW_ARGS
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in $KLV; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 300 python tools/bench_wmsa.py ${BW_ARGS:---only bwd --kl 1} || exit 1
done
