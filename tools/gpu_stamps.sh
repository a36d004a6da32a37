set -o pipefail
cd $GRAFT_REPO_ROOT
HVK_LIB_PATH=$PWD/abl/stamp.so timeout -k 10 300 python tools/bench_wmsa.py --only bwd --kl 1 --stamps --iters 5 || exit 1
