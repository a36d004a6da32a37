# W-MSA forward per stage: default build vs DMA without the nontemporal hint (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fa
for r in 1 2 3; do
  for v in base aux0; do
    timeout -k 10 120 python tools/bench_wmsa.py --lib abl/$v.so --only fwd --kl 0 --iters 30 > gpurun_out/fa/${v}_$r.txt 2>&1 || { tail -5 gpurun_out/fa/${v}_$r.txt; exit 1; }
    echo "== $v $r"; grep -v amdgpu.ids gpurun_out/fa/${v}_$r.txt
  done
done
