# W-MSA HBM traffic: FETCH_SIZE and WRITE_SIZE passes over a short bench run -> bench_traffic.json
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/traffic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --no-roofline > $O/$c.log 2>&1 || exit 1
done
python3 $R/tools/traffic.py $O/FETCH_SIZE $O/WRITE_SIZE $O/bench_traffic.json
