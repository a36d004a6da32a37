# rocprof kernel stats of a short default bench run (+ PROF_ARGS) -> gpurun_out/prof/summary.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PROF_OUT:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 $PROF_ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R && python3 tools/kernel_summary.py $(find $O/p -name "*kernel_trace.csv" | head -1) --anchor hxe_fwd --skip 3 --top 45 > $O/summary.txt && cat $O/summary.txt
