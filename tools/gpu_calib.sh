# FETCH_SIZE / WRITE_SIZE calibration passes over tools/probe/fetch_calib (separate runs)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/calib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o run --output-format csv -- $R/tools/probe/fetch_calib > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
cd $R && python3 tools/probe/fetch_calib.py $O/FETCH_SIZE $O/WRITE_SIZE | tee $O/calib.txt
