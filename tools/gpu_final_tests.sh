# End-of-session check of the committed tree: every -m gpu test (incl. the bounds-checked build) and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/endcheck
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/endcheck/tests.log 2>&1 || { tail -40 gpurun_out/endcheck/tests.log; exit 1; }
tail -2 gpurun_out/endcheck/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/endcheck/smoke.log 2>&1 || { tail -20 gpurun_out/endcheck/smoke.log; exit 1; }
tail -1 gpurun_out/endcheck/smoke.log
