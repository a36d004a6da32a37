# Round 4: where the q / k epilogue's end-to-end cost goes: rocprofv3 kernel stats of the default
# bench with HVK_QK_EPILOGUE=0 and =1 (per-kernel comparison), then the W-MSA counters and probes.
set -o pipefail
cd $GRAFT_REPO_ROOT
HVK_QK_EPILOGUE=0 PROF_OUT=prof_epi0 bash tools/gpu_prof.sh > /dev/null || exit 1
HVK_QK_EPILOGUE=1 PROF_OUT=prof_epi1 bash tools/gpu_prof.sh > /dev/null || exit 1
head -40 gpurun_out/prof_epi0/summary.txt
head -40 gpurun_out/prof_epi1/summary.txt
bash tools/gpu_r4g.sh
