# PMC passes (sq, lds) for the two W-MSA backward kernels at stage 0
set -o pipefail
cd $GRAFT_REPO_ROOT
KL=1 bash tools/pmc_wmsa.sh bwd bwd_kl sq,lds || exit 1
KL=0 bash tools/pmc_wmsa.sh bwd bwd_old sq,lds || exit 1
python3 tools/pmc_report.py gpurun_out/pmc_bwd_kl wmsa_bwd > gpurun_out/pmc_kl.txt
python3 tools/pmc_report.py gpurun_out/pmc_bwd_old wmsa_bwd >> gpurun_out/pmc_kl.txt
cat gpurun_out/pmc_kl.txt
