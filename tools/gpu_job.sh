# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
STOPS="1 2 4 5 6 7 0" KPAT=k_resid_sb bash tools/pmc_stops.sh r6i insts --config c3 --e2e-units 0 > /dev/null && STOPS="1 2 4 5 6 7 0" bash tools/ablate.sh r6i/abl --config c3
for k in 1 2 4 5 6 7 0; do python3 tools/pmc_summary.py gpurun_out/r6i/s$k | grep -A9 k_resid_sb | grep "INSTS_VALU\|INSTS_SALU" | tr '\n' ' '; echo " stop $k"; done
