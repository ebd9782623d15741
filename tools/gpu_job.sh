# scratch job file for one gpurun call (overwritten per call; the reusable steps are the
# other tools/gpu_*.sh, pmc_*.sh and profile.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--e2e-units 0 --no-parity"
bash tools/gpu_libab.sh r5q/a "default ntst ntld ntboth" c2 c5 && bash tools/gpu_libab.sh r5q/b "ntboth ntld ntst default" c5 c2
