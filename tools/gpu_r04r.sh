# c3 k_resid split with the sign-correlation bound (ablation stops, no counters).
set -o pipefail
TAG=${1:-r04r}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NOPMC=1 STOPS="0 1 2 13 3 4 5 7" bash tools/gpu_c3_split.sh $TAG/c3
