# Measurement pass (no tests): c3 k_resid split (tools/gpu_c3_split.sh, SQ passes included),
# then k_resid_stream instruction counts per phase stop for c2 (tools/pmc_phase_valu.sh).
# Usage: bash tools/gpu_measure.sh <tag>
set -o pipefail
TAG=${1:-meas}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_c3_split.sh $TAG/c3 || exit 1
CFGS=c2 bash tools/pmc_phase_valu.sh $TAG/phase || exit 1
