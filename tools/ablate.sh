# k_resid phase ablation: bench timing with the kernel truncated after each phase
# (FLACMI_DEBUG_STOP=k; timing only, outputs invalid).  Stops: k_resid_stream 1 staging, 2
# candidate sums, 3 choice, 4 chosen residual; k_resid / k_resid_sb (c3) also 5 Rice
# parameters, 6 row transform, 7 data bits; 0 = the whole kernel.
# Usage: [STOPS="1 2 4 5 6 7 0"] bash tools/ablate.sh <tag> [bench args, e.g. --config c3]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$OLDPWD}
TAG=${1:-abl}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for k in ${STOPS:-1 2 3 4 0}; do
  FLACMI_DEBUG_STOP=$k timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 "$@" > $OUT/stop$k.json 2> $OUT/stop$k.err || { tail $OUT/stop$k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/stop$k.json')); print('stop=$k', 'k_resid_ms %.3f' % d['kernels']['k_resid_ms'], 'k_lpc_ms %.3f' % d['kernels']['k_lpc_ms'])"
done
