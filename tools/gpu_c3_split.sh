# c3 k_resid time split: bench line, FLACMI_DEBUG_STOP ablations (1 staging, 2 candidate sums,
# 3 choice, 4 chosen residual, 5..7 Rice steps; 13 fixed sums only, 14 first LPC quarter
# without tier tests, 15 every LPC tile without tier tests -- 13..15 then run the rest of
# the kernel), then the SQ counter passes of tools/pmc_c3.sh.  Timing only for the stops.
# Usage: bash tools/gpu_c3_split.sh <tag>
set -o pipefail
TAG=${1:-c3split}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for k in ${STOPS:-0 1 2 13 14 15 3 4 5 6 7}; do
  FLACMI_DEBUG_STOP=$k timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-frames --no-parity --e2e-units 0 > $OUT/stop$k.json 2> $OUT/stop$k.err || { tail -20 $OUT/stop$k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/stop$k.json'));print('stop $k', round(d['kernels']['k_resid_ms'],2), round(d['kernels']['k_lpc_ms'],2))"
done
[ -n "$NOPMC" ] || bash tools/pmc_c3.sh $TAG/pmc
