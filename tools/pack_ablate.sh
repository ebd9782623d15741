# k_pack32 ablation: frame-writer leg timing with parts of the kernel switched off
# (FLACMI_PACK_ABLATE bits: 1 no CRC shift, 2 no residual codes, 4 no CRC fold, 8 no per-value
# bit counts, 16 no body stores, 32 no residual loads; outputs invalid, timing only).
# Usage: [MODES="0 1 2 3"] bash tools/pack_ablate.sh <tag> [bench args]
set -o pipefail
TAG=${1:-pab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for k in ${MODES:-0 1 2 3}; do
  FLACMI_PACK_ABLATE=$k timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --e2e-units 0 "$@" > $OUT/pab_$k.json 2>$OUT/pab_$k.err || { tail $OUT/pab_$k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pab_$k.json')); print('ablate=$k', 'frame_ms %.3f' % d['frame_writer']['ms_per_call'])"
done
