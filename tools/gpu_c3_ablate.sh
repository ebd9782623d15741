# c3 k_resid phase ablation (FLACMI_DEBUG_STOP=k truncates k_resid after phase k; timing only)
# Usage: bash tools/gpu_c3_ablate.sh <tag> [extra env assignments for every run]
set -o pipefail
TAG=${1:-c3abl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for k in ${STOPS:-1 2 0}; do
  env FLACMI_DEBUG_STOP=$k $2 timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 0 --no-frames --no-parity --e2e-units 0 > $OUT/stop$k.json 2> $OUT/stop$k.err || { tail -20 $OUT/stop$k.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/stop$k.json'));print('stop $k', d['kernels']['k_resid_ms'])"
done
