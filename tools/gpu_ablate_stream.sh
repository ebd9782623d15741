# Phase ablation of k_resid_stream (FLACMI_DEBUG_STOP=k stops each unit after phase k).
set -o pipefail
OUT=gpurun_out/${1:-abl}; shift
CFGS=${*:-c2 c5}
mkdir -p $OUT
for c in $CFGS; do
  for k in ${STOPS:-1 2 3 4 0}; do
    FLACMI_DEBUG_STOP=$k timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-frames --no-parity --steps 8 --warmup 2 > $OUT/$c.$k.json 2> $OUT/$c.$k.err || { tail -5 $OUT/$c.$k.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$c.$k.json'));k=d['kernels'];print('$c stop=$k resid %.2f ms'%k['k_resid_ms'])"
  done
done
