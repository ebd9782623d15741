# A/B of library builds on one box: bash tools/gpu_libab.sh <tag> "<lib names>" [configs...]
# lib name "default" = flac-py_amd/libflacmi.so, otherwise flac-py_amd/libflacmi_<name>.so
set -o pipefail
TAG=${1:-ab}; LIBS=${2:-default}; shift 2
CFGS=${*:-c2 c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in $CFGS; do
  for v in $LIBS; do
    if [ "$v" = default ]; then L=$PWD/flac-py_amd/libflacmi.so; else L=$PWD/flac-py_amd/libflacmi_$v.so; fi
    FLACMI_LIB=$L timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-frames --steps 10 --warmup 2 $BENCH_ARGS > $OUT/$c.$v.json 2> $OUT/$c.$v.err || { tail -5 $OUT/$c.$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$c.$v.json'));k=d['kernels'];print('$c $v', '%.3e'%d['value'], 'lpc %.2f resid %.2f frac %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],d['roofline']['frac']), (d.get('parity') or {}).get('mismatches'))"
  done
done
