# A/B of the residual kernels on one box: default, persistent stream, old k_resid.
# Usage: bash tools/gpu_cmp.sh <tag> [configs...]
set -o pipefail
TAG=${1:-cmp}; shift
CFGS=${*:-c2 c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in $CFGS; do
  for v in default old; do
    case $v in default) E="";; persist) E="FLACMI_STREAM_PERSIST=1";; old) E="FLACMI_NO_STREAM=1";; esac
    env $E timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-frames --steps 10 --warmup 2 > $OUT/$c.$v.json 2> $OUT/$c.$v.err || { tail -5 $OUT/$c.$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$c.$v.json'));k=d['kernels'];print('$c $v', '%.3e'%d['value'], 'lpc %.2f resid %.2f frac %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],d['roofline']['frac']), d['parity']['mismatches'])"
  done
done
