# GPU suite, then a c3 (and c2) A/B on one box: this build vs flac-py_amd/libflacmi_r04base.so.
# Usage: bash tools/gpu_r04j.sh <tag>
set -o pipefail
TAG=${1:-r04j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
BASE=$PWD/flac-py_amd/libflacmi_r04base.so
for cfg in ${CFGS:-c3 c2}; do
for v in new base new base; do
  if [ $v = base ]; then export FLACMI_LIB=$BASE; else unset FLACMI_LIB; fi
  timeout -k 10 200 python bench.py --config $cfg $B > $OUT/${cfg}_$v.json 2> $OUT/${cfg}_$v.err || { tail -20 $OUT/${cfg}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${cfg}_$v.json'));k=d['kernels'];print('$cfg $v', '%.4e'%d['value'], 'lpc %.3f resid %.3f call %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']), (d.get('parity') or {}).get('mismatches'))"
done
done
unset FLACMI_LIB
