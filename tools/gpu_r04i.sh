# GPU suite, then a c2 A/B on one box: this build vs flac-py_amd/libflacmi_r04base.so (the
# previous HEAD's library).  Usage: bash tools/gpu_r04i.sh <tag>
set -o pipefail
TAG=${1:-r04i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
B="--steps 10 --warmup 3 --cpu-seconds 0 --no-frames --e2e-units 0"
BASE=$PWD/flac-py_amd/libflacmi_r04base.so
for v in new base new base; do
  if [ $v = base ]; then export FLACMI_LIB=$BASE; else unset FLACMI_LIB; fi
  timeout -k 10 200 python bench.py --config c2 $B > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -20 $OUT/c2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_$v.json'));k=d['kernels'];print('c2 $v', '%.4e'%d['value'], 'lpc %.3f resid %.3f call %.3f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']), (d.get('parity') or {}).get('mismatches'))"
done
unset FLACMI_LIB
