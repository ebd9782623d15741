# GPU suite (persistent kVarMf8 default, its copies issued in inline asm), c3 A/B vs
# FLACMI_MF8_PERSIST=0 (the k_lpc_2p A/B of that run: kernel since removed).
set -o pipefail
TAG=${1:-r04g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
for v in 1 0 1 0; do
  FLACMI_MF8_PERSIST=$v timeout -k 10 200 python bench.py --config c3 $B > $OUT/c3_p$v.json 2> $OUT/c3_p$v.err || { tail -20 $OUT/c3_p$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_p$v.json'));k=d['kernels'];print('c3 MF8_PERSIST=$v', '%.3e'%d['value'], 'lpc %.2f resid %.2f call %.2f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']), (d.get('parity') or {}).get('mismatches'))"
done
