# k_lpc_2p (FLACMI_LPC_2PASS=1): the 24-bit/L=32 parity tests under it, then c3 A/B.
set -o pipefail
TAG=${1:-r04f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
FLACMI_LPC_2PASS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3 or 24bit or int8 or golden or production or L32 or bucket or edge" > $OUT/pytest_2p.log 2>&1
rc=$?; echo "pytest (FLACMI_LPC_2PASS=1) rc=$rc $(tail -1 $OUT/pytest_2p.log)"
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $OUT/pytest_2p.log | head -60; exit 1; }
B="--steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0"
for v in 0 1 0 1; do
  FLACMI_LPC_2PASS=$v timeout -k 10 200 python bench.py --config c3 $B > $OUT/c3_2p_$v.json 2> $OUT/c3_2p_$v.err || { tail -20 $OUT/c3_2p_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c3_2p_$v.json'));k=d['kernels'];print('c3 LPC_2PASS=$v', '%.3e'%d['value'], 'lpc %.2f resid %.2f call %.2f'%(k['k_lpc_ms'],k['k_resid_ms'],k['call_ms']), (d.get('parity') or {}).get('mismatches'))"
done
